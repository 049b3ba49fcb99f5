#!/usr/bin/env python3
"""comb-ntsc on the MI355X: the reference comb's frame stream (comb-ntsc.cxx
main :956-1125) with the 2D comb or the 3D comb without optical flow on the GPU.

    python ld-decode_amd/comb_ntsc.py [-d 2|3] [-F] [-c core] [-r range] [-i infile] > out.rgb

Reads 910x525 uint16 .tbc frames from stdin (or -i), writes 744x480 rgb48
frames to stdout, as `comb-ntsc` does with its defaults (dim 2, HQ colour LPF,
nr_y 1 IRE, 7.5 IRE setup, brightness 236).  -d 3 needs -F: the optical-flow 3D
path uses OpenCV's Farneback flow, which this build does not restate.  A short
final frame ends the stream like the reference's exit(0) (:1104,1114).  Other
reference options (-W -L -Q -a -R -8 -D -O -v -B -b -I -n -N -f -p -o -l -m -t
-k) are rejected rather than silently ignored.
"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

IN_X, IN_Y = 910, 525
FRAME_BYTES = IN_X * IN_Y * 2


def parse(argv=None):
    p = argparse.ArgumentParser(description='NTSC comb filter (.tbc -> rgb48)', add_help=True)
    p.add_argument('-d', dest='dim', type=int, default=2, help='comb dimension: 2 (default) or 3')
    p.add_argument('-F', dest='no_of', action='store_true', help='3D without optical flow')
    p.add_argument('-c', dest='core', type=float, default=-1.0, help='3D core (IRE, -F default 1.25)')
    p.add_argument('-r', dest='range', type=float, default=-1.0, help='3D range (IRE, -F default 5.5)')
    p.add_argument('-i', dest='infile', default=None, help='input file (default stdin)')
    p.add_argument('--device', type=int, default=0, help='HIP device')
    p.add_argument('--chunk', type=int, default=32, help='frames per GPU call')
    return p.parse_args(argv)


def read_frames(fh, n):
    """Up to n whole frames; a short read at the end stops the stream (:1102-1105)."""
    buf = fh.read(n * FRAME_BYTES)
    k = len(buf) // FRAME_BYTES
    return np.frombuffer(buf[:k * FRAME_BYTES], dtype=np.uint16).reshape(k, IN_Y, IN_X), k < n


def main(argv=None):
    args = parse(argv)
    if args.dim not in (2, 3):
        print('ERROR: -d must be 2 or 3 in this build', file=sys.stderr)
        return 1
    if args.dim == 3 and not args.no_of:
        print('ERROR: -d 3 with optical flow (OpenCV Farneback) is not available; use -d 3 -F', file=sys.stderr)
        return 1
    from ldgpu import native
    ctx = native.Context('NTSC', args.device, max_reads=1, max_frames=args.chunk)
    ctx.comb_reset()
    fin = open(args.infile, 'rb') if args.infile else sys.stdin.buffer
    out = sys.stdout.buffer
    while True:
        fr, last = read_frames(fin, args.chunk)
        if fr.shape[0]:
            rgb = ctx.comb_ntsc(fr) if args.dim == 2 else ctx.comb_ntsc3d(fr, args.core, args.range)
            out.write(rgb.tobytes())
        if last:
            break
    out.flush()
    return 0


if __name__ == '__main__':
    sys.exit(main())
