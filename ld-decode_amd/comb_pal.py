#!/usr/bin/env python3
"""comb-pal's frame stream on the MI355X (encode-pal:4: `cat x.tbc | ./comb-pal -d 2 -
| ffmpeg ... -pix_fmt rgb48 -s 974x576 -i /dev/stdin ...`), over the build-defined
PAL Y/C decoder (ldg_comb_pal; SURVEY §8 f row F2: the snapshot has no PAL comb for
lddecode's 1135x625 .tbc, so attic2/comb-pal.cxx's dim=2 path is adapted to it and
its parity is pinned only against oracle/combpal.cpp).

    python ld-decode_amd/comb_pal.py [-d 2] [-W] [-i infile] [-] > out.rgb

Reads 1135x625 uint16 frames from stdin (or -i) and writes 576-line rgb48 frames to
stdout, 974 wide as comb-pal writes them (columns 78..1051: its `in_x - 78` with
in_x = 1052, attic2/comb-pal.cxx:883-884) so encode-pal's ffmpeg -s 974x576 line
takes them unchanged; -W writes the decoder's whole 1057-column width instead
(columns 78..1134 of the 1135-sample line).  A short final frame ends the stream.
"""
import getopt
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

IN_X, IN_Y = 1135, 625
FRAME_BYTES = IN_X * IN_Y * 2
COMB_PAL_W = 974              # attic2/comb-pal.cxx:883 (1052 - 78)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    try:
        opts, _ = getopt.getopt(argv, 'Wd:i:', ['chunk=', 'device='])
    except getopt.GetoptError as e:
        print('comb_pal: %s' % e, file=sys.stderr)
        return 255
    wide, infile, chunk, device = False, None, 16, 0
    for k, v in opts:
        if k == '-W':
            wide = True
        elif k == '-d' and int(v) != 2:
            print('ERROR: this build decodes PAL with the 2D path only (-d 2)', file=sys.stderr)
            return 1
        elif k == '-i':
            infile = v
        elif k == '--chunk':
            chunk = int(v)
        elif k == '--device':
            device = int(v)
    from ldgpu import native
    ctx = native.Context('PAL', device, max_reads=1, max_frames=chunk)
    ctx.comb_reset()
    fin = open(infile, 'rb') if infile else sys.stdin.buffer
    out = sys.stdout.buffer
    while True:
        buf = fin.read(chunk * FRAME_BYTES)
        k = len(buf) // FRAME_BYTES
        if k:
            rgb = ctx.comb_pal(np.frombuffer(buf[:k * FRAME_BYTES], dtype=np.uint16).reshape(k, IN_Y, IN_X))
            out.write((rgb if wide else np.ascontiguousarray(rgb[:, :, :COMB_PAL_W])).tobytes())
        if k < chunk:
            break
    out.flush()
    return 0


if __name__ == '__main__':
    sys.exit(main())
