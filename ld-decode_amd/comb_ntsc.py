#!/usr/bin/env python3
"""comb-ntsc on the MI355X: the reference comb's frame stream (comb-ntsc.cxx
main :956-1125) with the 2D comb or the 3D comb without optical flow on the GPU.

    python ld-decode_amd/comb_ntsc.py [options] [-i infile] > out.rgb

Reads 910x525 uint16 .tbc frames from stdin (or -i) and writes rgb48 frames to
stdout, as `comb-ntsc` does.  The options are the reference's getopt string
"WQLakN:tFc:r:R:m8OwvDd:Bb:I:w:i:o:fphn:l:" with its meanings (:972-1068):

  -d N     comb dimension, 2 (default) or 3 (3D: optical flow, or -F)
  -F       3D without optical flow; -c core / -r range (IRE; defaults 1.25 / 5.5 with -F,
           0 / 0.5 with flow)
  -R x     p_3d2drej (parsed; the reference never uses it after main)
  -I ire   black level removed in the RGB conversion (default 7.5; encode-ntsc uses -I 0)
  -b x     brightness (default 236)
  -n ire   luma noise reduction clip (default 1; 0 turns DoYNR off)
  -N ire   chroma noise reduction clip (DoCNR; default 0 = off)
  -B       black and white (and dim 2)
  -a -L -Q toggle the adaptive 2D weights / the colour LPF / its HQ (I filter for Q)
  -v       525 output lines from line 20 (the VBI area; the last 20 lines black)
  -8       8-bit output (the high byte of each sample)
  -O       stop after the first frame written
  -p       pulldown: pair fields by the CAV / white-flag bits of line 0 px 13
  -f       one file per frame, <-o base><framecode>.rgb (16-bit), nothing on stdout
  -o base  the -f file name base (default FRAME)
  -l line  black out line (line + 25) of the output
  -W       910-wide output rows from x 0 instead of 744 from x 78 (a toggle, :974-976)
  -i file  input (default stdin)

-d 3 without -F (the reference's default) runs the 3D comb with optical flow:
OpenCV's Farneback is absent here, so the flow is this build's restatement of it
(csrc/flow.hip, oracle/farneback.py) -- BUILD-DEFINED, its parity with the
reference unpinned.  -k (combk view), -D (2D debug), -t
(training images) and -m (OpenCV monitor) are not built: they are rejected with a message rather than silently ignored.  A
short final frame ends the stream like the reference's exit(0) (:1104,1114).
Unknown options fail like the reference's getopt default (exit status 255).
"""
import getopt
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

IN_X, IN_Y = 910, 525
FRAME_BYTES = IN_X * IN_Y * 2
OUT_W = 744
OPTSTRING = 'WQLakN:tFc:r:R:m8OwvDd:Bb:I:w:i:o:fphn:l:'     # comb-ntsc.cxx:972
FRAME_INFO_CAV_EVEN, FRAME_INFO_CAV_ODD = 0x4, 0x8            # ld-decoder.h:247-252
FRAME_INFO_WHITE_ODD, FRAME_INFO_WHITE_EVEN = 0x100, 0x200
UNBUILT = {'-k': 'the combk view (-k)', '-D': 'the 2D debug mode (-D)',
           '-t': 'training mode (-t, OpenCV optical flow)', '-m': 'the OpenCV monitor (-m)'}


class Args:
    def __init__(self):
        self.dim, self.no_of, self.core, self.range = 2, False, -1.0, -1.0
        self.opts = {}
        self.write8, self.oneframe, self.pulldown, self.images = False, False, False, False
        self.image_base, self.infile = 'FRAME', None
        self.device, self.chunk = 0, 32


def parse(argv):
    """comb-ntsc's getopt loop (:972-1068); returns Args, or an int exit status."""
    a = Args()
    rest, i = [], 0
    while i < len(argv):                      # build-specific long options: --device N, --chunk N
        x = argv[i]
        if x in ('--device', '--chunk') and i + 1 < len(argv):
            setattr(a, x[2:], int(argv[i + 1]))
            i += 2
            continue
        if x.startswith('--device=') or x.startswith('--chunk='):
            k, v = x[2:].split('=', 1)
            setattr(a, k, int(v))
        else:
            rest.append(x)
        i += 1
    argv = rest
    try:
        opts, _ = getopt.getopt(argv, OPTSTRING)
    except getopt.GetoptError as e:
        print('comb: %s' % e, file=sys.stderr)
        return 255                            # default: return -1
    o = a.opts
    for k, v in opts:
        if k in UNBUILT:
            print('ERROR: %s is not available in this build' % UNBUILT[k], file=sys.stderr)
            return 1
        if k == '-W':
            o['wide'] = not o.get('wide', False)
        elif k == '-L':
            o['colorlpf'] = not o.get('colorlpf', True)
        elif k == '-Q':
            o['colorlpf_hq'] = not o.get('colorlpf_hq', True)
        elif k == '-a':
            o['adaptive2d'] = not o.get('adaptive2d', True)
        elif k == '-F':
            a.no_of = True
        elif k == '-c':
            a.core = float(v)
        elif k == '-r':
            a.range = float(v)
        elif k == '-R':
            pass                              # p_3d2drej: scaled in main, used nowhere
        elif k == '-8':
            a.write8 = True
        elif k == '-d':
            a.dim = int(v)
        elif k == '-O':
            a.oneframe = True
        elif k == '-v':
            o['linesout'] = IN_Y
        elif k == '-B':
            o['bw'] = True
            a.dim = 2
        elif k == '-b':
            o['brightness'] = float(v)
        elif k == '-I':
            o['black_ire'] = float(v)
        elif k == '-n':
            o['nr_y'] = float(v)
        elif k == '-N':
            o['nr_c'] = float(v)
        elif k == '-h':
            print('comb: \n-i [filename] : input filename (default: stdin)\n'
                  '-o [filename] : output filename/base (default: stdout/frame)\n'
                  '-d [dimensions] : Use 2D/3D comb filtering\n-B : B&W output\n'
                  '-f : use separate file for each frame\n-p : use white flag/frame # for pulldown\n'
                  '-l [line] : debug selected line - extra prints for that line, and blacks it out\n'
                  '-h : this', file=sys.stderr)
            return 0
        elif k == '-f':
            a.images = True
        elif k == '-p':
            a.pulldown = True
        elif k == '-i':
            a.infile = v
        elif k == '-o':
            a.image_base = v
        elif k == '-l':
            o['debug_line'] = int(v)
        else:                                 # -w (no case in the reference's switch)
            return 255
    return a


def read_frames(fh, n):
    """Up to n whole frames; a short read at the end stops the stream (:1102-1105)."""
    buf = fh.read(n * FRAME_BYTES)
    k = len(buf) // FRAME_BYTES
    return np.frombuffer(buf[:k * FRAME_BYTES], dtype=np.uint16).reshape(k, IN_Y, IN_X), k < n


class Writer:
    """PostProcess + WriteFrame (:894-938, :704-733) over the combed frames in order."""

    def __init__(self, a, out, lines, width=OUT_W):
        self.a, self.out, self.lines = a, out, lines
        self.obuf = np.zeros((lines, width, 3), dtype=np.uint16)   # persists across frames (pulldown)
        self.oddframe, self.framecode = False, 0

    def write(self, obuf, fnum):
        if self.a.images:
            with open('%s%d.rgb' % (self.a.image_base, fnum), 'wb') as fh:
                fh.write(obuf.tobytes())
        elif self.a.write8:
            self.out.write((obuf >> 8).astype(np.uint8).tobytes())
        else:
            self.out.write(obuf.tobytes())
        if self.a.oneframe:
            self.out.flush()
            raise SystemExit(0)

    def frame(self, rgb, raw):
        fstart = -1
        if not self.a.pulldown:
            fstart = 0
        elif self.oddframe:
            self.obuf[0::2] = rgb[0::2]
            self.write(self.obuf, self.framecode)
            self.oddframe = False
        flags = int(raw[0, 13])
        if flags & FRAME_INFO_CAV_ODD:
            fstart = 1
        elif flags & FRAME_INFO_CAV_EVEN:
            fstart = 0
        if flags & FRAME_INFO_WHITE_ODD:
            fstart = 1
        elif flags & FRAME_INFO_WHITE_EVEN:
            fstart = 0
        self.framecode = (int(raw[0, 14]) << 16) | int(raw[0, 15])
        if not self.a.pulldown or fstart == 0:
            self.obuf[:] = rgb
            self.write(self.obuf, self.framecode)
        elif fstart == 1:
            self.obuf[1::2] = rgb[1::2]
            self.oddframe = True


def main(argv=None):
    a = parse(sys.argv[1:] if argv is None else argv)
    if isinstance(a, int):
        return a
    if a.dim not in (2, 3):
        print('ERROR: -d must be 2 or 3 in this build', file=sys.stderr)
        return 1
    if a.dim == 3 and not a.no_of:
        if a.opts.get('wide'):
            print('ERROR: -W with the optical-flow 3D comb is not built (the flow path feeds the Y-NR '
                  'history -W shows); use -d 3 -F -W', file=sys.stderr)
            return 1
        a.opts['opticalflow'] = True
    from ldgpu import native
    ctx = native.Context('NTSC', a.device, max_reads=1, max_frames=a.chunk)
    ctx.comb_set_opts(**a.opts)
    ctx.comb_reset()
    fin = open(a.infile, 'rb') if a.infile else sys.stdin.buffer
    out = sys.stdout.buffer
    w = Writer(a, out, ctx.comb_lines, ctx.comb_width)
    held = []                                  # 3D: the raw frames of outputs still to come
    while True:
        fr, last = read_frames(fin, a.chunk)
        if fr.shape[0]:
            if a.dim == 2:
                rgb, raws = ctx.comb_ntsc(fr), fr
            else:
                rgb = ctx.comb_ntsc3d(fr, a.core, a.range)
                held.extend(fr)                # output k is input k + 1 (Process with f = 1)
                raws = held[1:1 + rgb.shape[0]]
                held = held[rgb.shape[0]:]
            for r, raw in zip(rgb, raws):
                w.frame(r, raw)
        if last:
            break
    out.flush()
    return 0


if __name__ == '__main__':
    sys.exit(main())
