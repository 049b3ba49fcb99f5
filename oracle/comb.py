"""ORACLE -- test infrastructure only.  ctypes wrapper of oracle/comb2d.cpp, the
C++ restatement of the reference NTSC comb (comb-ntsc.cxx dim=2 defaults, and
the non-optical-flow 3D path -d 3 -F).
Built by oracle/Makefile into oracle/_build/libcomb2d.so."""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, '_build', 'libcomb2d.so')
IN_X, IN_Y, OUT_W, OUT_H = 910, 525, 744, 480


def _load():
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(os.path.join(HERE, 'comb2d.cpp')):
        subprocess.check_call(['make', '-s', '-C', HERE])
    lib = C.CDLL(LIB)
    lib.comb2d_create.restype = C.c_void_p
    lib.comb2d_destroy.argtypes = [C.c_void_p]
    lib.comb2d_process.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    lib.comb2d_set_opts.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    lib.comb3d_set_opts.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    lib.comb2d_aburstlev.argtypes = [C.c_void_p]
    lib.comb2d_aburstlev.restype = C.c_double
    lib.comb3d_create.restype = C.c_void_p
    lib.comb3d_destroy.argtypes = [C.c_void_p]
    lib.comb3d_process.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_double, C.c_double]
    lib.comb3d_process.restype = C.c_int
    lib.comb3d_aburstlev.argtypes = [C.c_void_p]
    lib.comb3d_aburstlev.restype = C.c_double
    lib.comb2d_process_of.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    lib.comb2d_flow_luma.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    lib.comb2d_set_nr_min.argtypes = [C.c_void_p, C.c_double]
    return lib


DEFAULT_OPTS = dict(black_ire=7.5, brightness=236.0, nr_y=1.0, nr_c=0.0, bw=False, adaptive2d=True,
                    colorlpf=True, colorlpf_hq=True, linesout=480, debugline=-1000, wide=False)


def _set_opts(fn, h, opts):
    """comb-ntsc's options (comb-ntsc.cxx:972-1091): -I black_ire, -b brightness, -n nr_y,
    -N nr_c (IRE), -B bw, -a / -L / -Q toggles, -v linesout 525, -l debugline, -W wide."""
    o = dict(DEFAULT_OPTS)
    for k, v in opts.items():
        if k not in o:
            raise TypeError('unknown comb option %s' % k)
        o[k] = v
    d = np.array([o['black_ire'], o['brightness'], o['nr_y'], o['nr_c']], dtype=np.float64)
    i = np.array([o['bw'], o['adaptive2d'], o['colorlpf'], o['colorlpf_hq'], o['linesout'], o['debugline'],
                  o['wide']], dtype=np.int32)
    fn(h, d.ctypes.data, i.ctypes.data)
    return o


class Comb2D:
    """One reference comb process: state (aburstlev, Y-NR / C-NR FIR histories) carries
    across calls.  Keyword options as in DEFAULT_OPTS (comb-ntsc's command line)."""

    def __init__(self, **opts):
        self.lib = _load()
        self.h = self.lib.comb2d_create()
        self.opts = _set_opts(self.lib.comb2d_set_opts, self.h, opts)

    def __del__(self):
        if getattr(self, 'h', None):
            self.lib.comb2d_destroy(self.h)
            self.h = None

    def process(self, frames):
        f = np.ascontiguousarray(frames, dtype=np.uint16).reshape(-1, IN_Y, IN_X)
        out = np.zeros((f.shape[0], self.opts['linesout'], IN_X if self.opts['wide'] else OUT_W, 3),
                       dtype=np.uint16)
        self.lib.comb2d_process(self.h, f.shape[0], f.ctypes.data, out.ctypes.data)
        return out

    @property
    def aburstlev(self):
        return self.lib.comb2d_aburstlev(self.h)


class Comb3D:
    """One reference comb process run as `comb-ntsc -d 3 -F [-c core] [-r range]`:
    frame k is output once frame k+1 has arrived (none for the first two inputs)."""

    def __init__(self, core_ire=-1.0, range_ire=-1.0, **opts):
        self.lib = _load()
        self.h = self.lib.comb3d_create()
        self.core, self.range = core_ire, range_ire
        self.opts = _set_opts(self.lib.comb3d_set_opts, self.h, opts)

    def __del__(self):
        if getattr(self, 'h', None):
            self.lib.comb3d_destroy(self.h)
            self.h = None

    def process(self, frames):
        f = np.ascontiguousarray(frames, dtype=np.uint16).reshape(-1, IN_Y, IN_X)
        out = np.zeros((f.shape[0], self.opts['linesout'], IN_X if self.opts['wide'] else OUT_W, 3),
                       dtype=np.uint16)
        n = self.lib.comb3d_process(self.h, f.shape[0], f.ctypes.data, out.ctypes.data, self.core, self.range)
        return out[:n]

    @property
    def aburstlev(self):
        return self.lib.comb3d_aburstlev(self.h)


class Comb3DFlow:
    """One reference comb process run as `comb-ntsc -d 3` (optical flow; comb-ntsc.cxx
    Process :834-892 with f = 1, OpticalFlow3D :600-662, Split3D(f, true) :369-412).
    BUILD-DEFINED and parity unpinned: the flow is oracle/farneback.py's restatement of
    OpenCV's Farneback.  Per input frame g: from g = 1 the flow path's luma fields; from
    g = 2 the flow against the previous frame's (the last flow as the initial estimate from
    g = 3) and the weight map of frame g - 1, which is then output (clp2 = frame g -
    frame g - 1): nothing for the first two inputs, one frame late, never the last.  The
    flow path raises the Y / C noise-reduction clips to 4 (raw) from the second frame."""

    def __init__(self, core_ire=-1.0, range_ire=-1.0, **opts):
        self.lib = _load()
        self.h = self.lib.comb2d_create()
        self.opts = _set_opts(self.lib.comb2d_set_opts, self.h, opts)
        # comb-ntsc main() with flow: p_3dcore / p_3drange 0 / 0.5 IRE by default, times irescale
        self.core = (0.0 if core_ire < 0 else core_ire) * 358.4
        self.range = (0.5 if range_ire < 0 else range_ire) * 358.4
        self.g, self.prev_fields, self.flow, self.held = 0, None, None, None
        self.kmaps = {}

    def __del__(self):
        if getattr(self, 'h', None):
            self.lib.comb2d_destroy(self.h)
            self.h = None

    def luma_fields(self, frame):
        from .farneback import field_images
        y = np.zeros((IN_Y, IN_X), dtype=np.float64)
        f = np.ascontiguousarray(frame, dtype=np.uint16)
        self.lib.comb2d_flow_luma(self.h, f.ctypes.data, y.ctypes.data)
        return field_images(y)

    def process(self, frames):
        from .farneback import combk_from_flow, farneback
        f = np.ascontiguousarray(frames, dtype=np.uint16).reshape(-1, IN_Y, IN_X)
        W = IN_X if self.opts['wide'] else OUT_W
        outs = []
        for fr in f:
            g = self.g
            self.g += 1
            if g >= 1:
                self.lib.comb2d_set_nr_min(self.h, 4.0)
                cur = self.luma_fields(fr)
                if g >= 2:
                    init = self.flow if g >= 3 else [None, None]
                    self.flow = [farneback(cur[k], self.prev_fields[k], init[k]) for k in range(2)]
                    km = np.ascontiguousarray(combk_from_flow(self.flow[0], self.flow[1], self.core, self.range))
                    out = np.zeros((self.opts['linesout'], W, 3), dtype=np.uint16)
                    self.lib.comb2d_process_of(self.h, self.held.ctypes.data, fr.ctypes.data, km.ctypes.data,
                                               out.ctypes.data)
                    outs.append(out)
                self.prev_fields = cur
            self.held = np.ascontiguousarray(fr)
        return np.stack(outs) if outs else np.zeros((0, self.opts['linesout'], W, 3), dtype=np.uint16)

    @property
    def aburstlev(self):
        return self.lib.comb2d_aburstlev(self.h)


PAL_IN_X, PAL_IN_Y, PAL_OUT_W, PAL_OUT_H = 1135, 625, 1057, 576
LIB_PAL = os.path.join(HERE, '_build', 'libcombpal.so')


class CombPAL:
    """The build-defined PAL Y/C decoder's checker (oracle/combpal.cpp): one process."""

    def __init__(self):
        if not os.path.exists(LIB_PAL) or os.path.getmtime(LIB_PAL) < os.path.getmtime(os.path.join(HERE, 'combpal.cpp')):
            subprocess.check_call(['make', '-s', '-C', HERE])
        self.lib = C.CDLL(LIB_PAL)
        self.lib.combpal_create.restype = C.c_void_p
        self.lib.combpal_destroy.argtypes = [C.c_void_p]
        self.lib.combpal_process.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
        self.lib.combpal_aburstlev.argtypes = [C.c_void_p]
        self.lib.combpal_aburstlev.restype = C.c_double
        self.h = self.lib.combpal_create()

    def __del__(self):
        if getattr(self, 'h', None):
            self.lib.combpal_destroy(self.h)
            self.h = None

    def process(self, frames):
        f = np.ascontiguousarray(frames, dtype=np.uint16).reshape(-1, PAL_IN_Y, PAL_IN_X)
        out = np.zeros((f.shape[0], PAL_OUT_H, PAL_OUT_W, 3), dtype=np.uint16)
        self.lib.combpal_process(self.h, f.shape[0], f.ctypes.data, out.ctypes.data)
        return out

    @property
    def aburstlev(self):
        return self.lib.combpal_aburstlev(self.h)
