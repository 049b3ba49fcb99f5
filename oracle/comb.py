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
