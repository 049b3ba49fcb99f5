"""Per-phase workgroup time of the comb / TBC kernels from in-kernel clock stamps.

    python tools/demod_stamps.py --build    # here: the -DLDG_STAMPS variant (all stamps)
    python tools/kstamps.py [--seconds 3]   # on the GPU box

Decodes a short synthetic capture with the 2D comb through the stamps build and
prints, per stamped kernel (common.hpp KSTAMP), the median cycles of each phase
of a workgroup (the last launch's first 4096 workgroups)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'ld-decode_amd'))
VARIANT = os.path.join(ROOT, 'ld-decode_amd', 'ldgpu', 'libldgpu_stamps.so')
KERNELS = ['comb_fused', 'final_lines', 'burst_field', 'sync', 'burst_lines', 'philips']
NK, NB, NP = 6, 4096, 16


def main():
    secs = float(sys.argv[sys.argv.index('--seconds') + 1]) if '--seconds' in sys.argv else 3.0
    os.environ['LDGPU_LIB'] = VARIANT
    from ldgpu import native
    from ldgpu.decoder import GPUDecoder
    lib = native.load()
    lib.ldg_debug_kstamps.argtypes = [C.c_void_p, C.c_int]
    dec = GPUDecoder(system='NTSC', device=0, batch=64)
    n = int(40e6 * secs)
    dec.ctx.synth(n, fmt=0, first_frame=1, seed=5)
    st = np.zeros((NK, NB, NP), np.uint64)
    lib.ldg_debug_kstamps(st.ctypes.data, 1)
    dec.use_resident_capture(0, n)
    fr = dec.decode(sink=None, comb=True)
    dec.ctx.sync()
    lib.ldg_debug_kstamps(st.ctypes.data, 0)
    print('%d frames decoded' % fr)
    st = st.astype(np.int64)
    for k in range(NK):
        a = st[k]
        ok = a[:, 0] > 0
        if not ok.any():
            continue
        a = a[ok]
        last = max(i for i in range(NP) if (a[:, i] > 0).all())
        d = np.diff(a[:, :last + 1], axis=1)
        tot = a[:, last] - a[:, 0]
        span = a[:, last].max() - a[:, 0].min()
        print('%s: %d workgroups, median %.0f cycles (%.1f us at 2.4 GHz); first start -> last end %.1f us'
              % (KERNELS[k], ok.sum(), np.median(tot), np.median(tot) / 2400, span / 2400))
        for i in range(d.shape[1]):
            print('   phase %2d  median %8.0f  p90 %8.0f cycles' % (i, np.median(d[:, i]), np.percentile(d[:, i], 90)))


if __name__ == '__main__':
    main()
