"""Per-phase time of the demod kernel from in-kernel clock stamps.

    python tools/demod_stamps.py --build        # here: the -DLDG_STAMPS variant of libldgpu
    python tools/demod_stamps.py                # on the GPU box: decode 64 reads, print phases

The variant lives at ld-decode_amd/ldgpu/libldgpu_stamps.so and is loaded through LDGPU_LIB.
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'ld-decode_amd'))
VARIANT = os.path.join(ROOT, 'ld-decode_amd', 'ldgpu', 'libldgpu_stamps.so')
PHASES = {0: 'prologue+load', 1: 'raw FFT', 2: 'split/filter/park', 3: 'E IFFT wait', 4: 'E IFFT',
          5: 'E atan2 + O reload', 6: 'O IFFT', 7: 'O atan2 + phase', 8: 'FM demod', 9: 'D FFT', 10: 'D split',
          11: '05 merge', 12: '05 IFFT', 13: '05 store + bits', 14: 'sync scan + store', 15: 'video merge',
          16: 'video IFFT', 17: 'video store', 18: 'burst scan + store'}


def main():
    if '--build' in sys.argv:
        sys.path.insert(0, os.path.join(ROOT, 'ld-decode_amd'))
        import build
        build.build_variant(VARIANT, ('LDG_STAMPS',))
        return
    os.environ['LDGPU_LIB'] = VARIANT
    from ldgpu import native
    from ldgpu.rfparams import RFTables
    from ldgpu.synth import make_capture
    lib = native.load()
    lib.ldg_debug_stamps.argtypes = [C.c_void_p]
    n = 32
    data = np.frombuffer(make_capture(int(40e6 * 0.85), 'u8'), np.uint8)
    rf = RFTables('NTSC')
    ctx = native.Context('NTSC', 0, max_reads=n)
    ctx.set_filters(rf.params(), rf.tables)
    ctx.set_capture(data, data.size, 0, 0)
    starts = [int(i * 1.0e6) for i in range(n)]
    for _ in range(3):
        ctx.decode_reads(starts, [1.0] * n)
    st = np.zeros((8192, 32), np.uint64)
    lib.ldg_debug_stamps(st.ctypes.data)
    blocks = 66 * n
    st = st[:min(blocks, 8192)].astype(np.int64)
    last = max(i for i in range(32) if (st[:, i] > 0).any())
    ok = st[:, last] > 0
    d = np.diff(st[ok][:, :last + 1], axis=1)
    tot = st[ok, last] - st[ok, 0]
    print('blocks %d, median block %.0f cycles (%.1f us at 2.4 GHz)' % (ok.sum(), np.median(tot), np.median(tot) / 2400))
    for i in range(d.shape[1]):
        name = PHASES.get(i, '?')
        if name == '-':
            continue
        med = np.median(d[:, i])
        print('%2d %-22s %8.0f cycles  %5.1f%%' % (i, name, med, 100 * med / np.median(tot)))

if __name__ == '__main__':
    main()
