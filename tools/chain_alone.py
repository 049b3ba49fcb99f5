"""Field-chain kernels alone on the GPU: decode a batch once (everything), then
re-run only the field chains (LDG_STAGES=4) on the same slots, so each kernel's
HIP-event time is its time with the whole GPU and no demod beside it.

    BATCH=96 REPS=10 python tools/chain_alone.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'ld-decode_amd'))


def main():
    from ldgpu import native
    from ldgpu.rfparams import RFTables
    batch, reps = int(os.environ.get('BATCH', '96')), int(os.environ.get('REPS', '10'))
    rf = RFTables('NTSC')
    ctx = native.Context('NTSC', 0, max_reads=batch)
    ctx.set_filters(rf.params(), rf.tables)
    n = int(100000 + (batch + 2) * 667333)
    ctx.synth(n, fmt=0, first_frame=1, seed=3)
    starts = [100000 + i * 667333 for i in range(batch)]
    slots = list(range(batch))
    for stages in ('7', '4'):
        os.environ['LDG_STAGES'] = stages
        ctx.decode_reads_async(starts, [1.0] * batch, slots)
        ctx.decode_reads_wait()
    for mode in ('4', '5', '1'):
        os.environ['LDG_STAGES'] = mode
        ctx.profile(True)
        t0 = time.perf_counter()
        for r in range(reps):
            ctx.decode_reads_async(starts, [1.0] * batch, slots)
            ctx.decode_reads_wait()
        wall = (time.perf_counter() - t0) / reps * 1e3
        st = ctx.profile_stats()
        ctx.profile(False)
        print('stages %s: wall %.3f ms per call' % (mode, wall))
        for k, (nl, ms) in sorted(st.items(), key=lambda kv: -kv[1][1]):
            print('   %-14s %6.1f us per call (%d launches)' % (k, ms / reps * 1e3, nl))
    os.environ.pop('LDG_STAGES')


if __name__ == '__main__':
    main()
