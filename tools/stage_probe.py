"""Throughput of the decode stages in isolation (GPU box).

    python tools/stage_probe.py [--batch 64] [--reps 8]

Decodes a batch of field reads fully once, then times repeated launches with
the LDG_STAGES mask (1 demod, 2 audio phase 2, 4 field chains; 7 = all), with
1 and 2 launches in flight.  Field-chain-only launches (4) re-run the chains
on the slots' demodulated channels."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'ld-decode_amd'))


def main():
    batch = int(sys.argv[sys.argv.index('--batch') + 1]) if '--batch' in sys.argv else 64
    reps = int(sys.argv[sys.argv.index('--reps') + 1]) if '--reps' in sys.argv else 8
    from ldgpu import native
    from ldgpu.rfparams import RFTables
    rf = RFTables('NTSC')
    ctx = native.Context('NTSC', 0, max_reads=2 * batch)
    ctx.set_filters(rf.params(), rf.tables)
    n = int(100000 + (batch + 2) * 667333)
    ctx.synth(n, fmt=0, first_frame=1, seed=3)
    starts = [100000 + i * 667333 for i in range(batch)]
    mt = [1.0] * batch
    sl = [list(range(batch)), list(range(batch, 2 * batch))]
    for q in range(2):
        ctx.decode_reads(starts, mt, sl[q])
    for mask in (7, 3, 1, 2, 4):
        os.environ['LDG_STAGES'] = str(mask)
        for depth in (1, 2):
            ctx.sync()
            t0 = time.perf_counter()
            for r in range(reps):
                ctx.decode_reads_async(starts, mt, sl[r % 2])
                if len(ctx._pending) >= depth:
                    ctx.decode_reads_wait()
            while ctx._pending:
                ctx.decode_reads_wait()
            dt = time.perf_counter() - t0
            print('stages %d depth %d: %.3f ms per batch of %d reads' % (mask, depth, dt / reps * 1e3, batch),
                  flush=True)
    os.environ['LDG_STAGES'] = '7'
    if '--prof' in sys.argv:
        # per-kernel launch durations, one launch in flight (LDG_DECODE_STREAMS=1: one chain per launch)
        for mask in (1, 2, 4):
            os.environ['LDG_STAGES'] = str(mask)
            ctx.profile(True)
            for r in range(reps):
                ctx.decode_reads(starts, mt, sl[r % 2])
            ctx.sync()
            st = ctx.profile_stats()
            ctx.profile(False)
            for k, (nl, ms) in sorted(st.items(), key=lambda kv: -kv[1][1]):
                print('  stages %d %-14s %5d launches  %8.1f us per launch' % (mask, k, nl, ms / nl * 1e3))
        os.environ['LDG_STAGES'] = '7'


if __name__ == '__main__':
    main()
