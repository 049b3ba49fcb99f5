"""One steady-state decode loop (64-read launches, LDG_DEPTH (2) in flight) for a kernel trace:
    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof/st -o run -- python3 tools/stage_trace.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'ld-decode_amd'))


def main():
    from ldgpu import native
    from ldgpu.rfparams import RFTables
    batch, reps = int(os.environ.get('BATCH', '64')), int(os.environ.get('REPS', '12'))
    depth = int(os.environ.get('LDG_DEPTH', '2'))
    rf = RFTables('NTSC')
    ctx = native.Context('NTSC', 0, max_reads=depth * batch)
    ctx.set_filters(rf.params(), rf.tables)
    n = int(100000 + (batch + 2) * 667333)
    ctx.synth(n, fmt=0, first_frame=1, seed=3)
    starts = [100000 + i * 667333 for i in range(batch)]
    sl = [list(range(d * batch, (d + 1) * batch)) for d in range(depth)]
    import time
    t0 = time.perf_counter()
    log = []
    for r in range(reps):
        if r == 2:
            ctx.profile('demod')            # spans of the steady-state launches only
        a = time.perf_counter()
        ctx.decode_reads_async(starts, [1.0] * batch, sl[r % depth])
        b = time.perf_counter()
        if len(ctx._pending) >= depth:
            ctx.decode_reads_wait()
        c = time.perf_counter()
        log.append((r, (a - t0) * 1e6, (b - a) * 1e6, (c - b) * 1e6))
    if os.environ.get('VERBOSE'):
        for r, a, da, dw in log:
            print(f'rep {r:2d} async@{a:9.1f} us  async {da:7.1f} us  wait {dw:7.1f} us')
    import statistics
    while ctx._pending:
        ctx.decode_reads_wait()
    nsp, tsp = ctx.profile_spans()
    per = [b[1] - a[1] for a, b in zip(log[depth:], log[depth + 1:])]
    print(f"demod span {tsp / max(nsp, 1) * 1000:.1f} us/launch ({nsp}); stages {os.environ.get('LDG_STAGES', '7')} depth {depth}: period median {statistics.median(per):.1f} us "
          f"mean {statistics.mean(per):.1f} us (async {statistics.median(x[2] for x in log[depth:]):.1f}, "
          f"wait {statistics.median(x[3] for x in log[depth:]):.1f})")
    while ctx._pending:
        ctx.decode_reads_wait()


if __name__ == '__main__':
    main()
