"""Host timeline of bench.py's step (one full 60 s decode): when each launch is
issued / waited for, relative to the step start, to see the start-up and tail
costs of a decode.

    python tools/step_probe.py [--steps 3]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'ld-decode_amd'))


def main():
    steps = int(sys.argv[sys.argv.index('--steps') + 1]) if '--steps' in sys.argv else 3
    from ldgpu.decoder import GPUDecoder
    dec = GPUDecoder(system='NTSC', device=0, batch=96)
    nsamp = int(40e6 * 60)
    dec.ctx.synth(nsamp, fmt=0, first_frame=1, seed=20181015)
    log = []
    orig_async, orig_wait, orig_flush = dec._launch_async, dec._launch_wait, dec._flush

    def la(keys, protect):
        log.append(('launch', time.perf_counter(), len(keys)))
        return orig_async(keys, protect)

    def lw():
        t = time.perf_counter()
        r = orig_wait()
        log.append(('wait', t, time.perf_counter() - t))
        return r

    def fl(frames, W, H, sink):
        t = time.perf_counter()
        r = orig_flush(frames, W, H, sink)
        log.append(('flush', t, time.perf_counter() - t, len(frames)))
        return r
    dec._launch_async, dec._launch_wait, dec._flush = la, lw, fl
    for s in range(steps + 1):
        dec.use_resident_capture(0, nsamp)
        log.clear()
        t0 = time.perf_counter()
        dec.decode(sink=None, comb=True)
        t1 = time.perf_counter()
        if s == 0:
            continue
        print('step %d: %.2f ms, %d launches' % (s, (t1 - t0) * 1e3, sum(1 for e in log if e[0] == 'launch')))
        for e in log[:14]:
            print('   %-6s at %7.2f ms  %s' % (e[0], (e[1] - t0) * 1e3, ' '.join('%.2f' % (x * 1e3) if isinstance(x, float) else str(x) for x in e[2:])))
        print('   ...')
        for e in log[-8:]:
            print('   %-6s at %7.2f ms  %s' % (e[0], (e[1] - t0) * 1e3, ' '.join('%.2f' % (x * 1e3) if isinstance(x, float) else str(x) for x in e[2:])))
        print('   return at %.2f ms' % ((t1 - t0) * 1e3))


if __name__ == '__main__':
    main()
