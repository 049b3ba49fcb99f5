"""Long-capture decode probe: synthesise SECONDS of NTSC RF (CLV with --clv) in HBM,
decode it, and on failure print where the decode stood.

    python tools/long_probe.py 300 --clv
"""
import os
import sys
import time
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'ld-decode_amd'))


def main():
    from ldgpu.decoder import GPUDecoder
    secs = float(sys.argv[1])
    clv = '--clv' in sys.argv
    dec = GPUDecoder(system='NTSC', device=0, batch=96)
    log = {'miss': [], 'plan': []}
    orig_miss, orig_plan = dec._note_miss, dec._plan

    def note_miss(key):
        log['miss'] = (log['miss'] + [(key, dec.last_read, dec.mtf_level, dec.last_framenr, len(dec.frame_numbers))])[-4:]
        return orig_miss(key)

    def plan(nextsample, mtf, *a, **k):
        new, chain = orig_plan(nextsample, mtf, *a, **k)
        log['plan'] = (log['plan'] + [(nextsample, mtf, a[0], a[1], new[:3], len(new), chain[:3], len(chain))])[-4:]
        return new, chain
    dec._note_miss, dec._plan = note_miss, plan
    n = int(40e6 * secs)
    t0 = time.perf_counter()
    dec.ctx.synth(n, fmt=0, first_frame=1, clv=clv, seed=7)
    dec.use_resident_capture(0, n)
    print('synth %.1f s' % (time.perf_counter() - t0), flush=True)
    t0 = time.perf_counter()
    try:
        nfr = dec.decode(sink=None, comb=False)
        print('decoded %d frames in %.2f s; stats %s' % (nfr, time.perf_counter() - t0,
                                                       {k: v for k, v in dec.stats.items() if k != 'miss_log'}))
    except Exception:
        traceback.print_exc()
        nrs = dec.frame_numbers
        print('FAILED after %.2f s: %d frames, last framenrs %s' % (time.perf_counter() - t0, len(nrs), nrs[-5:]))
        print('cache %d entries, pending %d, stats %s' % (len(dec.cache), len(dec.pending),
                                                         {k: v for k, v in dec.stats.items() if k != 'miss_log'}))
        print('miss log tail', dec.stats.get('miss_log', [])[-10:])
        for m in log['miss']:
            print('miss', m)
        for p in log['plan']:
            print('plan', p)
        ks = sorted(dec.cache)
        print('cache keys (first/last 5):', ks[:5], ks[-5:])
        sys.exit(1)


if __name__ == '__main__':
    main()
