"""Which reads does the planner decode without the replay using them (PAL CLV)?

    python tools/pal_waste.py [--seconds 4] [--dump out.json]

--dump writes the used read starts, the launches and every decoded read's next
start (start + nextfieldoffset) for offline study of the read chain.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'ld-decode_amd'))


def main():
    secs = float(sys.argv[sys.argv.index('--seconds') + 1]) if '--seconds' in sys.argv else 4.0
    from ldgpu.decoder import GPUDecoder
    from ldgpu.synth import make_capture
    data = make_capture(int(40e6 * secs), 'u8', system='PAL', clv=True, first_frame=3000, seed=20181018)
    dec = GPUDecoder(system='PAL', batch=96)
    launched = []
    orig = dec._launch_async

    def la(keys, protect):
        r = orig(keys, protect)
        launched.append(list(keys))
        return r
    dec._launch_async = la
    used = []
    orig_get = dec._get

    def get(rs, mtf, ao):
        f = orig_get(rs, mtf, ao)
        used.append((int(rs), mtf))
        return f
    dec._get = get
    dec.set_capture(data, 0)
    n = dec.decode(sink=None)
    allk = [k for b in launched for k in b]
    us = set(used)
    print('frames %d, launches %d, reads %d, used %d, unused %d' % (n, len(launched), len(allk), len(us), len([k for k in allk if k not in us])))
    last_used = max(k[0] for k in us)
    seq = sorted(k[0] for k in us)
    import collections
    for P in (2, 4, 8):
        d = collections.Counter(seq[i + P] - seq[i] for i in range(len(seq) - P))
        print('r[k+%d] - r[k]: %s' % (P, d.most_common(6)))
    print('first diffs', [seq[i + 1] - seq[i] for i in range(min(30, len(seq) - 1))])
    for i, b in enumerate(launched):
        un = [k for k in b if k not in us]
        past = sum(1 for k in un if k[0] > last_used)
        near = []
        for k in un[:6]:
            d = min(abs(k[0] - u[0]) for u in us)
            near.append((k[0], d))
        print('launch %2d: %3d reads, %3d unused (%3d past the last used read) e.g. %s' % (i, len(b), len(un), past, near))
    if '--dump' in sys.argv:
        import json
        out = {'used': seq, 'launches': [[k[0] for k in b] for b in launched],
               'next': {str(k): int(v[0]) for k, v in dec.hints.items()},
               'status': {str(k[0]): int(v[1].status) for k, v in dec.cache.items()}}
        with open(sys.argv[sys.argv.index('--dump') + 1], 'w') as f:
            json.dump(out, f)


if __name__ == '__main__':
    main()
