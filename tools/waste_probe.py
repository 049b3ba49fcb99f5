"""Where the speculative planner's unused reads come from (one bench-sized decode).

    python tools/waste_probe.py            # on the GPU box

Prints the decoded-but-never-requested reads, grouped by position in the capture,
and whether a read of the same field (within +-4096 samples) was used instead.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'ld-decode_amd'))


def main():
    import numpy as np
    from ldgpu.decoder import GPUDecoder
    secs = float(os.environ.get('SECONDS_', '60'))
    dec = GPUDecoder('NTSC', device=0, batch=int(os.environ.get('BATCH', '96')))
    n = int(40e6 * secs)
    dec.ctx.synth(n, fmt=0, first_frame=1, seed=7)
    dec.use_resident_capture(0, n)
    launched, requested = [], []
    orig_async = dec._launch_async

    def rec_async(keys, protect):
        launched.extend(keys)
        return orig_async(keys, protect)
    dec._launch_async = rec_async
    orig_get = dec._get

    def rec_get(readsample, mtf, audio_offset):
        requested.append((int(readsample), mtf))
        return orig_get(readsample, mtf, audio_offset)
    dec._get = rec_get
    nf = dec.decode(comb=False)
    req = set(requested)
    unused = [k for k in launched if k not in req]
    used_starts = np.array(sorted({k[0] for k in req}))
    print('frames', nf, 'launched', len(launched), 'distinct', len(set(launched)), 'requested', len(req),
          'unused', len(unused), 'batches', dec.stats['batches'])
    near, far = 0, []
    for s, m in unused:
        i = np.searchsorted(used_starts, s)
        d = min([abs(s - used_starts[j]) for j in (i - 1, i) if 0 <= j < len(used_starts)] or [10 ** 9])
        if d <= 4096:
            near += 1
        else:
            far.append(s)
    print('unused near a used read (mispredicted start/mtf):', near, ' far from any used read:', len(far))
    if far:
        far = np.array(sorted(far))
        print('far ones: first %d last %d (capture %d samples); beyond the last used read: %d' % (
            far[0], far[-1], n, int((far > used_starts[-1]).sum())))
    mis_mtf = sum(1 for s, m in unused if any(abs(s - u) <= 4096 for u in used_starts[max(0, np.searchsorted(used_starts, s) - 1):np.searchsorted(used_starts, s) + 1]) and (s, m) not in req and any(k[0] == s for k in req))
    print('same start, other mtf:', mis_mtf)


if __name__ == '__main__':
    main()
