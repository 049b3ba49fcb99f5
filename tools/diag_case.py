"""Diagnose an end-to-end golden case: per frame, where the GPU .tbc differs from the oracle's.
    python tools/diag_case.py CASE BATCH [REPS]"""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'ld-decode_amd'), os.path.join(ROOT, 'tests', 'golden')]


def main():
    case, batch = sys.argv[1], int(sys.argv[2])
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    import json
    import make_golden
    from oracle.capture import FMT_BY_EXT
    from oracle.framer import decode_capture
    from ldgpu.decoder import GPUDecoder
    from ldgpu.formats import NAME_TO_FMT
    gold = json.load(open(os.path.join(ROOT, 'tests', 'golden', case + '.json')))
    c = make_golden.CASES[case]
    data = make_golden.build_capture(case)
    frames, pcm, meta = decode_capture(data, FMT_BY_EXT[c['fmt']], system=c['system'])
    s = gold['settings']
    for r in range(reps):
        dec = GPUDecoder(system=s['system'], batch=batch)
        dec.set_capture(data, NAME_TO_FMT[s['fmt']])
        got = []
        dec.decode(sink=lambda fr, au, m: got.append((fr.copy(), au.copy(), m)))
        print('rep', r, 'frames', len(got), 'oracle', len(frames), 'stats', dec.stats)
        for k, ((fr, au, m), f) in enumerate(zip(got, frames)):
            d = np.abs(fr.astype(np.int64) - f.astype(np.int64)).reshape(f.shape)
            if d.max() > 1:
                rows = np.where(d.max(axis=1) > 1)[0]
                cols = np.where(d.max(axis=0) > 1)[0]
                print('  frame %d: %d px > 1, rows %s..%s (%d), cols %s..%s, max %d' % (
                    k, int((d > 1).sum()), rows.min(), rows.max(), len(rows), cols.min(), cols.max(), d.max()))
                for row in rows[:4]:
                    cc = np.where(d[row] > 1)[0]
                    print('    row', row, 'gpu', fr.reshape(f.shape)[row, cc[:6]], 'oracle', f[row, cc[:6]])


if __name__ == '__main__':
    main()
