"""Nondeterminism probe: decode each golden case REPS times (batches 3 and 16) in one process
and report frames whose .tbc differs between repetitions or from the oracle by more than 1 LSB.
    python tools/nondet_probe.py REPS"""
import hashlib
import json
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'ld-decode_amd'), os.path.join(ROOT, 'tests', 'golden')]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    import make_golden
    from oracle.capture import FMT_BY_EXT
    from oracle.framer import decode_capture
    from ldgpu.decoder import GPUDecoder
    from ldgpu.formats import NAME_TO_FMT
    bad = 0
    cases = sys.argv[2].split(',') if len(sys.argv) > 2 else sorted(make_golden.CASES)
    for case in cases:
        gold = json.load(open(os.path.join(ROOT, 'tests', 'golden', case + '.json')))
        c = make_golden.CASES[case]
        data = make_golden.build_capture(case)
        frames, _, _ = decode_capture(data, FMT_BY_EXT[c['fmt']], system=c['system'])
        s = gold['settings']
        for batch in (3, 16):
            hashes = []
            for r in range(reps):
                dec = GPUDecoder(system=s['system'], batch=batch)
                dec.set_capture(data, NAME_TO_FMT[s['fmt']])
                got = []
                dec.decode(sink=lambda fr, au, m: got.append(fr.copy()))
                hashes.append([hashlib.sha256(f.tobytes()).hexdigest()[:8] for f in got])
                for k, (fr, f) in enumerate(zip(got, frames)):
                    W = 1135 if s['system'] == 'PAL' else 910
                    d = np.abs(fr.astype(np.int64) - f.astype(np.int64)).reshape(-1, W)
                    if d.max() > 1:
                        bad += 1
                        rows = np.where(d.max(axis=1) > 1)[0]
                        cols = np.where(d.max(axis=0) > 1)[0]
                        print('%s b%d rep %d frame %d: %d px > 1 rows %s (%d rows) cols %d..%d max %d' % (
                            case, batch, r, k, int((d > 1).sum()), list(rows[:12]), len(rows), cols.min(),
                            cols.max(), d.max()), flush=True)
            same = all(h == hashes[0] for h in hashes)
            print('%s batch %d: %d frames, reps identical: %s' % (case, batch, len(hashes[0]), same), flush=True)
    print('bad frames', bad)


if __name__ == '__main__':
    main()
