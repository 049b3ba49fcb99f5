"""GPU probe: the sharded decode's frames against one decode,
repeated, with the differing frames described.  python tools/shard_probe.py [world] [reps]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'ld-decode_amd'))


def main():
    from ldgpu.decoder import GPUDecoder
    from ldgpu.shard import ShardedDecode, check_chain
    from ldgpu.synth import make_capture
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    data = make_capture(int(40e6 * 0.6), 'u8', first_frame=1200, seed=21)
    for rep in range(reps):
        ref = GPUDecoder(system='NTSC', batch=8)
        ref.set_capture(data, 0)
        want = []
        ref.decode(sink=lambda fr, au, m: want.append((fr.copy(), au.copy(), m)))
        decs = [GPUDecoder(system='NTSC', batch=8) for _ in range(world)]
        for d in decs:
            d.set_capture(data, 0)
        sds = [ShardedDecode(d, r, world) for r, d in enumerate(decs)]
        summ = [sd.local() for sd in sds]
        assert check_chain(summ) == []
        got = []
        for sd in sds:
            got += [(np.array(pic), a, m) for (g, a, m), pic in zip(sd.finish(summ), sd.frames)]
        bad = []
        for i, ((gf, ga, gm), (wf, wa, wm)) in enumerate(zip(got, want)):
            if gm != wm:
                bad.append((i, 'meta'))
            elif not np.array_equal(gf, wf):
                d = np.flatnonzero(gf != wf)
                bad.append((i, d.size, int(d[0]) // 910, int(d[-1]) // 910,
                            int(np.abs(gf.astype(int) - wf.astype(int)).max())))
            elif not np.array_equal(ga, wa):
                bad.append((i, 'audio'))
        ranks = [s['n'] for s in summ]
        print('rep %d: frames %d/%d per-rank %s mismatches %s' % (rep, len(got), len(want), ranks, bad[:8]), flush=True)


if __name__ == '__main__':
    main()
