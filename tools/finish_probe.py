"""Where the sharded decode's finish phase (ShardedDecode.finish: the exact 48 kHz audio
from the archive, global frame indices) spends its time, on config 5's one-GPU leg.

    python tools/finish_probe.py [seconds]      # GPU box; prints phase times and a cProfile of finish
"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'ld-decode_amd'))


def main():
    from ldgpu.decoder import GPUDecoder
    from ldgpu.shard import ShardedDecode
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 120.0
    n = int(40e6 * seconds)
    dec = GPUDecoder(system='NTSC', batch=96)
    dec.ctx.synth(n, fmt=0, first_frame=1, clv=True, seed=20181015, start_sample=0)
    for rep in range(3):
        dec.use_resident_capture(0, n)
        sd = ShardedDecode(dec, 0, 1, resident=True, comb=True)
        t0 = time.perf_counter()
        loc = sd.local()
        t1 = time.perf_counter()
        prof = cProfile.Profile() if rep == 2 else None
        if prof:
            prof.enable()
        res = sd.finish([loc])
        if prof:
            prof.disable()
        t2 = time.perf_counter()
        print('rep %d: %d frames, local %.1f ms, finish %.1f ms' % (rep, len(res), (t1 - t0) * 1e3, (t2 - t1) * 1e3),
              flush=True)
    pstats.Stats(prof).sort_stats('cumulative').print_stats(18)


if __name__ == '__main__':
    main()
