"""Throughput of the §8 f rows beside the headline path (GPU box):

    python tools/extras_bench.py [--frames 60]

2D NTSC comb, 3D NTSC comb (-d 3 -F), PAL Y/C decoder: host frames in, rgb48
out through the C ABI (H2D + kernels + D2H, the comb-ntsc stream boundary), and
device-resident 2D comb kernels alone; CX expander on the host.  Synthetic
frames (tests/test_comb.py / test_combpal.py patterns plus noise).  Prints one
JSON line."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'ld-decode_amd'), os.path.join(ROOT, 'tests')):
    sys.path.insert(0, p)


def timed(fn, reps=3):
    fn()                                   # warm-up
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return min(t)


def main():
    nf = int(sys.argv[sys.argv.index('--frames') + 1]) if '--frames' in sys.argv else 60
    from ldgpu import native
    from test_comb import frames_3d
    from test_combpal import pal_frames_noisy
    ctx = native.Context('NTSC', 0, max_reads=2, max_frames=nf)
    ntsc = np.concatenate([frames_3d(seed=s, n=6) for s in range((nf + 5) // 6)])[:nf]
    pal = np.concatenate([pal_frames_noisy(seed=s, n=3) for s in range((nf + 2) // 3)])[:nf]
    res = {'frames': nf}

    def c2():
        ctx.comb_reset()
        ctx.comb_ntsc(ntsc)
    res['comb2d_host_frames_per_s'] = nf / timed(c2)

    def c3():
        ctx.comb_reset()
        ctx.comb_ntsc3d(ntsc)
    res['comb3d_host_frames_per_s'] = nf / timed(c3)

    def cp():
        ctx.comb_reset()
        ctx.comb_pal(pal)
    res['combpal_host_frames_per_s'] = nf / timed(cp)

    cx = native.CXExpander()
    rng = np.random.default_rng(1)
    pcm = (32768 + rng.integers(-12000, 12000, (48000 * 60, 2))).astype(np.uint16)
    dt = timed(lambda: cx.process(pcm), reps=2)
    res['cx_host_stereo_samples_per_s'] = pcm.shape[0] / dt
    res['cx_realtime_x'] = pcm.shape[0] / dt / 48000
    print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in res.items()}))


if __name__ == '__main__':
    main()
