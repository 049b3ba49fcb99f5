"""Per-kernel time of the 2D comb on its own (GPU box): decode a short capture
into the context's device frame buffer, then comb those frames repeatedly.

    python tools/comb_probe.py [--frames 30] [--reps 5]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'ld-decode_amd'))


def main():
    nf = int(sys.argv[sys.argv.index('--frames') + 1]) if '--frames' in sys.argv else 30
    reps = int(sys.argv[sys.argv.index('--reps') + 1]) if '--reps' in sys.argv else 5
    from ldgpu.decoder import GPUDecoder
    dec = GPUDecoder(system='NTSC', device=0, batch=64)
    n = int(40e6 * (nf / 29.97 * 1.25 + 0.3))
    dec.ctx.synth(n, fmt=0, first_frame=1, seed=7)
    dec.use_resident_capture(0, n)
    got = dec.decode(sink=None, comb=False, length=nf)
    dec.ctx.sync()
    print('frames in the device buffer: %d (last batch)' % got)
    m = min(nf, dec.ctx.max_frames)
    dec.ctx.comb_reset()
    dec.ctx.profile(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        dec.ctx.comb_ntsc_device(m)
    dec.ctx.sync()
    dt = time.perf_counter() - t0
    st = dec.ctx.profile_stats()
    dec.ctx.profile(False)
    print('comb of %d frames: %.3f ms per call (%.1f us per frame)' % (m, dt / reps * 1e3, dt / reps / m * 1e6))
    for k, (nl, ms) in sorted(st.items(), key=lambda kv: -kv[1][1]):
        print('  %-12s %4d launches %9.1f us per launch' % (k, nl, ms / nl * 1e3))


if __name__ == '__main__':
    main()
