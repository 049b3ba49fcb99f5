"""Decode-pipeline configuration sweep (GPU box): wall time of one full decode of a
synthetic NTSC capture per configuration, in one process.

    python tools/pipe_probe.py [--seconds 20] [--batch 64]

Configurations vary the launch depth (LDG_DEPTH semantics, set on the decoder)
and in-library event timing (on / off)."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'ld-decode_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--seconds', type=float, default=20.0)
    ap.add_argument('--batch', type=int, default=64)
    ap.add_argument('--comb', action='store_true')
    args = ap.parse_args()
    from ldgpu.decoder import GPUDecoder
    dec = GPUDecoder(system='NTSC', device=0, batch=args.batch)
    n = int(40e6 * args.seconds)
    dec.ctx.synth(n, fmt=0, first_frame=1, seed=1)
    for depth in (2, 1, 2):
        for prof in (False, True):
            dec.depth = depth
            dec.ctx.profile(prof)
            dec.stats = {k: 0 for k in ('batches', 'reads', 'reads_used')}
            dec.stats.update(gpu_s=0.0, replay_s=0.0)
            dec.use_resident_capture(0, n)
            t0 = time.perf_counter()
            fr = dec.decode(sink=None, comb=args.comb)
            dt = time.perf_counter() - t0
            st = dec.stats
            print('depth %d prof %d: %d frames %.1f ms  %.0f MS/s  host %s' % (
                depth, prof, fr, dt * 1e3, dec.last_meta['nextsample'] / dt / 1e6,
                {k: round(v, 4) for k, v in st.items() if k.endswith('_s')}), flush=True)
    dec.ctx.profile(False)


if __name__ == '__main__':
    main()
