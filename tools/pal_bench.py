"""PAL decode throughput (SURVEY §8 d config C3 shape: PAL CLV, 40 MSPS u8), GPU box:

    python tools/pal_bench.py [--seconds 4] [--steps 2] [--no-comb]

The capture is synthesised on the host (ldgpu/synth.py, PAL timing, CLV
timecode) and made resident in HBM before the timed region; each step decodes
all of it RF -> .tbc + .pcm -> the PAL Y/C decoder's rgb48 (ldg_comb_async on
the assembled frames in HBM; config C3's "comb-pal Y/C path"), frames and rgb
left in HBM.  Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'ld-decode_amd'))


def main():
    secs = float(sys.argv[sys.argv.index('--seconds') + 1]) if '--seconds' in sys.argv else 4.0
    steps = int(sys.argv[sys.argv.index('--steps') + 1]) if '--steps' in sys.argv else 2
    from ldgpu.decoder import GPUDecoder
    from ldgpu.synth import make_capture
    t0 = time.perf_counter()
    data = make_capture(int(40e6 * secs), 'u8', system='PAL', clv=True, first_frame=3000, seed=20181018)
    synth_s = time.perf_counter() - t0
    batch = int(sys.argv[sys.argv.index('--batch') + 1]) if '--batch' in sys.argv else 96
    comb = '--no-comb' not in sys.argv
    dec = GPUDecoder(system='PAL', batch=batch)
    dec.set_capture(data, 0)
    dec._reset_cache()
    dec.decode(sink=None, comb=comb)                   # warm-up
    t0 = time.perf_counter()
    frames = consumed = 0
    for _ in range(steps):
        dec._reset_cache()                             # fresh read cache: no reuse across steps
        frames += dec.decode(sink=None, comb=comb)
        consumed += dec.last_meta['nextsample']
    dec.ctx.sync()
    dt = time.perf_counter() - t0
    msps = consumed / dt / 1e6
    print(json.dumps({'metric': 'RF Msamples/s (40 MSPS PAL CLV, RF->.tbc+.pcm%s)' % ('->PAL Y/C rgb48' if comb else ''),
                      'value': round(msps, 1),
                      'fields_per_s': round(2 * frames / dt, 1), 'realtime_x': round(msps / 40.0, 1),
                      'frames_per_step': frames // steps, 'seconds_of_rf': secs, 'steps': steps,
                      'synth_s': round(synth_s, 1), 'reads_decoded_total': dec.stats['reads'],
                      'reads_used_total': dec.stats['reads_used'], 'batches': dec.stats['batches'],
                      'misses': dec.stats.get('misses', 0), 'miss_sample': dec.stats.get('miss_log', [])[:8]}))


if __name__ == '__main__':
    main()
