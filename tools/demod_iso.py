"""The isolated demod leg alone (no CPU baseline, no timed pipeline): decode 10 s of
synthetic NTSC RF once, then time `iters` back-to-back launches of the roofline
kernel over 96 reads.  For quick A/B and rocprofv3 --pmc passes of the demod.

    python tools/demod_iso.py [iters] [seconds]
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), 'ld-decode_amd'))

from ldgpu.decoder import GPUDecoder  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    seconds = float(sys.argv[2]) if len(sys.argv) > 2 else 10.0
    dec = GPUDecoder(system='NTSC', batch=96)
    n = int(40e6 * seconds)
    dec.ctx.synth(n, fmt=0, first_frame=1, clv=False, seed=20181017)
    dec.use_resident_capture(0, n)
    t0 = time.perf_counter()
    dec.decode(length=100)
    t1 = time.perf_counter()
    reads, ms = dec.demod_isolated(iters)
    print(json.dumps({'reads': reads, 'iters': iters, 'ms_per_launch': round(ms, 4), 'decode_s': round(t1 - t0, 2),
                      'demod2': os.environ.get('LDG_DEMOD2', '0') != '0'}))


if __name__ == '__main__':
    main()
