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
    if os.environ.get('LDG_ISO_ANY') == '1':
        # timing probes of deliberately broken builds: 96 reads at the nominal field
        # spacing, decoded once (whatever their fields come out as), then the leg
        starts = [1000000 + 667333 * k for k in range(96)]
        dec.ctx.decode_reads_async(starts, [1.0] * 96, list(range(96)))
        dec.ctx.decode_reads_wait()
        t1 = time.perf_counter()
        reads, ms = 96, dec.ctx.demod_isolated(list(range(96)), iters)
    else:
        dec.decode(length=100)
        t1 = time.perf_counter()
        reads, ms = dec.demod_isolated(iters)
    print(json.dumps({'reads': reads, 'iters': iters, 'ms_per_launch': round(ms, 4), 'decode_s': round(t1 - t0, 2)}))


if __name__ == '__main__':
    main()
