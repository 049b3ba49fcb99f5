"""Benchmark: RF Msamples/s and fields/s of the MI355X decode path (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W]
    (N > 1: torch.distributed.run, one rank per GPU, weak scaling)

Workload (BASELINE.json configs[1]): 60 s of synthetic NTSC CAV RF, 40 MSPS,
8-bit, per GPU, synthesised on the GPU straight into HBM (same signal model as
ldgpu/synth.py).  One step = the full reference decode of that capture:
RF -> demod -> TBC -> .tbc frames (+ .pcm audio), every frame of the 60 s,
with the .tbc frames assembled in HBM.  Ranks decode independent captures
(fields shard by capture; no data-path collective).
"""
import argparse
import contextlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'ld-decode_amd'))

import numpy as np  # noqa: E402

# each of the decode context's streams gets a hardware queue (ldgpu/__init__.py);
# set before torch (N > 1) initialises the HIP runtime
if int(os.environ.get('GPU_MAX_HW_QUEUES', '0') or 0) < 12:
    os.environ['GPU_MAX_HW_QUEUES'] = '12'

NTSC_TBC_BYTES_PER_SAMPLE = 955500 / 1334667
NTSC_PCM_BYTES_PER_SAMPLE = 0.0048
NTSC_COMB_BYTES_PER_SAMPLE = (955500 + 2142720) / 1334667   # .tbc in + rgb48 out per frame
BYTES_PER_SAMPLE = {0: 1.0, 1: 2.0, 2: 4 / 3, 3: 1.25}
FMT_NAME = {0: 'u8', 1: 's16', 2: '10-bit .r30', 3: '10-bit .lds'}
HBM_PEAK_GBS = 8000.0
FP64_PEAK_TFLOPS = 78.6                           # MI355X FP64 vector (spec)
READ_BLOCKS = 66                                  # overlap-save blocks per 1e6-sample field read
ISO_ITERS = 20                                    # launches of the isolated roofline leg
# the FFT flops the demod executes per block (5 N log2 N): six 8192-point complex transforms
# (raw R2C, analytic even / odd, demod R2C, C2R 0.5 MHz, C2R video) + two 1024-point audio IFFTs;
# sync / burst / pilot are time-domain recurrences (iir.hpp) and are not counted
DEMOD_FLOPS_PER_BLOCK = 6 * 5 * 8192 * 13 + 2 * 5 * 1024 * 10


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=2)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--seconds', type=float, default=60.0)
    # reads per launch: over the driver's 20 sustained steps 96 beat 128 in 5 of 6 interleaved
    # comparisons (-0.5..-0.9% time, profiles/r02_s92_s93_batch_20step.txt); in 2-step runs
    # 128 had measured +1% (tools/batch_ab2.sh), before the clock settles
    ap.add_argument('--batch', type=int, default=96)
    ap.add_argument('--fmt', type=int, default=0, help='capture format: 0 u8, 1 s16, 2 .r30, 3 .lds (10-bit packed)')
    ap.add_argument('--clv', action='store_true',
                    help='CLV timecode instead of CAV picture numbers (captures past 79,999 frames, e.g. 1 h: config C5)')
    ap.add_argument('--cpu-seconds', type=float, default=1.0, help='oracle baseline sample (seconds of RF)')
    ap.add_argument('--no-cpu', action='store_true')
    ap.add_argument('--no-comb', action='store_true', help='stop at .tbc (skip the 2D comb stage)')
    ap.add_argument('--host-io', action='store_true',
                    help='PCIe-inclusive (not the headline): each step hands the capture over from host memory '
                         '(ldg_set_capture) and returns the .tbc frames, audio and rgb48 to host buffers, '
                         "as lddecode.py's file path does minus the disk (u8 only)")
    ap.add_argument('--prof-all', action='store_true',
                    help='HIP-event timing of every kernel (default: the demod only, the roofline kernel)')
    return ap.parse_args()


def cpu_baseline(seconds):
    """Oracle (numpy restatement of lddecode_core.py) on a bounded sample, one core."""
    from threadpoolctl import threadpool_limits
    from ldgpu.synth import make_capture
    from oracle.capture import FMT_U8
    from oracle.framer import decode_capture
    data = make_capture(int(40e6 * seconds), 'u8', seed=99)
    # the oracle prints the reference's log lines ('not valid', ...): to stderr, so
    # the JSON line stays the only stdout output
    with threadpool_limits(limits=1), contextlib.redirect_stdout(sys.stderr):
        t0 = time.perf_counter()
        frames, pcm, meta = decode_capture(data, FMT_U8)
        dt = time.perf_counter() - t0
    consumed = meta[-1]['nextsample'] if meta else 0
    return {'value': consumed / dt / 1e6, 'unit': 'RF Msamples/s', 'cores': 1, 'kind': 'port',
            'sample': '%.2f s synthetic NTSC CAV u8 RF -> %d frames through the oracle (numpy restatement of '
                      'lddecode_core.py), %.1f s wall on 1 core' % (seconds, len(frames), dt),
            'fields_per_s': 2 * len(frames) / dt}


def progress(rank, what):
    """a heartbeat on stderr (the JSON line stays the only stdout output)"""
    print('[bench rank %d] %s' % (rank, what), file=sys.stderr, flush=True)


def main():
    args = parse()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        ndev = torch.cuda.device_count()
        # one rank per GPU over RCCL; more ranks than GPUs (a rehearsal on a smaller
        # box) share devices and exchange the timing scalars over gloo
        use_nccl = ndev >= world
        local = local % max(ndev, 1)
        torch.cuda.set_device(local)
        tdist.init_process_group('nccl' if use_nccl else 'gloo')
        dist = tdist

    from ldgpu.decoder import GPUDecoder
    dec = GPUDecoder(system='NTSC', device=local, batch=args.batch)
    nsamp = int(40e6 * args.seconds)
    t0 = time.perf_counter()
    # per-rank capture: its own CAV picture-number range and noise seed
    dec.ctx.synth(nsamp, fmt=args.fmt, first_frame=1 + 2000 * (rank % 39), clv=args.clv, seed=20181015 + rank)
    dec.use_resident_capture(args.fmt, nsamp)
    synth_s = time.perf_counter() - t0
    progress(rank, 'capture synthesised (%.1f s)' % synth_s)

    host_cap = None
    if args.host_io:
        if args.fmt != 0:
            raise SystemExit('--host-io: u8 captures only')
        host_cap = dec.ctx.capture_download(0, nsamp)  # the capture in host memory, as a loader would hold it

    def step():
        if host_cap is not None:
            dec.set_capture(host_cap, args.fmt)         # H2D of the whole capture inside the step
            return dec.decode(sink=lambda fr, au, meta: None, comb=not args.no_comb, comb_sink=lambda rgb: None)
        dec.use_resident_capture(args.fmt, nsamp)      # fresh read cache: no reuse across steps
        return dec.decode(sink=None, comb=not args.no_comb)

    for w in range(args.warmup):
        nfr = step()
        progress(rank, 'warm-up step %d done' % (w + 1))

    def barrier():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    dec.ctx.profile(True if args.prof_all else 'demod')
    reads0 = dec.stats['reads']
    barrier()
    t0 = time.perf_counter()
    frames = 0
    consumed = 0
    for k in range(args.steps):
        frames += step()
        consumed += dec.last_meta['nextsample']
        progress(rank, 'step %d done' % (k + 1))
    barrier()
    dt = time.perf_counter() - t0
    stats = dec.ctx.profile_stats()
    if dec.htrace is not None:                 # LDG_HOSTTRACE=<file>: the host timeline of the timed steps
        with open(os.environ['LDG_HOSTTRACE'], 'w') as f:
            for t, ev, n in dec.htrace:
                if t >= t0:
                    f.write('%.4f %s %d\n' % ((t - t0) * 1e3, ev, n))
    spans = dec.ctx.profile_spans()        # (launches, total ms) of the demod's execution spans
    busy = dec.ctx.profile_spans_union()   # (launches, ms with at least one demod executing)
    dec.ctx.profile(False)
    # the roofline leg: the demod alone (kernel ldg_k_demod_iso) over one full-width launch's
    # reads, ISO_ITERS launches back to back, HIP events on its stream -- the per-dispatch
    # figure a kernel trace of this command reports for ldg_k_demod_iso (profiles/)
    iso_reads, iso_ms = dec.demod_isolated(ISO_ITERS)
    reads_timed = dec.stats['reads'] - reads0
    # sanity on the full-size output: consecutive CAV picture numbers, all frames present
    nrs = dec.frame_numbers
    consecutive = all(b == a + 1 for a, b in zip(nrs, nrs[1:]))

    if dist is not None:
        import torch
        t = torch.tensor([dt, float(frames), float(consumed)], dtype=torch.float64,
                         device='cuda' if tdist.get_backend() == 'nccl' else 'cpu')
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        dt_max, frames_all, consumed_all = float(tmax[0]), float(t[1]), float(t[2])
    else:
        dt_max, frames_all, consumed_all = dt, float(frames), float(consumed)

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    disc = 'CLV' if args.clv else 'CAV'
    msps = consumed_all / dt_max / 1e6
    fields_s = 2 * frames_all / dt_max
    # Roofline of the dominant kernel, the demod (the one kernel that consumes the capture and
    # fills the chip: one 150 KiB-LDS workgroup per CU).  Unit of work = one RF sample consumed;
    # algorithmic bytes per unit = SURVEY §8(d): input (1 B u8, 5/4 .lds, 4/3 .r30, 2 s16) +
    # .tbc out 955,500 / 1,334,667 B + .pcm 0.0048 B (1.7207 B for u8).  One launch of the
    # roofline leg demodulates `iso_reads` field reads; a read yields consumed / reads_decoded
    # new samples of the capture (reads overlap by ~1/3 and a few are speculative), so
    # units per launch = iso_reads * consumed / reads_decoded over the timed steps.
    bps = BYTES_PER_SAMPLE[args.fmt] + NTSC_TBC_BYTES_PER_SAMPLE + NTSC_PCM_BYTES_PER_SAMPLE
    samples_per_read = consumed / max(reads_timed, 1)
    units_iso = iso_reads * samples_per_read
    achieved = bps * units_iso / (iso_ms * 1e-3) / 1e9
    traffic, lds = None, None
    pmc = os.path.join(ROOT, 'profiles', 'pmc_traffic.json')
    if os.path.exists(pmc):
        try:
            pj = json.load(open(pmc))
            traffic = pj['kernels'].get('demod_iso')
            lds = pj.get('demod_iso_sq')
        except Exception:
            traffic = None
    # the pipeline's own demod launches (co-running with the field kernels, two demod streams
    # overlapping consecutive launches): in-kernel execution spans and HIP-event intervals
    dom_launches, dom_ms = stats.get('demod', (1, float('nan')))
    event_ms = dom_ms / max(dom_launches, 1)
    span_ms = spans[1] / spans[0] if spans[0] else float('nan')
    busy_ms = busy[1] / busy[0] if busy[0] else float('nan')
    units_pipe = consumed / max(dom_launches, 1)
    # secondary bound of the demod: FP64 vector issue (FFT-convention flops 5 N log2 N:
    # 6 x 8192-point + 2 x 1024-point complex FFTs per block, READ_BLOCKS blocks per read)
    iso_flops = iso_reads * READ_BLOCKS * DEMOD_FLOPS_PER_BLOCK
    fp64 = {'achieved_tflops': round(iso_flops / (iso_ms * 1e-3) / 1e12, 3), 'peak_tflops': FP64_PEAK_TFLOPS,
            'frac': iso_flops / (iso_ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
            'flops_per_block': DEMOD_FLOPS_PER_BLOCK, 'blocks_per_launch': iso_reads * READ_BLOCKS}
    roofline = {
        'bound': 'hbm', 'kernel': 'demod', 'achieved': round(achieved, 4), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
        'frac': achieved / HBM_PEAK_GBS, 'traffic': traffic,
        'avg_launch_ms': round(iso_ms, 4),
        'timing': ('isolated leg: %d launches of ldg_k_demod_iso over %d field reads (%d blocks) back to back, '
                   'HIP events on its stream; the kernel trace in profiles/ reports ldg_k_demod_iso per dispatch'
                   % (ISO_ITERS, iso_reads, iso_reads * READ_BLOCKS)),
        'units_per_launch': round(units_iso), 'algorithmic_bytes_per_sample': round(bps, 4),
        'algorithmic_bytes_per_launch': round(bps * units_iso),
        'traffic_unit': 'bytes per launch, 2*FETCH_SIZE + WRITE_SIZE (profiles/pmc_traffic.json, demod_iso)',
        'traffic_x_algorithmic': (traffic / (bps * units_iso)) if traffic else None,
        'lds': lds, 'fp64': fp64,
        'pipeline': {'launches': dom_launches, 'span_ms': round(span_ms, 4), 'hip_event_ms': round(event_ms, 4),
                     'busy_ms_per_launch': round(busy_ms, 4), 'units_per_launch': round(units_pipe),
                     'achieved_busy': round(bps * units_pipe / (busy_ms * 1e-3) / 1e9, 4),
                     'demod_streams': int(os.environ.get('LDG_DEMOD_STREAMS', '2')),
                     'note': 'the timed steps\' demod launches: in-kernel execution span (device clock), HIP-event '
                             'interval, and the union of the spans per launch (two demod streams overlap '
                             'consecutive launches; field kernels co-run on the CUs)'},
    }
    if not args.no_comb:
        roofline['bytes_per_sample_with_comb'] = round(bps + NTSC_COMB_BYTES_PER_SAMPLE, 4)
    cpu = None if args.no_cpu else cpu_baseline(args.cpu_seconds)
    line = {
        'metric': 'RF Msamples/s (40 MSPS NTSC, full RF->.tbc decode)', 'value': round(msps, 3),
        'unit': 'RF Msamples/s', 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
        'ms_per_step': round(dt_max / args.steps * 1e3, 3), 'higher_is_better': True, 'scaling': 'weak',
        'vs_baseline': None, 'dtype': 'f64',
        'data': 'synthetic (GPU-synthesised NTSC %s RF, %s)' % (disc, FMT_NAME[args.fmt]),
        'config': {'workload': '%g s NTSC %s, 40 MSPS %s RF per GPU: RF->demod->TBC->.tbc+.pcm%s'
                               % (args.seconds, disc, FMT_NAME[args.fmt], '' if args.no_comb else '->2D comb rgb48'),
                   'frames_per_step': frames // max(args.steps, 1), 'batch_reads': args.batch,
                   'parallelism': 'capture-sharded x%d' % world,
                   'io': 'host buffers over PCIe (--host-io)' if args.host_io else 'HBM-resident'},
        'fields_per_s': round(fields_s, 1), 'realtime_x': round(msps / 40.0, 2),
        'roofline': roofline,
        'kernels_ms': {k: round(v[1], 3) for k, v in sorted(stats.items(), key=lambda kv: -kv[1][1])},
        'cpu_baseline': cpu,
        'checks': {'framenr_consecutive': consecutive, 'synth_s': round(synth_s, 2),
                   'reads_decoded': dec.stats['reads'], 'reads_used': dec.stats['reads_used'],
                   'batches': dec.stats['batches'], 'misses': dec.stats.get('misses', 0),
                   'drain_waits': dec.stats.get('drain_waits', 0),
                   'host_s': {k: round(dec.stats.get(k, 0.0), 4) for k in ('plan_s', 'gpu_s', 'replay_s', 'flush_s', 'wait_s')},
                   'miss_sample': dec.stats.get('miss_log', [])[:12],
                   'inflight_at_wait': dec.stats.get('inflight_at_wait')},
    }
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
