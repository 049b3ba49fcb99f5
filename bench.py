"""Benchmark: RF Msamples/s and fields/s of the MI355X decode path (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W]
    (N > 1: torch.distributed.run, one rank per GPU: one capture field-sharded, strong scaling)

N = 1 (default; BASELINE.json configs[1]): 60 s of synthetic NTSC CAV RF,
40 MSPS, 8-bit, synthesised on the GPU straight into HBM (same signal model as
ldgpu/synth.py).  One step = the full reference decode of that capture:
RF -> demod -> TBC -> .tbc frames (+ .pcm audio) -> 2D comb, every frame of the
60 s, with the frames assembled in HBM.

N > 1 (default under torch.distributed.run; BASELINE.json configs[4], or
--sharded at any N): ONE 1-hour 40 MSPS NTSC CLV capture field-sharded across
the ranks (ldgpu/shard.py, as lddecode.py runs it): each rank holds its window
of the capture in HBM, and one step = the RCCL halo exchange of the window
tails (batch_isend_irecv between the GPUs' capture buffers), the rank's
decode, the summary all_gather and chain check, and the exact audio of its
frames -- strong scaling of a fixed capture.  --independent instead gives
every rank its own 60 s capture (weak scaling, no data-path collective).
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
PAL_TBC_BYTES_PER_SAMPLE = 1418750 / 1600000        # 1135 x 625 uint16 per 1.6 M samples
PAL_COMB_BYTES_PER_SAMPLE = (1418750 + 1057 * 576 * 3 * 2) / 1600000
BYTES_PER_SAMPLE = {0: 1.0, 1: 2.0, 2: 4 / 3, 3: 1.25}
FMT_NAME = {0: 'u8', 1: 's16', 2: '10-bit .r30', 3: '10-bit .lds'}
HBM_PEAK_GBS = 8000.0
FP64_PEAK_TFLOPS = 78.6                           # MI355X FP64 vector (spec)
READ_BLOCKS = 66                                  # overlap-save blocks per 1e6-sample field read
ISO_ITERS = 20                                    # launches of the isolated roofline leg
ISO_READS = 96                                    # reads per isolated launch (rounds 1-5 quote 96-read launches)
# the leg's kernels: ldg_k_demod_iso (full blocks) and ldg_k_demod_iso_cut (the shipped body);
ISO_VARIANTS = (0, 1)


def iso_leg(dec):
    """(reads, full-body ms, shipped-body ms or None) of the isolated roofline leg"""
    reads, ms = dec.demod_isolated(ISO_ITERS, ISO_VARIANTS, reads=ISO_READS)
    return (reads, ms, None) if len(ISO_VARIANTS) == 1 else (reads, ms[0], ms[1])
# the FFT flops the demod executes per block (5 N log2 N): six 8192-point complex transforms
# (raw R2C, analytic even / odd, demod R2C, C2R 0.5 MHz, C2R video) + two 1024-point audio IFFTs;
# sync / burst / pilot are time-domain recurrences (iir.hpp) and are not counted
DEMOD_FLOPS_PER_BLOCK = 6 * 5 * 8192 * 13 + 2 * 5 * 1024 * 10


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=2)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--seconds', type=float, default=None,
                    help='capture length (default 60 s; 3600 s for the sharded config-5 leg)')
    ap.add_argument('--sharded', action='store_true',
                    help='config 5: one 1 h NTSC CLV capture field-sharded across the ranks (default when N > 1)')
    ap.add_argument('--independent', action='store_true',
                    help='N > 1: each rank decodes its own capture (weak scaling) instead of the sharded config 5')
    # reads per launch: 128 since round 5 (probes): PAL +1.6% in 5 of 5 interleaved pairs, NTSC
    # level at 20 steps and +0.6% at 2 (profiles/r05_zs_batch.txt, r05_zt_batch.txt); round 2 had
    # 96 ahead by 0.5-0.9% (profiles/r02_s92_s93_batch_20step.txt), before the planner's hints
    ap.add_argument('--batch', type=int, default=128)
    ap.add_argument('--fmt', type=int, default=0, help='capture format: 0 u8, 1 s16, 2 .r30, 3 .lds (10-bit packed)')
    ap.add_argument('--system', default='NTSC', choices=('NTSC', 'PAL'),
                    help='PAL: config 3 (PAL CLV 40 MSPS u8, host-synthesised, the PAL Y/C decoder)')
    ap.add_argument('--clv', action='store_true',
                    help='CLV timecode instead of CAV picture numbers (captures past 79,999 frames, e.g. 1 h: config C5)')
    ap.add_argument('--cpu-frames', type=int, default=60,
                    help='oracle baseline sample: frames per process (SURVEY §8(d): a 60-frame prefix)')
    ap.add_argument('--cpu-procs', type=int, default=0,
                    help='processes of the multi-process CPU baseline (default: the CPUs visible, at most 16)')
    ap.add_argument('--no-cpu', action='store_true')
    ap.add_argument('--no-comb', action='store_true', help='stop at .tbc (skip the 2D comb stage)')
    ap.add_argument('--host-io', action='store_true',
                    help='PCIe-inclusive (not the headline): each step hands the capture over from host memory '
                         '(ldg_set_capture) and returns the .tbc frames, audio and rgb48 to host buffers, '
                         "as lddecode.py's file path does minus the disk (u8 only)")
    ap.add_argument('--stream-file', default=None,
                    help='not the headline: the capture is written to this file once, and each step streams it '
                         'from there through the HBM ring (ldg_stream_open, 2 GiB; lddecode.py\'s path minus the '
                         'output writes), frames and rgb48 left in HBM; NTSC, one rank or --independent')
    ap.add_argument('--prof-all', action='store_true',
                    help='HIP-event timing of every kernel (default: the demod only, the roofline kernel)')
    args = ap.parse_args()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    if (args.stream_file or args.host_io) and (args.system == 'PAL' or args.sharded or
                                               (world > 1 and not args.independent)):
        ap.error('--stream-file / --host-io: the NTSC capture workload (one rank, or --independent)')
    return args


def _oracle_decode(data, fmt=0, system='NTSC', frames=None):
    """One oracle decode (the numpy restatement of lddecode.py / lddecode_core.py), one core,
    of the first `frames` frames (lddecode.py -l); returns (RF samples consumed, frames, seconds)."""
    from threadpoolctl import threadpool_limits
    from oracle.framer import decode_capture
    # the oracle prints the reference's log lines ('not valid', ...): to stderr, so
    # the JSON line stays the only stdout output
    with threadpool_limits(limits=1), contextlib.redirect_stdout(sys.stderr):
        t0 = time.perf_counter()
        out, pcm, meta = decode_capture(bytes(data), fmt, system=system, length=frames)
        dt = time.perf_counter() - t0
    first = meta[0]['fields'][0]['readsample'] if meta else 0
    return ((meta[-1]['nextsample'] - first) if meta else 0), len(out), dt


SLICE_SHIFT = 170004          # about a quarter field of 40 MSPS RF (a multiple of 12: whole packing groups)


def bytes_for_samples_(fmt, n):
    from ldgpu.formats import bytes_for_samples
    return bytes_for_samples(fmt, n)


def _sample_bytes(fmt, n):
    """Bytes of n samples (n a multiple of 12) in a capture format."""
    return {0: n, 1: 2 * n, 2: n // 3 * 4, 3: n // 4 * 5}[fmt]


def _oracle_worker(args):
    """One slice of mode (ii).  A slice that starts inside a vertical sync stops the oracle
    as it stops the reference (vsync within the first 11 peaks, oracle/field.py); such a slice
    starts a quarter field later instead, as a sharded CPU runner would place its starts."""
    from oracle.demod import ReferenceCrash
    path, off, nbytes, fmt, system, frames = args
    with open(path, 'rb') as fh:
        for j in range(4):
            fh.seek(off + _sample_bytes(fmt, j * SLICE_SHIFT))
            try:
                return _oracle_decode(fh.read(nbytes), fmt, system, frames)
            except ReferenceCrash:
                if j == 3:
                    raise


def cpu_model():
    try:
        for line in open('/proc/cpuinfo'):
            if line.startswith('model name'):
                return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return 'unknown'


def cpu_sample_samples(system, frames):
    """RF samples a `frames`-frame oracle decode needs: the 10-bit EOF guard
    (lddecode.py:42,89) stops a capture of B bytes after ~B / (spf * 5 / 4) frames,
    so the sample holds frames + 2 of those (a multiple of 12)."""
    spf = 1600001 if system == 'PAL' else 1334668
    return -(-((frames + 2) * (spf * 5 // 4)) // 12) * 12


def cpu_baseline(get_capture, fmt, system, frames, procs):
    """The oracle on this box's host cores: (i) one process on
    one core, the reference's own execution model (numpy FFT single-threaded), over the first
    `frames` frames of the benchmark's capture (lddecode.py -l frames); (ii) `procs`
    processes at once, one core each, each over `frames` frames of its own slice of the same
    capture (field-group sharding of the CPU path).  Bounded samples, not the whole capture
    (about 16 s of CPU per second of RF).  get_capture(nbytes) -> the capture's first bytes."""
    import multiprocessing as mp
    import tempfile
    n = cpu_sample_samples(system, frames)
    nb = _sample_bytes(fmt, n)
    consumed, nfr, dt = _oracle_decode(get_capture(nb), fmt, system, frames)
    fname = {0: 'u8', 1: 's16', 2: '10-bit .r30', 3: '10-bit .lds'}[fmt]
    out = {'value': consumed / dt / 1e6, 'unit': 'RF Msamples/s', 'cores': 1, 'kind': 'port',
           'cpu_model': cpu_model(), 'host_cpus_visible': len(os.sched_getaffinity(0)),
           'sample': ('the first %d frames of the benchmark capture (synthetic %s %s RF, lddecode.py -l %d) through '
                      'the oracle (numpy restatement of lddecode_core.py:373-427,1193-1311), %.1f s wall on 1 core'
                      % (nfr, system, fname, frames, dt)),
           'fields_per_s': 2 * nfr / dt}
    total = _sample_bytes(fmt, procs * n + 3 * SLICE_SHIFT)
    if procs > 1:
        cap = get_capture(total)
        stride, note = n, ''
        if cap is not None and len(cap) < total:
            # a capture shorter than procs slices (config 3's 10 s PAL): the slices overlap,
            # each still its own 60-frame decode from its own start
            from ldgpu.formats import samples_in_bytes
            stride = (samples_in_bytes(fmt, len(cap)) - n - 3 * SLICE_SHIFT) // (procs - 1) // 12 * 12
            note = ', overlapping (starts %d samples apart)' % stride
            total = _sample_bytes(fmt, (procs - 1) * stride + n + 3 * SLICE_SHIFT)
        if cap is not None and len(cap) >= total and stride >= SLICE_SHIFT:
            with tempfile.NamedTemporaryFile(prefix='ldg_cpu_') as fh:
                fh.write(bytes(cap[:total]))
                fh.flush()
                ctx = mp.get_context('spawn')       # no inherited HIP state in the workers
                t0 = time.perf_counter()
                with ctx.Pool(procs) as pool:
                    res = pool.map(_oracle_worker, [(fh.name, _sample_bytes(fmt, k * stride), nb, fmt, system, frames)
                                                    for k in range(procs)])
                wall = time.perf_counter() - t0
            tot = sum(r[0] for r in res)
            out['multi_process'] = {'value': tot / wall / 1e6, 'unit': 'RF Msamples/s', 'processes': procs,
                                    'cores': procs, 'fields_per_s': 2 * sum(r[1] for r in res) / wall,
                                    'process_cap': ('min(16, CPUs visible): the GPU box allots each GPU a 16-CPU share '
                                                    '(os.cpu_count() there shows the whole host, %d CPUs); '
                                                    '--cpu-procs N overrides' % len(os.sched_getaffinity(0))),
                                    'sample': '%d slices of the benchmark capture%s, %d frames each, one process '
                                              '(one core) each, %.1f s wall' % (procs, note, frames, wall)}
    return out


LDS_PEAK_TBS = 150.0          # ds_read_b64/b128 with every CU streaming (MI355X_MICROARCH.md, LDS)


def bound_analysis(sq, traffic, iso_ms, name='demod_iso_sq'):
    """Which resource the demod sits against, from the committed PMC passes over the same
    isolated leg (profiles/pmc_traffic.json, tools/pmc_summary.py) and this run's launch time:
    HBM (PMC bytes / time), LDS (ds bytes / time against ~150 TB/s, and LDS-array busy
    cycles), VALU issue (wave64 VALU instructions x 4 cycles over the SIMDs' cycles) and
    the share of wave time parked at s_waitcnt / barriers."""
    if not sq:
        return None
    c, d = sq['per_launch'], sq['derived']
    out = {'valu_issue_frac': d.get('valu_issue_frac'), 'fp64_share_of_valu_insts': d.get('fp64_share_of_valu_insts'),
           'lds_array_busy_frac': d.get('lds_array_busy_frac'),
           'wave_time': {'issuing': d.get('active_inst_any_per_wave_cycle'),
                         'parked_waitcnt_barrier': d.get('wait_any_per_wave_cycle'),
                         'issue_stalled': d.get('wait_inst_any_per_wave_cycle')}}
    if traffic:
        out['hbm_tbs'] = traffic / (iso_ms * 1e-3) / 1e12
        out['hbm_frac'] = out['hbm_tbs'] / (HBM_PEAK_GBS / 1e3)
    if d.get('lds_bytes'):
        out['lds_bytes_per_launch'] = d['lds_bytes']
        out['lds_tbs'] = d['lds_bytes'] / (iso_ms * 1e-3) / 1e12
        out['lds_frac'] = out['lds_tbs'] / LDS_PEAK_TBS
    out['source'] = 'profiles/pmc_traffic.json %s (rocprofv3 --pmc passes over this bench\'s isolated leg)' % name
    return out


def demod_issue_lag(tab):
    """Was the host on the demod's critical path?  tab: the timed steps' demod launches in
    issue order (start, end, host issue; ms on the device clock, ldg_profile_span_table).
    For each launch after the first, against the latest end of the launches issued before
    it: gap = its start - that end (> 0: no demod was executing, the demod pipeline ran
    dry) and late = its host issue - that end (> 0: the host had not issued it yet).  A
    launch is host-late when both are positive: the GPU waited on the host."""
    ok = ~np.isnan(tab[:, 0]) if len(tab) else np.zeros(0, bool)
    tab = tab[ok]
    if len(tab) < 2:
        return None
    prev_end = np.maximum.accumulate(tab[:-1, 1])
    gap = tab[1:, 0] - prev_end
    late = tab[1:, 2] - prev_end
    idle = gap > 0.005
    hl = idle & (late > 0)
    return {'launches': int(len(gap)), 'idle_gaps': int(idle.sum()), 'host_late': int(hl.sum()),
            'host_late_frac': round(float(hl.mean()), 4), 'idle_ms': round(float(gap[idle].sum()), 3),
            'host_late_ms': round(float(np.minimum(gap, late)[hl].sum()), 3),
            'median_gap_ms': round(float(np.median(gap)), 4),
            'note': 'timed steps\' demod launches, issue order; gap = start - latest earlier end, late = host issue '
                    '(steady clock mapped onto the device clock) - that end; host-late: gap > 5 us and late > 0'}


def progress(rank, what):
    """a heartbeat on stderr (the JSON line stays the only stdout output)"""
    print('[bench rank %d] %s' % (rank, what), file=sys.stderr, flush=True)


class CaptureWorkload:
    """configs[1] (and --independent N > 1): each rank decodes its own capture, 60 s of NTSC
    (CAV by default) synthesised straight into HBM.  Weak scaling, no data-path collective."""

    def __init__(self, args, dec, rank):
        self.args, self.dec, self.rank = args, dec, rank
        self.nsamp = int(40e6 * (args.seconds or 60.0))
        t0 = time.perf_counter()
        # per-rank capture: its own CAV picture-number range and noise seed
        dec.ctx.synth(self.nsamp, fmt=args.fmt, first_frame=1 + 2000 * (rank % 39), clv=args.clv,
                      seed=20181015 + rank)
        dec.use_resident_capture(args.fmt, self.nsamp)
        self.synth_s = time.perf_counter() - t0
        self.host_cap = None
        self.stream_acc = {}
        # --stream-file: each rank streams its own file (--independent N > 1: path.<rank>)
        self.stream_path = None
        if args.stream_file:
            world = int(os.environ.get('WORLD_SIZE', '1'))
            self.stream_path = args.stream_file if world == 1 else '%s.%d' % (args.stream_file, rank)
            nbytes = bytes_for_samples_(args.fmt, self.nsamp)
            with open(self.stream_path, 'wb') as fh:
                for off in range(0, nbytes, 1 << 28):
                    fh.write(dec.ctx.capture_download(off, min(1 << 28, nbytes - off)))
        if args.host_io:
            if args.fmt != 0:
                raise SystemExit('--host-io: u8 captures only')
            self.host_cap = dec.ctx.capture_download(0, self.nsamp)   # as a loader would hold it
        self.scaling = 'weak'
        self.fmt, self.system = args.fmt, 'NTSC'
        self.data = 'synthetic (GPU-synthesised NTSC %s RF, %s)' % ('CLV' if args.clv else 'CAV', FMT_NAME[args.fmt])

    def step(self):
        dec, args = self.dec, self.args
        if args.stream_file:
            t0 = time.perf_counter()
            dec.open_stream(self.stream_path, args.fmt, 2 << 30)      # the file read inside the step
            t1 = time.perf_counter()
            n = dec.decode(sink=None, comb=not args.no_comb)
            st = dec.ctx.stream_stats()
            acc = self.stream_acc
            acc['open_s'] = acc.get('open_s', 0.0) + t1 - t0
            for k in ('read_s', 'launch_wait_s', 'space_wait_s', 'stage_wait_s', 'bytes_read', 'launch_waits'):
                acc[k] = acc.get(k, 0.0) + st[k]
            return n, dec.last_meta['nextsample']
        if self.host_cap is not None:
            dec.set_capture(self.host_cap, args.fmt)         # H2D of the whole capture inside the step
            n = dec.decode(sink=lambda fr, au, meta: None, comb=not args.no_comb, comb_sink=lambda rgb: None)
        else:
            dec.use_resident_capture(args.fmt, self.nsamp)   # fresh read cache: no reuse across steps
            n = dec.decode(sink=None, comb=not args.no_comb)
        return n, dec.last_meta['nextsample']

    def host_capture(self, nbytes):
        from ldgpu.formats import bytes_for_samples
        nbytes = min(nbytes, bytes_for_samples(self.fmt, self.nsamp))
        if self.stream_path:
            return np.fromfile(self.stream_path, dtype=np.uint8, count=nbytes)
        return self.host_cap[:nbytes] if self.host_cap is not None else \
            np.asarray(self.dec.ctx.capture_download(0, nbytes))

    def before_iso(self):
        """The roofline leg re-demodulates cached reads from a resident capture: after
        streamed steps, the capture is made resident again and a few frames decoded."""
        if self.args.stream_file:
            a = self.args
            self.dec.ctx.synth(self.nsamp, fmt=a.fmt, first_frame=1 + 2000 * (self.rank % 39), clv=a.clv,
                               seed=20181015 + self.rank)
            self.dec.use_resident_capture(a.fmt, self.nsamp)
            self.dec.decode(sink=None, comb=False, length=120)

    def config(self, frames):
        a = self.args
        return {'workload': '%g s NTSC %s, 40 MSPS %s RF per GPU: RF->demod->TBC->.tbc+.pcm%s'
                            % (a.seconds or 60.0, 'CLV' if a.clv else 'CAV', FMT_NAME[a.fmt],
                               '' if a.no_comb else '->2D comb rgb48'),
                'frames_per_step': frames // max(a.steps, 1), 'batch_reads': a.batch,
                'parallelism': 'capture-sharded x%d' % int(os.environ.get('WORLD_SIZE', '1')),
                'io': ('host buffers over PCIe (--host-io)' if a.host_io else
                       'streamed from a file through a 2 GiB HBM ring (--stream-file)' if a.stream_file else
                       'HBM-resident')}

    def checks(self):
        nrs = self.dec.frame_numbers       # consecutive picture numbers, all frames present
        ok = all(b == a + 1 for a, b in zip(nrs, nrs[1:]))
        out = {'framenr_consecutive': ok, 'cav_framenr_consecutive': ok}   # (the round-1 key, kept)
        if self.stream_acc:
            out['stream'] = {k: round(v, 4) for k, v in self.stream_acc.items()}
        return out


class ShardedWorkload:
    """configs[4]: ONE 40 MSPS NTSC CLV capture (1 h by default) field-sharded across the
    ranks exactly as lddecode.py runs it under torch.distributed.run (ldgpu/shard.py):
    rank k holds its window [lo_k, hi_k) of the capture in HBM -- its own part synthesised
    on its GPU (as if read from storage), the tail halo [cut_k, hi_k) received from rank k+1.
    One step: the halo exchange over RCCL (batch_isend_irecv between the GPUs' capture
    buffers), the rank's decode (frames and the fused 2D comb in HBM, audio inputs archived),
    the summary all_gather and chain check, and the exact 48 kHz audio of its frames.
    Strong scaling: the capture is fixed, each rank gets 1/N of it.  The comb's burst-level
    EMA starts uninitialised on every rank here (lddecode.py's sharded --comb hands the exact
    state over after the exchange: tests/test_cli.py::test_cli_sharded_two_ranks_equal_single)."""

    def __init__(self, args, dec, rank, world, dist):
        import torch
        from ldgpu.shard import decode_bounds, shard_windows
        self.args, self.dec, self.rank, self.world, self.dist = args, dec, rank, world, dist
        self.seconds = args.seconds or 3600.0
        self.total = int(40e6 * self.seconds)
        spf = dec.rf.samples_per_frame
        w = shard_windows(decode_bounds(self.total, self.total, spf, world)[0], spf, self.total)
        # The synthetic "storage": rank k's stored part ends where rank k+1's begins, so each
        # sample of the capture is synthesised by exactly one rank and every rank sees the
        # same bytes (a window synthesised on its own starts its carrier phase and noise
        # afresh); the rest of the window, [lo_{k+1}, hi_k), comes over the halo exchange.
        self.windows = [(lo, w[k + 1][0] if k + 1 < world else cut, hi) for k, (lo, cut, hi) in enumerate(w)]
        lo, cut, hi = self.windows[rank]
        t0 = time.perf_counter()
        dec.ctx.synth(cut - lo if world > 1 else hi - lo, fmt=0, first_frame=1, clv=True, seed=20181015,
                      start_sample=lo)
        self.buf = None
        # RCCL moves the halo between the GPUs' capture buffers; a rehearsal with more
        # ranks than GPUs (gloo) moves it through host memory instead
        self.on_device = dist is not None and dist.get_backend() == 'nccl'
        if world > 1 and self.on_device:
            # the window in a torch CUDA tensor (RCCL sends / receives its tail in place)
            self.buf = torch.empty(hi - lo, dtype=torch.uint8, device='cuda')
            dec.ctx.capture_copy_to_device(self.buf.data_ptr(), 0, cut - lo)
            torch.cuda.synchronize()
        elif world > 1:
            self.buf = torch.zeros(hi - lo, dtype=torch.uint8)
            self.buf[:cut - lo] = torch.from_numpy(dec.ctx.capture_download(0, cut - lo))
        self.synth_s = time.perf_counter() - t0
        self.stats = {}
        self.scaling = 'strong'
        self.fmt, self.system = 0, 'NTSC'
        self.data = 'synthetic (GPU-synthesised NTSC CLV RF, u8; each rank its window of one capture)'
        self.halo_rccl = False

    def _allgather(self, obj):
        if self.world == 1:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def step(self):
        from ldgpu.shard import decode_sharded, exchange_halo, torch_p2p
        dec, lo, hi = self.dec, self.windows[self.rank][0], self.windows[self.rank][2]
        if self.buf is not None and self.on_device:
            import torch
            self.halo_rccl = exchange_halo(self.buf, self.rank, self.windows, 0, torch_p2p) or self.halo_rccl
            torch.cuda.synchronize()
            dec.set_capture(None, 0, device_ptr=self.buf.data_ptr(), nsamples=hi - lo, first_sample=lo,
                            total_bytes=self.total)
        elif self.buf is not None:
            exchange_halo(self.buf, self.rank, self.windows, 0, torch_p2p)
            dec.set_capture(self.buf.numpy(), 0, nsamples=hi - lo, first_sample=lo, total_bytes=self.total)
        else:
            dec.use_resident_capture(0, self.total)
        res = decode_sharded(dec, self.rank, self.world, self._allgather, resident=True,
                             comb=not self.args.no_comb, stats=self.stats)
        if not res:
            return 0, 0
        first = res[0][3]['fields'][0]['readsample']
        return len(res), res[-1][3]['nextsample'] - first

    def host_capture(self, nbytes):
        if self.buf is not None:
            return self.buf[:nbytes].cpu().numpy()
        return self.dec.ctx.capture_download(0, nbytes)

    def config(self, frames):
        a = self.args
        return {'workload': 'config 5: %g s NTSC CLV, 40 MSPS u8 RF, ONE capture field-sharded across %d GPU(s) '
                            '(1/%d each, HBM-resident windows, RCCL halo exchange): RF->demod->TBC->.tbc+.pcm%s'
                            % (self.seconds, self.world, self.world, '' if a.no_comb else '->2D comb rgb48'),
                'frames_per_step_rank0': frames // max(a.steps, 1), 'batch_reads': a.batch,
                'parallelism': 'field-group sharded x%d' % self.world, 'io': 'HBM-resident',
                'comb_state': 'each rank combs from an uninitialised burst-level EMA; lddecode.py re-combs the '
                              'first frame(s) from the exact state after the exchange (shard.comb_fix), '
                              'not timed here'}

    def same_share_single(self, steps=2):
        """Rank 0's share of the capture decoded by this GPU alone (no exchange, the other
        ranks idle), in the same session: the N = 1 rate of the per-rank work, beside the
        N-rank line (config 5's scaling then has a baseline on its own workload).
        Returns (RF Msamples/s, ms per step, frames per step)."""
        dec, lo, cut = self.dec, self.windows[self.rank][0], self.windows[self.rank][1]
        if self.buf is not None and self.on_device:
            dec.set_capture(None, 0, device_ptr=self.buf.data_ptr(), nsamples=self.windows[self.rank][2] - lo,
                            first_sample=lo, total_bytes=self.total)
        elif self.buf is not None:
            dec.set_capture(self.buf.numpy(), 0, nsamples=self.windows[self.rank][2] - lo, first_sample=lo,
                            total_bytes=self.total)
        else:
            dec.use_resident_capture(0, self.total)
        out = []
        for k in range(steps + 1):
            dec._reset_cache()
            t0 = time.perf_counter()
            n = dec.decode(sink=None, comb=not self.args.no_comb, start_sample=lo, stop_sample=cut,
                           firstframe=lo == 0)
            dt = time.perf_counter() - t0
            if k:                                   # the first pass warms up
                out.append((dec.last_meta['nextsample'] - lo if dec.last_meta else 0, dt, n))
        ns = sum(o[0] for o in out)
        dt = sum(o[1] for o in out)
        return ns / dt / 1e6, dt / len(out) * 1e3, out[-1][2]

    def checks(self):
        return {'frames_per_step_all_ranks': self.stats.get('frames_total'),
                'chain_refixes': self.stats.get('refixes', 0), 'window_misses': self.stats.get('window_misses', 0),
                'halo_over_rccl': bool(self.halo_rccl),
                'phase_s': {k: round(self.stats.get(k, 0.0), 4) for k in ('local_s', 'exchange_s', 'finish_s')}}


class PALWorkload:
    """configs[2]: PAL CLV, 40 MSPS u8 (10 s by default), synthesised on the
    host (ldgpu/synth.py: PAL timing, 3.75 MHz pilot, CLV timecode) and made resident in HBM
    before the timed region; one step decodes all of it RF -> .tbc + .pcm -> the PAL Y/C
    decoder's rgb48 (row F2, build-defined), frames and rgb48 left in HBM."""

    def __init__(self, args, dec, rank):
        from ldgpu.synth import make_capture
        self.args, self.dec = args, dec
        self.nsamp = int(40e6 * (args.seconds or 10.0))
        t0 = time.perf_counter()
        seed = 20181018 + rank
        # LDG_SYNTH_CACHE=<dir>: keep the host-synthesised capture between runs of a sweep
        cache = os.environ.get('LDG_SYNTH_CACHE')
        path = os.path.join(cache, 'pal_clv_u8_%d_%d.raw' % (self.nsamp, seed)) if cache else None
        if path and os.path.exists(path):
            self.raw = np.fromfile(path, dtype=np.uint8)
        else:
            import threading
            done = threading.Event()

            def beat():                          # the host synthesis is slow: heartbeats on stderr
                while not done.wait(30.0):
                    progress(rank, 'synthesising PAL capture (%.0f s)' % (time.perf_counter() - t0))
            threading.Thread(target=beat, daemon=True).start()
            try:
                self.raw = np.frombuffer(make_capture(self.nsamp, 'u8', system='PAL', clv=True, first_frame=3000,
                                                      seed=seed), np.uint8)
            finally:
                done.set()
            if path:
                os.makedirs(cache, exist_ok=True)
                self.raw.tofile(path)
        dec.set_capture(self.raw, 0)
        self.synth_s = time.perf_counter() - t0
        self.scaling, self.fmt, self.system = 'weak', 0, 'PAL'
        self.data = 'synthetic (host-synthesised PAL CLV RF, u8, 3.75 MHz pilot)'

    def step(self):
        dec = self.dec
        dec._reset_cache()                           # fresh read cache: no reuse across steps
        n = dec.decode(sink=None, comb=not self.args.no_comb)
        return n, dec.last_meta['nextsample']

    def host_capture(self, nbytes):
        return self.raw[:nbytes]

    def config(self, frames):
        a = self.args
        return {'workload': 'config 3: %g s PAL CLV, 40 MSPS u8 RF per GPU: RF->demod->TBC->.tbc+.pcm%s'
                            % (self.nsamp / 40e6, '' if a.no_comb else '->PAL Y/C rgb48 (build-defined, row F2)'),
                'frames_per_step': frames // max(a.steps, 1), 'batch_reads': a.batch, 'io': 'HBM-resident'}

    def checks(self):
        nrs = self.dec.frame_numbers
        return {'framenr_consecutive': all(b == a + 1 for a, b in zip(nrs, nrs[1:]))}


def main():
    args = parse()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    dist = None
    shared_device = False
    if world > 1:
        import torch
        import torch.distributed as tdist
        ndev = torch.cuda.device_count()
        # one rank per GPU over RCCL; more ranks than GPUs (a rehearsal on a smaller
        # box) share devices and exchange the timing scalars over gloo
        use_nccl = ndev >= world
        shared_device = not use_nccl
        local = local % max(ndev, 1)
        torch.cuda.set_device(local)
        tdist.init_process_group('nccl' if use_nccl else 'gloo')
        if use_nccl:
            # the RCCL communicator made by a collective every rank joins, before the halo's
            # batched send / receive (which only neighbouring ranks join)
            tdist.all_reduce(torch.zeros(1, device='cuda'))
        dist = tdist

    from ldgpu.decoder import GPUDecoder
    dec = GPUDecoder(system=args.system, device=local, batch=args.batch)
    sharded = args.system == 'NTSC' and (args.sharded or (world > 1 and not args.independent))
    if args.system == 'PAL':
        wl = PALWorkload(args, dec, rank)
    else:
        wl = ShardedWorkload(args, dec, rank, world, dist) if sharded else CaptureWorkload(args, dec, rank)
    progress(rank, 'capture synthesised (%.1f s)' % wl.synth_s)

    for w in range(args.warmup):
        wl.step()
        progress(rank, 'warm-up step %d done' % (w + 1))

    def barrier():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    dec.ctx.profile(True if args.prof_all else 'demod')
    reads0, used0 = dec.stats['reads'], dec.stats['reads_used']
    barrier()
    t0 = time.perf_counter()
    frames = 0
    consumed = 0
    step_ms = []                               # per-step wall (each step's decode ends synchronised)
    for k in range(args.steps):
        ts = time.perf_counter()
        nf, ns = wl.step()
        step_ms.append(round((time.perf_counter() - ts) * 1e3, 2))
        frames += nf
        consumed += ns
        progress(rank, 'step %d done' % (k + 1))
    barrier()
    dt = time.perf_counter() - t0
    stats = dec.ctx.profile_stats()
    if dec.htrace is not None:                 # LDG_HOSTTRACE=<file>: the host timeline of the timed steps
        with open(os.environ['LDG_HOSTTRACE'], 'w') as f:
            f.write('# t0_ms %.4f (time.perf_counter() * 1e3 at the timed region\'s start)\n' % (t0 * 1e3))
            for t, ev, n in dec.htrace:
                if t >= t0:
                    f.write('%.4f %s %d\n' % ((t - t0) * 1e3, ev, n))
    spans = dec.ctx.profile_spans()        # (launches, total ms) of the demod's execution spans
    busy = dec.ctx.profile_spans_union()   # (launches, ms with at least one demod executing)
    span_tab = dec.ctx.profile_span_table()
    issue = demod_issue_lag(span_tab)
    if os.environ.get('LDG_SPANTABLE'):        # per-launch (start, end, issue, host issue) for timeline tools
        np.savetxt(os.environ['LDG_SPANTABLE'], span_tab, fmt='%.4f')
    dec.ctx.profile(False)
    # the roofline leg: the demod alone (kernel ldg_k_demod_iso) over one full-width launch's
    # reads, ISO_ITERS launches back to back, HIP events on its stream -- the per-dispatch
    # figure a kernel trace of this command reports for ldg_k_demod_iso (profiles/)
    if hasattr(wl, 'before_iso'):
        wl.before_iso()
    if dist is not None and shared_device:
        # ranks sharing a GPU (a rehearsal on a smaller box) take the leg in turn, so each
        # times the kernel alone on the device as a one-rank-per-GPU run does
        for r in range(world):
            barrier()
            if r == rank:
                iso_reads, iso_ms, cut_ms = iso_leg(dec)
        barrier()
    else:
        iso_reads, iso_ms, cut_ms = iso_leg(dec)
    reads_timed = dec.stats['reads'] - reads0
    used_timed = dec.stats['reads_used'] - used0
    checks = wl.checks()
    same_share = None
    if dist is not None and isinstance(wl, ShardedWorkload):
        # the N = 1 rate of the same per-rank work, rank 0 alone on its GPU (others wait)
        barrier()
        if rank == 0:
            progress(rank, 'same-share single-GPU leg')
            same_share = wl.same_share_single()
        barrier()

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

    msps = consumed_all / dt_max / 1e6
    fields_s = 2 * frames_all / dt_max
    # Roofline of the dominant kernel, the demod (the one kernel that consumes the capture and
    # fills the chip: one 150 KiB-LDS workgroup per CU).  Unit of work = one RF sample consumed;
    # algorithmic bytes per unit = SURVEY §8(d): input (1 B u8, 5/4 .lds, 4/3 .r30, 2 s16) +
    # .tbc out 955,500 / 1,334,667 B + .pcm 0.0048 B (1.7207 B for u8).  One launch of the
    # roofline leg demodulates `iso_reads` decoded field reads (FS_VALID: all their blocks
    # inside the resident capture, so a sharded rank's out-of-window speculative reads
    # are not among them); a field read the replay used advances the capture by
    # consumed / reads_used samples (reads overlap by ~1/3), so
    # units per launch = iso_reads * consumed / reads_used over the timed steps.
    pal = args.system == 'PAL'
    bps = BYTES_PER_SAMPLE[wl.fmt] + (PAL_TBC_BYTES_PER_SAMPLE if pal else NTSC_TBC_BYTES_PER_SAMPLE) + \
        NTSC_PCM_BYTES_PER_SAMPLE
    samples_per_read = consumed / max(used_timed, 1)
    units_iso = iso_reads * samples_per_read
    achieved = bps * units_iso / (iso_ms * 1e-3) / 1e9
    traffic, lds, traffic_cut, lds_cut = None, None, None, None
    # the committed --pmc passes of this system's bench command (PAL stores the pilot channel
    # too), attached only when they were taken of this same library (its build's source hash)
    from ldgpu.native import lib_source_hash
    pmc = os.path.join(ROOT, 'profiles', 'pmc_traffic_pal.json' if pal else 'pmc_traffic.json')
    lib_hash = lib_source_hash()
    counters = {'lib_source_sha256': lib_hash, 'pmc_file': 'profiles/' + os.path.basename(pmc), 'state': 'absent'}
    if os.path.exists(pmc):
        pj = json.load(open(pmc))
        counters['pmc_lib_source_sha256'] = pj.get('lib_source_sha256')
        if lib_hash is not None and pj.get('lib_source_sha256') == lib_hash:
            counters['state'] = 'fresh'
            traffic = pj['kernels'].get('demod_iso')
            lds = bound_analysis(pj.get('demod_iso_sq'), traffic, iso_ms)
            traffic_cut = pj['kernels'].get('demod_iso_cut')
            if cut_ms:
                lds_cut = bound_analysis(pj.get('demod_iso_cut_sq'), traffic_cut, cut_ms, 'demod_iso_cut_sq')
        else:
            counters['state'] = 'stale'      # profiled from another build: not attached
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
        'units_per_launch': round(units_iso), 'samples_per_read': round(samples_per_read),
        'algorithmic_bytes_per_sample': round(bps, 4),
        'algorithmic_bytes_per_launch': round(bps * units_iso),
        'traffic_unit': 'bytes per launch, 2*FETCH_SIZE + WRITE_SIZE (profiles/%s, demod_iso)' % os.path.basename(pmc),
        'traffic_x_algorithmic': (traffic / (bps * units_iso)) if traffic else None,
        'issue': lds, 'fp64': fp64, 'counters': counters,
        'production': {
            'kernel': 'ldg_k_demod_iso_cut: the shipped demod body (ldg_k_demod, video cut) under its own symbol, '
                      'same reads, launches and units as the leg above',
            'avg_launch_ms': round(cut_ms, 4) if cut_ms else None,
            'achieved': round(bps * units_iso / (cut_ms * 1e-3) / 1e9, 4) if cut_ms else None,
            'frac': bps * units_iso / (cut_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if cut_ms else None,
            'traffic': traffic_cut, 'issue': lds_cut},
        'pipeline': {'launches': dom_launches, 'span_ms': round(span_ms, 4), 'hip_event_ms': round(event_ms, 4),
                     'busy_ms_per_launch': round(busy_ms, 4), 'units_per_launch': round(units_pipe),
                     'achieved_busy': round(bps * units_pipe / (busy_ms * 1e-3) / 1e9, 4),
                     'demod_streams': int(os.environ.get('LDG_DEMOD_STREAMS', '2')),
                     'note': 'the timed steps\' demod launches: in-kernel execution span (device clock), HIP-event '
                             'interval, and the union of the spans per launch (two demod streams overlap '
                             'consecutive launches; field kernels co-run on the CUs)'},
    }
    if not args.no_comb:
        roofline['bytes_per_sample_with_comb'] = round(bps + (PAL_COMB_BYTES_PER_SAMPLE if pal else
                                                              NTSC_COMB_BYTES_PER_SAMPLE), 4)
    cpu = None
    if not args.no_cpu and world == 1:
        # the capture in host memory, as a loader would read it (the CPU path's input)
        procs = args.cpu_procs or min(16, len(os.sched_getaffinity(0)))
        progress(rank, 'CPU baseline (oracle, %d frames per process, 1 and %d processes)' % (args.cpu_frames, procs))
        cpu = cpu_baseline(wl.host_capture, wl.fmt, wl.system, args.cpu_frames, procs)
    line = {
        'metric': 'RF Msamples/s (40 MSPS %s, full RF->.tbc decode)' % args.system, 'value': round(msps, 3),
        'unit': 'RF Msamples/s', 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
        'ms_per_step': round(dt_max / args.steps * 1e3, 3), 'higher_is_better': True, 'scaling': wl.scaling,
        'vs_baseline': None, 'dtype': 'f64', 'data': wl.data, 'config': wl.config(frames),
        'fields_per_s': round(fields_s, 1), 'realtime_x': round(msps / 40.0, 2),
        'roofline': roofline,
        'kernels_ms': {k: round(v[1], 3) for k, v in sorted(stats.items(), key=lambda kv: -kv[1][1])},
        'cpu_baseline': cpu,
        'checks': dict(checks, synth_s=round(wl.synth_s, 2), reads_decoded=dec.stats['reads'],
                       reads_used=dec.stats['reads_used'], batches=dec.stats['batches'],
                       misses=dec.stats.get('misses', 0), drain_waits=dec.stats.get('drain_waits', 0), vcut_redo=dec.stats.get('vcut_redo', 0), step_ms=step_ms,
                       park_redo=dec.stats.get('migrated', 0),
                       # SURVEY §8(d)'s protocol reports the median step: rank 0's, beside the mean
                       step_ms_median=round(float(np.median(step_ms)), 3) if step_ms else None,
                       value_at_median_step=(round(msps * (dt_max / args.steps * 1e3) / float(np.median(step_ms)), 3)
                                             if step_ms else None),
                       host_s={k: round(dec.stats.get(k, 0.0), 4)
                               for k in ('plan_s', 'gpu_s', 'replay_s', 'flush_s', 'wait_s')},
                       inflight_at_wait=dec.stats.get('inflight_at_wait'), demod_issue=issue),
    }
    if world > 1:
        line['per_rank_value'] = round(msps / world, 3)
        if same_share is not None:
            line['same_share_n1'] = {
                'value': round(same_share[0], 3), 'unit': 'RF Msamples/s', 'ms_per_step': round(same_share[1], 3),
                'frames_per_step': same_share[2],
                'note': ("rank 0's share of this capture (1/%d) decoded by one GPU alone in this session, no "
                         'exchange: the N = 1 rate of the per-rank work, so the N-rank value has a baseline on '
                         'its own workload (N x this = perfect scaling)' % world)}
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
