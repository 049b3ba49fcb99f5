"""Field-group sharding of one capture across GPUs.

Fields are independent except for four chains (F10): the read position
(`nextsample = readsample + nextfieldoffset`), the MTF level from the previous
CAV frame number, the 48 kHz audio time offset, and the comb's burst-level EMA.
Each rank decodes a contiguous range of the capture:

1. rank k starts two frames before its boundary B_k and decodes warm-up frames
   that are not output. The read position is signal-locked: a start converges
   onto the true chain after one field, and the MTF after one frame. It outputs
   the frames that start in [B_k, B_{k+1}), with audio deferred: each field's
   audio inputs go to the device field archive.
2. One small exchange (all_gather of a per-rank summary):
   - each rank's first frame start, its last `nextsample` and its end MTF;
   - the frame count;
   - the audio-offset transitions (the line count of each frame's last field).
3. Verification and fix-up:
   - The chain is exact iff rank k's first frame starts at rank k-1's
     `nextsample` with rank k-1's end MTF. On a mismatch the rank re-decodes
     from that boundary state.
   - The exact audio offset at each rank's start is the offset chain replayed
     over the transitions of the ranks before it. Each field's 48 kHz audio is
     then computed from the archive.
   - Global frame indices are the prefix sum of the frame counts.

The result is identical to a single decode of the whole capture:
tests/test_shard.py checks it on the GPU, with ranks run one after another, and
on CPU with gloo for the exchange logic.

Capture windows (shard_windows / exchange_halo): a rank keeps only the samples
its reads touch in HBM -- its own range from storage, [lo_k, cut_k), plus a
tail halo [cut_k, hi_k) of the next shard's first samples (the last frames
before B_{k+1} read up to two fields and one 1,000,001-sample read past it).
The halo comes from rank k+1, which already holds those samples, over a
point-to-point exchange: RCCL (torch.distributed 'nccl') between the GPUs'
capture buffers when every rank has its own GPU, gloo through host memory
otherwise.  A read that still falls outside the window raises WindowMiss and
the rank re-runs with the whole capture.
"""
import tempfile

import numpy as np

from .decoder import WindowMiss, arange_last
from .formats import FMT_LDS, FMT_R30, FMT_S16, FMT_U8

GROUP = 12                      # window cuts on whole packing groups of every format (3 and 4 samples)
CHAIN_KEYS = ('mtf_level', 'last_framenr', 'last_isclv', 'last_read')   # the framer state a decode continues from
READ_SPAN = 1000001 + 2 * 16384  # a read's samples past its start (RFDecode.demod blocks)


def sample_byte(fmt, s):
    """Byte offset of sample s (s a multiple of GROUP)."""
    return {FMT_U8: s, FMT_S16: 2 * s, FMT_R30: (s // 3) * 4, FMT_LDS: (s // 4) * 5}[fmt]


def shard_windows(bounds, spf, nsamples, warmup_frames=2, halo_frames=2):
    """Per rank (lo, cut, hi): the resident samples [lo, hi), read from storage
    [lo, cut) and received from the next rank [cut, hi).  The last rank's window ends
    like the others' past the decode's end (bounds[-1], the frame limit's reach), not at
    the end of the capture: an epoch of a long capture keeps O(epoch) samples resident.
    Reads past it (the last rank extending over skipped fields, ShardedDecode.extend)
    widen the window (ShardedDecode widen)."""
    world = len(bounds) - 1
    out = []
    for k in range(world):
        first = bounds[k] - (warmup_frames * spf if k else 0)
        lo = max(0, (first - 1024) // GROUP * GROUP)
        hi = min(nsamples, -(-(bounds[k + 1] + halo_frames * spf + READ_SPAN) // GROUP) * GROUP)
        cut = hi if k == world - 1 else bounds[k + 1] // GROUP * GROUP
        out.append((lo, cut, hi))
    return out


def widen_window(sample, spf, nsamples, ahead_frames=8):
    """The window a rank reloads when a resumed decode reads past its window at `sample`
    (WindowMiss.resume_at): from a frame before it to `ahead_frames` frames and a read past it."""
    lo = max(0, (sample - spf - 1024) // GROUP * GROUP)
    hi = min(nsamples, -(-(sample + ahead_frames * spf + READ_SPAN) // GROUP) * GROUP)
    return lo, hi


def halo_plan(windows):
    """For each rank k < world-1: True if rank k+1 holds all of rank k's halo in the part
    it reads from storage (then the halo travels rank k+1 -> k), else False (rank k
    reads its halo from storage too).  The same on every rank."""
    plan = []
    for k in range(len(windows) - 1):
        lo, cut, hi = windows[k]
        nlo, ncut, _ = windows[k + 1]
        plan.append(nlo <= cut and hi <= ncut)
    return plan


def exchange_halo(buf, rank, windows, fmt, p2p):
    """Fill this rank's halo bytes of `buf` (the window's bytes, its own part already
    in place) from the next rank, and send the previous rank its halo.  buf is
    sliced by bytes; p2p([(kind, tensor, peer)]) runs the point-to-point transfers
    (kind 'send' / 'recv') together, e.g. torch.distributed.batch_isend_irecv.
    Returns True if this rank's halo came over the exchange."""
    world = len(windows)
    plan = halo_plan(windows)
    lo, cut, hi = windows[rank]
    ops = []
    if rank > 0 and plan[rank - 1]:
        plo, pcut, phi = windows[rank - 1]
        a, b = sample_byte(fmt, pcut) - sample_byte(fmt, lo), sample_byte(fmt, phi) - sample_byte(fmt, lo)
        ops.append(('send', buf[a:b], rank - 1))
    got = False
    if rank < world - 1 and plan[rank]:
        a, b = sample_byte(fmt, cut) - sample_byte(fmt, lo), sample_byte(fmt, hi) - sample_byte(fmt, lo)
        ops.append(('recv', buf[a:b], rank + 1))
        got = True
    if ops:
        p2p(ops)
    return got


def torch_p2p(ops):
    """exchange_halo's transfers over torch.distributed (RCCL for device tensors
    under the 'nccl' backend, gloo for host tensors)."""
    import torch.distributed as dist
    reqs = dist.batch_isend_irecv([dist.P2POp(dist.isend if k == 'send' else dist.irecv, t, peer)
                                   for k, t, peer in ops])
    for r in reqs:
        r.wait()


def audio_next(offset, linecount, line_period):
    """downscale_audio's returned next offset (lddecode_core.py:432-437, 484):
    np.arange(offset, frametime + gap, gap)[-1] - frametime, without the array
    (decoder.arange_last); an empty range raises IndexError as ticks[-1] would.
    ldg_audio_offsets runs the same recurrence in the library (replay_offsets)."""
    frametime = (line_period * linecount) / 1000000
    gap = 1 / 48000.0
    try:
        return arange_last(offset, frametime + gap, gap) - frametime
    except ValueError:
        raise IndexError('index -1 is out of bounds for axis 0 with size 0') from None


def shard_bounds(start, end, spf, world):
    """Frame-aligned sample boundaries B_0 = start < B_1 < ... < B_world = end."""
    nfr = max(0, (end - start) // spf)
    return [start + (nfr * k // world) * spf for k in range(world)] + [end]


def decode_bounds(nsamples, nbytes, spf, world, start_frame=0, length=None, start_sample=None):
    """The shard boundaries of a decode, its frame limit and its start sample.
    Frames past the limit (lddecode.py:49, -l; by default the 10-bit EOF guard's
    count, ~80% of a u8 capture) are dropped, so the shards split only the samples
    the limit can reach -- the limit's nominal start plus two frames -- instead of
    the whole capture (whose last fifth a single decode never reads).  Every caller
    (the decode, the capture windows, the benchmark) uses this one split.  The split
    is nominal (one frame per samples_per_frame): when skipped fields leave the ranks
    short of the limit, the last rank reads on past its boundary (ShardedDecode.extend;
    its capture window runs to the end of the capture)."""
    bpf = spf * 5 // 4
    limit = length if length is not None else nbytes // bpf - start_frame
    start = start_frame * spf if start_sample is None else start_sample
    end = min(nsamples, start + (max(limit, 0) + 2) * spf)
    return shard_bounds(start, end, spf, world), limit, start


def replay_offsets(o0, transitions, line_period):
    """Offsets after each transition, starting from o0: [o0, o1, ..., on] (audio_next's
    recurrence, run in the library: a shard replays every earlier shard's fields)."""
    from .native import audio_offsets
    return audio_offsets(o0, transitions, line_period)


def check_chain(summaries):
    """Ranks whose first frame does not continue the previous rank's chain (exactly).
    first_mtf is the MTF in force when the first kept frame's readframe began (the
    framer's checkpoint, before any MTF re-read inside it), which is what the
    previous rank hands over as end_mtf."""
    bad = []
    prev = None
    for k, s in enumerate(summaries):
        if s['n'] == 0:
            continue
        if prev is not None and (s['first_start'] != prev['last_next'] or s['first_mtf'] != prev['end_mtf']):
            bad.append(k)
        prev = s
    return bad


def start_offsets(summaries, line_period, o0=0.0):
    """Exact audio time offset at each rank's first frame (rank 0 starts at o0: 0 at
    the capture's start, the previous epoch's end offset for a later epoch)."""
    o, out = o0, []
    for s in summaries:
        out.append(o)
        o = replay_offsets(o, s['transitions'], line_period)[-1]
    return out


def frame_offsets(summaries):
    """Global index of each rank's first frame (exclusive prefix sum of the counts)."""
    out, acc = [], 0
    for s in summaries:
        out.append(acc)
        acc += s['n']
    return out


class FrameSpill:
    """A rank's output frames on storage until the exchange has fixed their global
    offsets: appended as they arrive, read back through a memory map.  Host memory
    stays bounded by one frame, whatever the shard's length (an hour of NTSC is
    ~13 GB of .tbc frames per rank on 8 GPUs)."""

    def __init__(self, directory=None):
        self.directory = directory
        self.fh = None
        self.shape = None
        self.n = 0
        self._map = None

    def reset(self):
        self.close()
        self.fh = tempfile.TemporaryFile(prefix='ldgpu_shard_', dir=self.directory)
        self.n = 0

    def append(self, pic):
        pic = np.ascontiguousarray(pic)
        if self.shape is None:
            self.shape, self.dtype = pic.shape, pic.dtype
        assert pic.shape == self.shape and pic.dtype == self.dtype
        self._map = None
        self.fh.write(pic.tobytes())
        self.n += 1

    def _frames(self):
        if self._map is None and self.n:
            self.fh.flush()
            self._map = np.memmap(self.fh, dtype=self.dtype, mode='r', shape=(self.n,) + tuple(self.shape))
        return self._map

    def __len__(self):
        return self.n

    def write_at(self, i, pic):
        """Overwrite frame i (a re-combed frame)."""
        pic = np.ascontiguousarray(pic)
        assert pic.shape == self.shape and pic.dtype == self.dtype and 0 <= i < self.n
        self._map = None
        self.fh.seek(i * pic.nbytes)
        self.fh.write(pic.tobytes())
        self.fh.seek(0, 2)

    def __getitem__(self, i):
        if isinstance(i, slice):
            m = self._frames()
            return m[i] if m is not None else []
        if not -self.n <= i < self.n:
            raise IndexError(i)
        return self._frames()[i]

    def __iter__(self):
        return (self[i] for i in range(self.n))

    def close(self):
        self._map = None
        if self.fh is not None:
            self.fh.close()
            self.fh = None


class ShardedDecode:
    """One rank's part of a field-group sharded decode, in two phases."""

    def __init__(self, dec, rank, world, start_frame=0, warmup_frames=2, length=None, start_sample=None,
                 whole_capture=None, spill_dir=None, resident=False, comb=False, init=None, widen=None):
        """whole_capture: callable that makes the whole capture resident (the fallback
        when a capture window turns out too small).  widen: callable(sample) that makes
        a window around `sample` resident (widen_window): a resumed decode (the last
        rank's extension) that reads past its window continues there instead.  spill_dir: where the output
        frames wait for the exchange (FrameSpill; default: the system temp dir).
        resident: the frames stay in HBM (benchmark mode: decode(sink=None), the fused
        comb with comb=True); nothing is spilled.
        init: the exact chain state at start_sample when it is not the capture's first
        frame (a later epoch of an epoch-wise decode, epoch_state()): mtf_level,
        last_framenr, last_isclv, last_read, audio_offset, comb_state, frame0."""
        self.dec, self.rank, self.world = dec, rank, world
        self.init = init
        self.resident, self.comb = resident, comb
        self.whole_capture, self.window_misses, self.extended = whole_capture, 0, 0
        self.widen, self.widened = widen, 0
        self.spf = dec.rf.samples_per_frame
        # the whole decode's frame count limit (lddecode.py:49; -l): frames past it are dropped
        self.bounds, self.limit, self.start = decode_bounds(dec.cap_nsamples, dec.cap_bytes, self.spf, world,
                                                            start_frame, length, start_sample)
        self.warmup = warmup_frames
        self.frames = FrameSpill(spill_dir)   # this rank's output frames, in order
        # comb (CLI): the fused 2D comb's rgb48 frames, combed in HBM with the decode
        # (ldg_output_async) from a "not initialised" burst-level EMA; comb_fix() then
        # re-combs the first few with the exact state handed over from the earlier ranks
        self.rgb = FrameSpill(spill_dir) if (comb and not resident) else None

    def _stop(self):
        stop = self.bounds[self.rank + 1]
        if self.rank == self.world - 1 and stop >= self.dec.cap_nsamples:
            stop = None
        return stop

    def _run(self, sink, start_sample, keep_from, firstframe, init=None, stop='nominal', length=None, resume=False):
        """Decode [start_sample, stop) (stop 'nominal': this rank's boundary; None: no stop)."""
        dec = self.dec
        if stop == 'nominal':
            stop = self._stop()

        def keep(pic, audio, meta):
            self.frames.append(pic)
            if sink:
                sink(pic, None, meta)

        if resume:
            # continue the decode this rank holds; a read past the window (the decoder
            # stopped at the checkpoint of the frame that needed it, every earlier frame
            # emitted) widens the window and the decode goes on from that frame
            n0 = len(dec.shard_frames)
            while True:
                left = None if length is None else length - (len(dec.shard_frames) - n0)
                try:
                    dec.decode(start_sample=start_sample, stop_sample=stop, keep_from=keep_from, firstframe=firstframe,
                               archive=True, sink=None if self.resident else keep, init_state=init,
                               comb=self.comb, length=left, resume=True,
                               comb_sink=self.rgb.append if self.rgb is not None else None)
                    return
                except WindowMiss as e:
                    if self.widen is None or e.resume_at is None:
                        raise
                    self.widen(e.resume_at)
                    self.widened += 1
                    start_sample, init = e.resume_at, None

        for attempt in range(2):
            if not resume:
                self.frames.reset()
                if self.rgb is not None:
                    self.rgb.reset()
            try:
                dec.decode(start_sample=start_sample, stop_sample=stop, keep_from=keep_from, firstframe=firstframe,
                           archive=True, sink=None if self.resident else keep, init_state=init,
                           comb=self.comb, length=length, resume=resume,
                           comb_sink=self.rgb.append if self.rgb is not None else None)
                return
            except WindowMiss:
                # a read outside this rank's capture window: decode from the whole capture
                if attempt or self.whole_capture is None:
                    raise
                self.whole_capture()
                self.window_misses += 1

    def local(self, sink=None):
        """Phase 1: decode this rank's range; returns the summary to exchange."""
        b = self.bounds[self.rank]
        if self.rank == 0:
            if self.init is None:
                self._run(sink, b, None, True)
            else:
                self._run(sink, b, None, False, init={k: self.init[k] for k in CHAIN_KEYS})
        else:
            self._run(sink, max(0, b - self.warmup * self.spf), b, False)
        return self.summary()

    def summary(self):
        dec, sf = self.dec, self.dec.shard_frames
        t0 = sf[0]['tstart'] if sf else len(dec.transitions)
        return {'rank': self.rank, 'n': len(sf),
                'first_start': sf[0]['start'] if sf else None,
                'first_mtf': sf[0]['mtf0'] if sf else None,
                'last_next': sf[-1]['nextsample'] if sf else None,
                'end_mtf': float(dec.mtf_level), 'end_framenr': dec.last_framenr, 'end_isclv': dec.last_isclv,
                'end_read': dec.last_read,
                'transitions': list(dec.transitions[t0:]), 't0': t0}

    @staticmethod
    def _state(s):
        """The chain state a rank's summary hands to the next rank's first frame (the
        framer's MTF / frame number / CLV flag, and fd.tell()'s read for the EOF guard)."""
        return {'mtf_level': s['end_mtf'], 'last_framenr': s['end_framenr'], 'last_isclv': s['end_isclv'],
                'last_read': s['end_read']}

    def refix(self, summaries, sink=None):
        """Re-decode from the previous rank's exact end state (chain mismatch)."""
        prev = next(s for s in reversed(summaries[:self.rank]) if s['n'])
        self._run(sink, prev['last_next'], None, False, init=self._state(prev))
        return self.summary()

    def extend(self, summaries, sink=None):
        """The last rank decodes on past its nominal end while the whole decode has fewer
        frames than its limit.  The split assumes one frame per samples_per_frame; fields
        the reference skips (invalid fields, "no/corrupt VSYNC found, jumping forward",
        lddecode_core.py:909-920,1205-1212) move the limit's last frame later, and a single
        decode reads as far as it takes (lddecode.py:88-90).  Returns the (possibly new)
        summary, or None if nothing changed."""
        if self.rank != self.world - 1:
            return None
        stop = self._stop()
        base = frame_offsets(summaries)[self.rank]
        me = summaries[self.rank]
        want = self.limit - base - me['n']
        if stop is None or want <= 0:
            return None
        if me['n']:
            # the decoder still holds this rank's end state: continue from its last frame
            self._run(sink, me['last_next'], None, False, stop=None, length=want, resume=True)
        else:
            # no frame of this rank's own: decode the rest from the previous rank's end state
            prev = next((s for s in reversed(summaries[:self.rank]) if s['n']), None)
            if prev is None:
                return None
            self._run(sink, prev['last_next'], None, False, init=self._state(prev), stop=None, length=want)
        self.extended = len(self.dec.shard_frames) - me['n']
        return self.summary()

    def finish(self, summaries):
        """Phase 2: exact audio from the archive and global frame indices.
        Returns [(global_index, pcm int16, meta)] for this rank's output frames (those
        under the decode's frame limit); each pcm is a view of one array holding the
        rank's audio in frame order."""
        dec = self.dec
        lp = dec.sysp.line_period
        o0 = start_offsets(summaries, lp, self.init['audio_offset'] if self.init else 0.0)[self.rank]
        me = summaries[self.rank]
        offs = replay_offsets(o0, me['transitions'], lp)
        base = frame_offsets(summaries)[self.rank]
        frame0 = self.init['frame0'] if self.init else 0
        frames = dec.shard_frames[:max(0, min(len(dec.shard_frames), self.limit - base))]
        ents = [e for f in frames for e, _ in f['audio']]
        eoff = [offs[t - me['t0']] for f in frames for _, t in f['audio']]
        flat, lens = [], []
        step = max(len(ents), 1)          # one call: the library runs any number of entries at once
        for i in range(0, len(ents), step):
            pcm, counts, _ = dec.ctx.archive_audio(ents[i:i + step], eoff[i:i + step], packed=True)
            if (counts < 0).any():
                raise RuntimeError('audio index error (reference: field invalid)')
            flat.append(pcm)                  # the entries' samples one after another
            lens.append(2 * counts.astype(np.int64))
        flat = np.concatenate(flat) if flat else np.zeros(0, dtype=np.int16)
        ecum = np.concatenate([[0], np.cumsum(np.concatenate(lens))]) if lens else np.zeros(1, dtype=np.int64)
        fb = ecum[np.cumsum([0] + [len(f['audio']) for f in frames])].tolist()   # frame k: flat[fb[k]:fb[k+1]]
        return [(base + i, flat[fb[i]:fb[i + 1]],
                 {'frame': frame0 + base + i, 'vbi': f['vbi'], 'nextsample': f['nextsample'], 'fields': f['fields']})
                for i, f in enumerate(frames)]

    def end_state(self, summaries, comb_a0=None, line0=None):
        """The exact chain state after the last frame the decode outputs (frame limit - 1,
        or the last frame if fewer), if this rank holds that frame, else None: the next
        epoch's init (an epoch-wise decode, lddecode.py --epoch-frames).  comb_a0: the
        burst-level EMA entering this rank (comb_fix), run on over its frames up to that one."""
        total = sum(s['n'] for s in summaries)
        n = min(total, self.limit)
        base = frame_offsets(summaries)[self.rank]
        j = n - 1 - base
        if n == 0 or not 0 <= j < summaries[self.rank]['n']:
            return None
        f = self.dec.shard_frames[j]
        mtf, fnr, clv, last_read, tend = f['end']
        o0 = self.init['audio_offset'] if self.init else 0.0
        o = start_offsets(summaries, self.dec.sysp.line_period, o0)[self.rank]
        me = summaries[self.rank]
        o = replay_offsets(o, me['transitions'][:tend - me['t0']], self.dec.sysp.line_period)[-1]
        comb = -1.0
        if comb_a0 is not None:
            comb = comb_chain(comb_a0, comb_burst_levels(self.frames[:j + 1], line0=line0))
        return {'mtf_level': float(mtf), 'last_framenr': fnr, 'last_isclv': bool(clv),
                'last_read': int(last_read), 'nextsample': int(f['nextsample']), 'audio_offset': float(o),
                'comb_state': float(comb), 'frame0': (self.init['frame0'] if self.init else 0) + n}


def comb_fix(sd, allgather, nkept, stats=None):
    """The comb's burst-level EMA across the ranks (comb-ntsc.cxx:560-566, global over
    every frame): exchange each rank's chain summary, take the exact state entering this
    rank, and re-comb (on the GPU) the first frames whose speculative state differed.
    nkept: this rank's frames that are output (the frame limit may drop the rest).
    Collective: every rank calls it."""
    dec = sd.dec
    line0 = 20 if dec.ctx.comb_lines == 525 else COMB_LINE0
    lpf = 525 - line0
    levels = comb_burst_levels(sd.frames[:nkept] if nkept else [], line0=line0)
    summ = allgather(comb_summary(levels))
    first = sd.init['comb_state'] if sd.init else -1.0          # the EMA entering the decode
    a0 = comb_start_from_summaries(summ, sd.rank, first)
    full = False
    if any(comb_start_from_summaries(summ, r, first) is None for r in range(len(summ))):
        # some rank's chain had not converged within its prefix: exchange every level
        every = allgather(levels)
        a0, full = comb_start_state(every, sd.rank, first), True
    k = comb_redo_frames(a0, levels, lpf)
    if k:
        dec.ctx.comb_set_state(a0)
        for i in range(0, k, dec.ctx.max_frames):
            j = min(k, i + dec.ctx.max_frames)
            rgb = dec.ctx.comb_ntsc(np.stack([np.asarray(f) for f in sd.frames[i:j]]))
            for q in range(j - i):
                sd.rgb.write_at(i + q, rgb[q])
    if stats is not None:
        stats['comb_recombed_frames'] = stats.get('comb_recombed_frames', 0) + k
        stats['comb_full_exchange'] = full
    return a0


def comb3d_sharded(dec, rank, allgather, frames, base, core_ire=-1.0, range_ire=-1.0, stats=None):
    """The 3D comb without optical flow (comb-ntsc -d 3 -F, comb-ntsc.cxx:369-412,834-892)
    over one sharded decode's frames: every rank combs its own frames.  The single process
    combs frame g with frames g - 1 and g + 1 once g + 1 has arrived, every frame but the
    capture's first and last, with the burst-level EMA chained over those frames in order
    (ToRGB :560-566).  Here each rank receives the frames just outside its range (the
    previous rank's last, the next rank's first: one frame each way), takes the exact EMA
    entering its first combed frame from the earlier ranks' chain summaries (as the 2D
    comb_fix), and runs the device 3D comb over [prev] + its frames + [next]: the rgb48 of
    every frame it holds that has both neighbours, exactly the single process's.
    frames: this rank's decoded frames in order (global indices base, base + 1, ...).
    Returns [(output index, rgb48)], output index = global frame index - 1 (the single
    process's .rgb holds frames 1 .. N - 2).  Collective: every rank calls it."""
    n = len(frames)
    info = allgather({'n': n, 'base': base,
                      'first': np.array(frames[0]) if n else None, 'last': np.array(frames[-1]) if n else None})
    total = sum(i['n'] for i in info)
    prev = next((i['last'] for i in reversed(info[:rank]) if i['n']), None)
    nxt = next((i['first'] for i in info[rank + 1:] if i['n']), None)
    # the frames this rank combs (both neighbours in the capture), and the EMA entering them
    lo, hi = max(base, 1), min(base + n, total - 1)          # global [lo, hi)
    line0 = 20 if dec.ctx.comb_lines == 525 else COMB_LINE0
    levels = comb_burst_levels(frames[lo - base:hi - base] if hi > lo else [], line0=line0)
    summ = allgather(comb_summary(levels))
    a0 = comb_start_from_summaries(summ, rank, -1.0)
    if any(comb_start_from_summaries(summ, r, -1.0) is None for r in range(len(summ))):
        a0 = comb_start_state(allgather(levels), rank, -1.0)   # a chain without a burst for too long
    out = []
    if n:
        dec.ctx.comb_reset()
        dec.ctx.comb_set_state(a0)
        g = lo                                       # the next output's global frame index
        window = ([prev] if prev is not None else []) + [frames[i] for i in range(n)] + \
            ([nxt] if nxt is not None else [])
        step = max(1, dec.ctx.max_frames)
        for i in range(0, len(window), step):
            for rgb in dec.ctx.comb_ntsc3d(np.stack([np.asarray(f) for f in window[i:i + step]]), core_ire,
                                           range_ire):
                out.append((g - 1, rgb))
                g += 1
        assert g == max(hi, lo), (g, lo, hi)
    if stats is not None:
        stats['comb3d_frames'] = stats.get('comb3d_frames', 0) + len(out)
    return out


def decode_sharded(dec, rank, world, allgather, sink=None, start_frame=0, length=None, start_sample=None,
                   whole_capture=None, spill_dir=None, resident=False, comb=False, stats=None, init=None,
                   epoch_end=None, widen=None):
    """Run all phases with `allgather(obj) -> [obj per rank]` (torch.distributed
    all_gather_object, or an in-process stand-in).  Returns this rank's
    [(global_index, frame, pcm, meta)] (with comb: [(..., meta, rgb48)], the exact
    comb output, comb_fix); the frames are memory-mapped views of the rank's spill
    files (FrameSpill), valid while the returned list's frames are.
    resident: frames stay in HBM (benchmark mode) and frame is None.
    init: the chain state at start_sample (a later epoch, ShardedDecode); epoch_end: a dict
    that receives the exact state after the last output frame (ShardedDecode.end_state)."""
    import gc
    import time
    # the cyclic collector stays off for the whole phase sequence, as the decode keeps it
    # off (GPUDecoder.decode): a full collection over a shard's thousands of frame records
    # landing inside the exchange or the audio phase cost 10-100 ms (profiles/r04_j)
    gc_on = gc.isenabled()
    gc.disable()
    try:
        return _decode_sharded(dec, rank, world, allgather, sink, start_frame, length, start_sample,
                               whole_capture, spill_dir, resident, comb, stats, init, epoch_end, widen)
    finally:
        if gc_on:
            gc.enable()


def _decode_sharded(dec, rank, world, allgather, sink, start_frame, length, start_sample, whole_capture,
                    spill_dir, resident, comb, stats, init, epoch_end, widen):
    import time
    t0 = time.perf_counter()
    sd = ShardedDecode(dec, rank, world, start_frame, length=length, start_sample=start_sample,
                       whole_capture=whole_capture, spill_dir=spill_dir, resident=resident, comb=comb, init=init,
                       widen=widen)
    loc = sd.local()
    t1 = time.perf_counter()
    summ = allgather(loc)
    refixes = 0
    for _ in range(world):
        bad = check_chain(summ)
        if not bad:
            break
        refixes += len(bad)
        mine = sd.refix(summ) if rank in bad else summ[rank]
        summ = allgather(mine)
    if check_chain(summ):
        raise RuntimeError('sharded decode: chain did not converge')
    # the last rank reads on while the decode is short of its frame limit (skipped fields)
    ext = sd.extend(summ)
    summ = allgather(ext if ext is not None else summ[rank])
    t2 = time.perf_counter()
    res = sd.finish(summ)
    a0 = None
    if sd.rgb is not None and dec.sysp.name == 'NTSC':
        # the NTSC comb's burst-level EMA spans every frame (comb_fix); the PAL Y/C
        # decoder's is a constant-input chain at its fixed point from the first line
        # (csrc/combpal.hip pal_angle), so a PAL rank's frames comb exactly on their own
        a0 = comb_fix(sd, allgather, len(res), stats)
    if epoch_end is not None:
        # the exact state after the decode's last output frame (the next epoch's init)
        ends = allgather(sd.end_state(summ, a0, 20 if dec.ctx.comb_lines == 525 else COMB_LINE0))
        epoch_end.clear()
        epoch_end.update(next((e for e in ends if e is not None), {}))
    if stats is not None:
        for k, v in (('local_s', t1 - t0), ('exchange_s', t2 - t1), ('finish_s', time.perf_counter() - t2)):
            stats[k] = stats.get(k, 0.0) + v
        stats['refixes'] = stats.get('refixes', 0) + refixes
        stats['window_misses'] = stats.get('window_misses', 0) + sd.window_misses
        stats['window_widened'] = stats.get('window_widened', 0) + sd.widened
        stats['extended_frames'] = stats.get('extended_frames', 0) + sd.extended
        stats['frames_total'] = sum(s['n'] for s in summ)
    if resident:
        return [(g, None, a, m) for (g, a, m) in res]
    if sd.rgb is not None:
        return [(g, pic, a, m, rgb) for (g, a, m), pic, rgb in zip(res, sd.frames, sd.rgb)]
    return [(g, pic, a, m) for (g, a, m), pic in zip(res, sd.frames)]


# ---- the comb's chained state across shards -------------------------------------
COMB_LINE0, COMB_LINES, NTSC_IRESCALE = 38, 525 - 38, 358.4


def comb_burst_levels(frames, chunk=64, line0=COMB_LINE0):
    """The burst levels ToRGB reads (comb-ntsc.cxx:560-561: raw[l * 910 + 1] / irescale,
    lines line0..524: 38, or 20 with comb-ntsc -v), in frame order, for a sequence of
    525x910 .tbc frames (a list, an array or a FrameSpill; read `chunk` frames at a time)."""
    if not len(frames):
        return np.zeros(0)
    out = []
    for i in range(0, len(frames), chunk):
        part = frames[i:i + chunk]
        f = np.asarray(part if not isinstance(part, list) else np.stack(part), dtype=np.uint16).reshape(-1, 525, 910)
        out.append((f[:, line0:525, 1].astype(np.float64) / NTSC_IRESCALE).reshape(-1))
    return np.concatenate(out)


def comb_chain(a, levels):
    """The aburstlev EMA (comb-ntsc.cxx:562-565) run over `levels` from state a, in
    the kernel's and the reference's arithmetic order (exact)."""
    for b in levels.tolist():
        if b > 3:
            if a < 0:
                a = b
            a = (a * .99) + (b * .01)
    return a


def comb_start_state(levels_by_rank, rank, a=-1.0):
    """The EMA a shard's comb starts from: the chain over every earlier shard's frames
    (from a: -1, not initialised, at the capture's first frame)."""
    for r in range(rank):
        a = comb_chain(a, levels_by_rank[r])
    return a


# The EMA forgets: two runs over the same levels from different states differ by
# 0.99^k after k qualifying lines and, once below an ulp, are the same double from
# then on (csrc/comb.hip ldg_k_comb_burst).  A rank's chain over its frames is
# therefore summarised by its first COMB_PREFIX levels, the state a run from "not
# initialised" has after them and at the rank's end: a later rank replays the
# prefix from the exact state entering the rank, and if that equals the
# speculative state there, the exact state leaving the rank is the speculative
# one.  ~12 frames' levels instead of every frame's (one hour on 8 ranks: 48 KB
# per rank instead of 52 MB).
COMB_PREFIX = 6144


def comb_summary(levels):
    """This rank's part of the comb chain exchange (see COMB_PREFIX)."""
    levels = np.asarray(levels, dtype=np.float64)
    if levels.size <= COMB_PREFIX:
        return {'n': int(levels.size), 'levels': levels}
    pre = levels[:COMB_PREFIX]
    return {'n': int(levels.size), 'levels': pre, 'at_prefix': comb_chain(-1.0, pre),
            'exit': comb_chain(-1.0, levels)}


def comb_start_from_summaries(summaries, rank, a=-1.0):
    """The exact EMA entering `rank` from the earlier ranks' comb_summary()s (from a at
    rank 0), or None when some rank's speculative chain had not met the exact one by the
    end of its prefix (long stretches without burst: the caller then exchanges every level)."""
    for s in summaries[:rank]:
        a = comb_chain(a, s['levels'])
        if 'exit' in s:
            if a != s['at_prefix']:
                return None
            a = s['exit']
    return a


def comb_redo_frames(a0, levels, lines_per_frame):
    """How many of a rank's first frames the speculative comb (started "not
    initialised") combed with a burst-level EMA other than the exact one (started
    from a0): the frames before the first frame boundary where both states agree
    (all of them if they never do)."""
    levels = np.asarray(levels, dtype=np.float64)
    nfr = levels.size // lines_per_frame
    ex, sp = a0, -1.0
    for f in range(nfr):
        if ex == sp:
            return f
        part = levels[f * lines_per_frame:(f + 1) * lines_per_frame]
        ex, sp = comb_chain(ex, part), comb_chain(sp, part)
    return nfr
