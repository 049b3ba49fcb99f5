"""GPU decode driver: the reference Framer / readfield / readframe / findframe
control flow (lddecode_core.py:1193-1378, lddecode.py:39-107) over batched,
speculative field decodes on the GPU.

Why speculation: every field read starts where the previous field's sync
analysis says (``nextsample = readsample + nextfieldoffset``,
lddecode_core.py:1204) and uses the MTF level of the previous frame's VBI
(:1300-1309), and the demod of a read depends on its own overlap-save block
grid.  To keep the GPU busy, the driver predicts the next B read starts and
MTF levels, decodes them all in one ``ldg_decode_reads`` call, then replays
the reference control flow on the returned per-field records.  A read the
replay asks for that is not in the batch (a misprediction) ends the batch at
the last completed frame; the next batch restarts from that frame's
checkpoint.  Results are therefore exactly those of the sequential chain.

Audio offsets (:1289, :484) are a scalar recurrence computed here with the
reference's own numpy arithmetic; the per-sample audio resampling runs on the
GPU for all fields of a batch at once.
"""
import gc
import math
import os
import time

import numpy as np

from . import native
from .formats import FMT_LDS, FMT_R30, FMT_S16, FMT_U8, bytes_for_samples, samples_in_bytes
from .rfparams import RFTables

READLEN = 1000000
BLOCKLEN, BLOCKCUT, BLOCKSTEP = 16384, 1024, 15328
# a streamed capture keeps this many samples below the replay's position: a read's first
# block (start - 1024) and its start probe's block (start - 7664 - 1024, moved by up to
# 0.3 lines) begin there at most
STREAM_MARGIN = 32768


class Miss(Exception):
    """The replay needs a read that the current batch does not hold."""

    def __init__(self, key):
        super().__init__(key)
        self.key = key


class ReferenceCrash(RuntimeError):
    """The reference decoder would have raised (uncaught) here."""


class WindowMiss(RuntimeError):
    """A read needs capture samples outside the resident window (sharded decode).
    Raised by decode() after every frame before the one that needed the read was
    emitted, with the framer restored to that frame's start: resume_at is its start
    sample, so a resumed decode (resume=True) from there continues exactly."""

    def __init__(self, msg, resume_at=None):
        super().__init__(msg)
        self.resume_at = resume_at


def read_geometry(start):
    """Blocks of RFDecode.demod(start, 1e6) (lddecode_core.py:374-385): (s0, end, last block start)."""
    end = int(start + READLEN) + 1
    s0 = int(start - BLOCKCUT) if start > BLOCKCUT else 0
    nb = -(-(end - s0) // BLOCKSTEP)
    return s0, end, s0 + (nb - 1) * BLOCKSTEP


def loader_tell(fmt, sample, nbytes):
    """File position after loader(infile, sample, 16384) (lddutils.py:131-229) -- fd.tell()."""
    if fmt == FMT_U8:
        start, need = sample, BLOCKLEN
    elif fmt == FMT_S16:
        start, need = 2 * sample, 2 * BLOCKLEN
    elif fmt == FMT_R30:
        start, need = (sample // 3) * 4, int(np.ceil(BLOCKLEN * 3 / 4) * 4) + 4
    else:
        start, need = (sample // 4) * 5, int(np.ceil(BLOCKLEN * 5 // 4)) + 5
    return start + max(0, min(need, nbytes - start))


def arange_last(start, stop, step):
    """np.arange(start, stop, step, dtype=float64)[-1] without the array: numpy's
    length ceil((stop - start) / step) and its fill rule (element i = start +
    i * ((start + step) - start) from the third on; numpy/_core/src/multiarray/
    ctors.c PyArray_ArangeObj and the DOUBLE fill)."""
    n = math.ceil((stop - start) / step)
    if n < 1:
        raise ValueError('empty arange')
    if n == 1:
        return start
    nxt = start + step
    if n == 2:
        return nxt
    return start + float(n - 1) * (nxt - start)


class GPUField:
    """Field-like view of one decoded read (attributes of lddecode_core.Field).
    The VBI / line-code dicts are built on first use."""

    __slots__ = ('info', 'slot', 'readsample', 'mtf_level', 'audio_offset', 'valid', 'istop', 'linecount',
                 'nextfieldoffset', 'npeaks', 'nvsync', 'vbi', '_linecode', 'tbcstart', 'status',
                 'audio_next_offset', 'nextsample', 'dsaudio_used', 'tidx', 'sysp')

    def __init__(self, info, slot, readsample, mtf, audio_offset, sysp, frametime_lines):
        self.info, self.slot, self.readsample, self.mtf_level = info, slot, readsample, mtf
        self.audio_offset = audio_offset
        self.status = info.status
        self.valid = info.status == native.FS_VALID
        self.istop = bool(info.istop) if self.valid else None
        self.linecount = info.linecount
        self.nextfieldoffset = info.nextfieldoffset
        self.npeaks, self.nvsync = info.npeaks, info.nvsync
        self.tbcstart = info.tbcstart
        self.dsaudio_used = False
        self.sysp = sysp
        self._linecode = None
        self.vbi = None
        if self.valid:
            # the VBI dict (a plain attribute: the replay reads it ~18 times per frame)
            def v(x):
                return None if x == native.VBI_NONE else int(x)
            self.vbi = {'minutes': v(info.vbi_minutes), 'seconds': v(info.vbi_seconds),
                        'clvframe': v(info.vbi_clvframe), 'framenr': v(info.vbi_framenr),
                        'statuscode': None, 'status': v(info.vbi_status), 'isclv': bool(info.vbi_isclv)}
            # downscale_audio's returned next offset (lddecode_core.py:432-437,484)
            frametime = (sysp.line_period * self.linecount) / 1000000
            gap = 1 / 48000.0
            self.audio_next_offset = arange_last(audio_offset, frametime + gap, gap) - frametime
        else:
            self.audio_next_offset = audio_offset

    @property
    def linecode(self):
        if self._linecode is None and self.valid:
            info = self.info
            self._linecode = {str(self.sysp.codelines[q]): (list(info.linecode[q]) if info.linecode_ok[q] else None)
                              for q in range(3)}
        return self._linecode

    def record(self):
        rec = {'readsample': int(self.readsample), 'nextsample': int(self.nextsample), 'valid': bool(self.valid),
               'mtf_level': float(self.mtf_level)}
        if self.valid:
            rec.update({'istop': bool(self.istop), 'linecount': int(self.linecount),
                        'nextfieldoffset': int(self.nextfieldoffset), 'vbi': dict(self.vbi),
                        'linecode': dict(self.linecode)})
        return rec


def field_log_lines(fields, ntsc):
    """The lines the reference prints while reading these fields (in read order), from
    their status codes and log flags: Field.__init__'s "vsync vote needed i" / "no/corrupt
    VSYNC found, jumping forward" / 'unable to decode frame' (lddecode_core.py:620,918,939),
    FieldNTSC's 'not valid' (:1175), the TBC stage's "ERROR: Unable to decode frame,
    skipping" (:1047,1190), and readframe's `sample nextsample True istop` for every field
    a readfield call returns (:1263; `sample` is that call's first read position, istop
    the vsyncs array's 0/1)."""
    out = []
    call_start = None
    for f in fields:
        if call_start is None:
            call_start = f.readsample
        fl = f.info.log_flags
        for q in range(16):
            if (fl >> q) & 1:
                out.append('vsync vote needed %d' % q)
        if fl & native.LOG_NO_VSYNC:
            out.append('no/corrupt VSYNC found, jumping forward')
        st = f.status
        if st == native.FS_LINELOCS:
            out.append('unable to decode frame')
        if ntsc and st in (native.FS_NO_VSYNC, native.FS_SHORT, native.FS_LINELOCS):
            out.append('not valid')
        elif st == native.FS_TBC:
            out.append('ERROR: Unable to decode frame, skipping')
        if f.valid:
            out.append('%d %d True %d' % (call_start, f.nextsample, int(f.istop)))
            call_start = None
    return out


class FrameOut:
    __slots__ = ('top', 'bottom', 'audio_fields', 'vbi', 'nextsample', 'field_objs', '_fields', 'index', 'start',
                 'tstart', 'mtf0', 'log', 'end')

    def __init__(self, **kw):
        self._fields = None
        for k, v in kw.items():
            setattr(self, k, v)

    @property
    def fields(self):
        """The metadata records of the fields this frame's readframe read (GPUField.record),
        built on first use: the replay only keeps the fields (a field's record does not
        change once its frame is complete), so a decode whose per-frame metadata nobody
        reads (the benchmark's sink=None) does not build them on its critical path."""
        if self._fields is None:
            self._fields = [x.record() for x in self.field_objs]
        return self._fields


class GPUDecoder:
    """Decode a capture to .tbc frames / .pcm / per-frame metadata on one GPU.

    Device reads live in ``capacity`` slots (a read cache).  Each GPU launch
    decodes up to ``batch`` reads the forward simulator predicts the replay
    will ask for; the replay (the reference control flow) consumes cached
    reads, and a miss just triggers the next plan from the last completed
    frame, re-using every read already decoded.
    """

    def __init__(self, system='NTSC', device=0, batch=32, capacity=None, log=None):
        self.rf = RFTables(system)
        self.sysp = self.rf.system
        self.batch = batch
        # two launches in flight + the batch the host replays + the cached path
        # launches kept in flight (3 vs 2: +2% since the planner stops at the last frame).
        # NTSC 4: 20-step A/B +0.9 / +1.3 / +1.5% over 3 (r04_ze), its read chain
        # predicts exactly, so a deeper speculation costs no reads.  PAL 3: 4 was
        # 3-7% slower (more reads in flight over its start-up wander)
        self.depth = int(os.environ.get('LDG_DEPTH', '4' if self.sysp.name == 'NTSC' else '3'))
        if not 1 <= self.depth <= 7:
            raise ValueError('LDG_DEPTH must be 1..7')
        self.capacity = capacity or max((self.depth + 2) * batch, batch + 16)
        self.ctx = native.Context(system, device, max_reads=self.capacity, max_frames=self.capacity)
        self.ctx.set_filters(self.rf.params(), self.rf.tables)
        self.log = log or (lambda *a: None)
        self.stats = {'batches': 0, 'reads': 0, 'reads_used': 0, 'gpu_s': 0.0, 'replay_s': 0.0}
        self.cap_bytes = None
        self.cap_nsamples = None
        self.window = None          # (first, end) samples resident when a capture window is set
        self.stream = False         # the capture streams from its file (open_stream)
        self.cache = {}            # (start, mtf) -> (slot, info)
        self.hints = {}            # start -> absolute next start (start + nextfieldoffset)
        self._hint_keys = []       # sorted starts with hints
        P, D = (6, 4004000) if self.sysp.name == 'NTSC' else (2, 1600000)
        self.period, self.period_samples = P, D          # exact at 40 MSPS: 3 NTSC / 1 PAL frames
        self.field_nom = int(round(self.rf.freq_hz / self.sysp.fps / 2))
        self.trace = None          # diagnostics: planner steps (tools/miss_probe.py)
        self.boot_wide = os.environ.get('LDG_BOOT_WIDE', '1') == '1'   # +6.5% on the 60 s bench (tools/bootwide_ab.sh)
        self.miss_drain = os.environ.get('LDG_MISS_DRAIN', '1') == '1'
        # LDG_BOOT_AHEAD=1: _hint_ahead in the boot plans, one narrow boot launch fewer.  The
        # boot reads locate the next fields exactly, but they start mid-field and carry no
        # VBI, so the first wide launches are planned at the initial MTF: right on a CLV
        # disc (PAL config 3: +6%), wrong on a CAV one, whose MTF follows the frame number
        # (NTSC config 2: four wide launches redone per decode, -10%;
        # profiles/r05_zb_boot_ahead_ab.txt).  Off by default: the capture's disc type is
        # not known at boot, and the loss on CAV outweighs the gain on CLV.
        self.boot_ahead = os.environ.get('LDG_BOOT_AHEAD', '0') == '1'
        # while a drain waits for the launch that holds the missed read, keep `depth`
        # launches in flight, planned on from the miss (the GPU otherwise idles once
        # the launches ahead of that one land)
        self.drain_refill = os.environ.get('LDG_DRAIN_REFILL', '0') == '1'
        # read-start probes (ldg_decode_reads_async2 READ_PROBE): reads whose start the
        # plan predicted are moved on the GPU to the sync peak a one-block probe finds
        # there, so a start that jitters by a sample or two still decodes at the exact
        # start the replay will ask for
        # LDG_PROBE: 1 always, 0 never, auto (NTSC default) once the replay has missed a
        # read that a decoded read a few samples away stood in for (jitter, _note_miss) more
        # than 3 times and for over 1% of the reads used: a capture whose predictions hold
        # (the synthetic NTSC bench) saves the probes' ~2%, a jittering one gets them.  PAL
        # (default 1): config 3's start-up wander, 1.29 -> 1.04 reads per read used
        # (profiles/r05_o_probe_ab.txt)
        self.probe_mode = os.environ.get('LDG_PROBE', '1' if self.sysp.name == 'PAL' else 'auto')
        self.probe = self.probe_mode == '1'
        self.plan_idle_skip = os.environ.get('LDG_PLAN_IDLE', '1') == '1'   # (see _decode_loop)
        self.probe_win = int(0.3 * self.rf.linelen) if hasattr(self.rf, 'linelen') else 760
        self._probe_starts = []            # sorted (start, mtf) of probed reads in flight
        self.plan_guessed = set()
        self.grid_votes = int(os.environ.get('LDG_GRID_VOTES', '1'))   # _grid_next (1: the previous period's start)
        self.hist_len = max(16, self.grid_votes * P + 2)                  # valid field starts the planner keeps
        # Video cut (ldg_set_video_cut): a steady-state read starts ~10 peaks before its
        # field's vsync (lddecode_core.py:926, the previous field's nextfieldoffset), so its
        # field ends ~276 NTSC / ~326 PAL lines into the read; the demod skips the video,
        # burst and pilot channels of the read's blocks past the cut below (the last ~1/4
        # of a 1,000,001-sample read).  A field that reaches past it (a capture's first
        # read, a jump) comes back FS_VCUT and is decoded again in full.  LDG_VCUT=0: off.
        vc = os.environ.get('LDG_VCUT')
        self.video_cut = int(vc) if vc is not None else (740000 if self.sysp.name == 'NTSC' else 880000)
        self.full_keys = set()
        self.ctx.set_video_cut(self.video_cut)
        self.plan_located = 0              # leading fields the last plan walked on decoded reads
        self.htrace = [] if os.environ.get('LDG_HOSTTRACE') else None   # (perf_counter, event, n): host timeline
        self.comb, self.comb_sink = False, None
        self.comb3d = None                 # (core_ire, range_ire): the 3D comb (comb-ntsc -d 3 -F)
        self.pending = []                  # (keys, slots) of the outstanding decode launches, oldest first
        self.inflight = set()              # keys of those launches
        self.transitions = []              # audio-offset chain: linecount of each transition's field
        self.archive, self.arch_next, self.shard_frames = False, 0, []
        self._out_pending = None           # (frames, pics, audio fields, sink) awaiting their audio
        # A flushed batch whose audio launch and the previous batch's collection (the
        # host's one blocking wait besides the records) are deferred until the next
        # decode launch is issued (_finish_flush): otherwise that wait, which ends only
        # when the running demod leaves CUs to the audio kernels, sits between the
        # replay and the next launch, and the demod queue runs dry for ~1 ms per batch.
        self.defer_flush = os.environ.get('LDG_DEFER_FLUSH', '0') == '1'   # level on NTSC, PAL -8% in one pair (r04_zc): off
        self._staged = None
        self._staged_slots = set()         # slots the staged batch still reads (never evicted)
        self.frame_log = None              # callback(lines): the reference's stdout lines of each frame
        self._obufs = None                 # pinned host rings for the asynchronous output path
        self._oring = 0
        self.before_ring_reuse = None      # callback: the sink's use of the frames handed over is done

    # ---- capture ---------------------------------------------------------------
    def set_capture(self, data, fmt, device_ptr=None, nsamples=None, first_sample=0, total_bytes=None):
        """Capture resident in HBM (data: bytes/ndarray, or a device pointer).

        A window of a larger capture (field-group sharding, ldgpu/shard.py): the
        resident samples are [first_sample, first_sample + nsamples) of a capture
        of total_bytes bytes; the frame accounting (EOF guard, frame count) uses the
        whole capture, and a read that needs samples outside the window raises
        WindowMiss instead of ending the decode."""
        self.stream = False
        if device_ptr is None:
            buf = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data.view(np.uint8)
            nbytes = buf.size
            nsamples = samples_in_bytes(fmt, nbytes)
            self.ctx.set_capture(buf, nsamples, fmt, first_sample)
        else:
            nbytes = bytes_for_samples(fmt, nsamples)
            self.ctx.set_capture(None, nsamples, fmt, first_sample, device_ptr=device_ptr)
        if total_bytes is None:
            self.window = None
            self.fmt, self.cap_bytes, self.cap_nsamples = fmt, nbytes, nsamples
        else:
            self.window = (int(first_sample), int(first_sample) + int(nsamples))
            self.fmt, self.cap_bytes = fmt, int(total_bytes)
            self.cap_nsamples = samples_in_bytes(fmt, self.cap_bytes)
        self._reset_cache()

    def open_stream(self, path, fmt, ring_bytes, first_sample=0):
        """Stream the capture from its file (ldg_stream_open): the reference's loader reads
        each block from the file as the demod needs it (lddecode_core.py:373-392,
        lddutils.py:131-229), so device memory stays at ring_bytes whatever the capture's
        length; a reader thread keeps the ring filled ahead of the decode, and the decode
        releases what its replay has passed (STREAM_MARGIN below its position)."""
        self.ctx.stream_open(path, fmt, ring_bytes, first_sample)
        self.window = None
        self.stream = True
        self.fmt, self.cap_bytes = fmt, os.path.getsize(path)
        self.cap_nsamples = samples_in_bytes(fmt, self.cap_bytes)
        self._reset_cache()

    def _stream_fit(self, keys):
        """The leading keys a launch can decode from the stream's ring now: none below its
        lowest readable sample, none ending past its reach.  With nothing in flight and no
        key fitting, the stream restarts at the first key (a jump of the replay, a seek)."""
        def span(k):
            s0, _, last = read_geometry(k[0])
            return s0, min(last + BLOCKLEN, self.cap_nsamples)
        for attempt in range(2):
            lo, reach, _, _ = self.ctx.stream_window()
            n = 0
            for k in keys:
                a, b = span(k)
                if a < lo or b > reach:
                    break
                n += 1
            if n or self.pending or attempt or not keys:
                return keys[:n]
            self.stats['stream_seeks'] = self.stats.get('stream_seeks', 0) + 1
            self.ctx.stream_seek(max(0, span(keys[0])[0] - STREAM_MARGIN))
        return keys[:0]

    def use_resident_capture(self, fmt, nsamples):
        """The capture already lives in this context's HBM (e.g. Context.synth)."""
        self.stream = False
        self.window = None
        self.fmt, self.cap_nsamples = fmt, nsamples
        self.cap_bytes = bytes_for_samples(fmt, nsamples)
        self._reset_cache()

    def _reset_cache(self):
        self.cache, self.hints, self._hint_keys = {}, {}, []
        self._probe_starts = []
        self.plan_located = 0
        self.full_keys = set()             # reads that came back FS_VCUT (decoded again in full)

    # ---- forward simulator (plans the next GPU launch) ---------------------------
    def _next_known(self, start, info):
        """readfield's next position for a decoded read (lddecode_core.py:1204-1212)."""
        nxt = start + info.nextfieldoffset
        if info.status != native.FS_VALID:
            if info.npeaks < 100:
                nxt = start + (self.rf.freq_hz * 10)
            elif info.nvsync == 0:
                nxt = start + (self.rf.freq_hz * 1)
        return nxt

    def _hint_key(self, start):
        import bisect
        ks = self._hint_keys
        i = bisect.bisect_left(ks, start - 4096)
        best = None
        while i < len(ks) and ks[i] <= start + 4096:
            if best is None or abs(ks[i] - start) < abs(best - start):
                best = ks[i]
            i += 1
        if best is None:
            return None
        nx, inf = self.hints[best]
        return (best, nx, inf.status, inf.istop, inf.vbi_framenr, inf.nvsync, [tuple(inf.vsync[q]) for q in range(min(inf.nvsync, 3))])

    def _hint_ahead(self, start):
        """The next field start seen by a decoded read that starts inside the field starting
        at `start` (after it by less than half a field; valid or short) and lands about one
        field after it: a read anywhere before a field's vsync finds the same next field
        (the boot launch's nominal-spacing guesses, tools/boot_probe.py: reads at 799,232 /
        1,600,353 / 2,399,232 of the PAL bench capture report the chain's 1,311,073 /
        2,109,793 / 2,911,072).  None if there is none."""
        import bisect
        ks, f = self._hint_keys, self.field_nom
        i = bisect.bisect_right(ks, start + 4096)
        while i < len(ks) and ks[i] < start + f // 2:
            nx, inf = self.hints[ks[i]]
            if inf.status in (native.FS_VALID, native.FS_SHORT) and 0.95 * f < nx - start < 1.05 * f:
                return nx
            i += 1
        return None

    def _hint(self, start):
        """(next start, field info) of the decoded read nearest `start` within 4096 samples, or None.

        Sync peaks, field parity and VBI are signal-locked: a read a few samples
        away sees the same field and lands on the same next-field position."""
        import bisect
        ks = self._hint_keys
        i = bisect.bisect_left(ks, start - 4096)
        best = None
        while i < len(ks) and ks[i] <= start + 4096:
            if best is None or abs(ks[i] - start) < abs(best - start):
                best = ks[i]
            i += 1
        return None if best is None else self.hints[best]

    def _plan(self, nextsample, mtf, last_framenr, isclv, firstframe, want, hist, frames_left=None):
        """Simulate the replay from a frame checkpoint; return up to `want` undecoded keys it will need.
        frames_left: the decode stops after this many more frames (lddecode.py:49,88 num_frames),
        so reads past that frame are never needed."""
        new, seen, chain = [], set(), []
        self.plan_complete = False         # the walk reached the decode's end (its last frame, EOF)
        located, guessing = 0, False   # leading steps resolved by a decoded read (hit or hint)
        self.plan_guessed = guessed = set()      # new keys whose start came from a prediction
        starts = list(hist)
        # the replay stops once the last read's fd.tell() + 1.05 frames passes the
        # file size (lddecode.py:89): plan at most the rest of that frame beyond it
        bpf = self.rf.samples_per_frame * 5 // 4
        limit = (self.cap_bytes - bpf * 1.05) if self.cap_bytes is not None else None
        past_limit = 0
        sample, cur_mtf, fr = int(nextsample), mtf, last_framenr
        prev_top = None
        steps = 0
        nframes = 0
        while len(new) < want and steps < 8 * want and (frames_left is None or nframes < frames_left):
            fieldcount = 0
            last = None
            while fieldcount < 2 and steps < 8 * want:
                steps += 1
                key = (int(sample), cur_mtf)
                hit = self.cache.get(key)
                if hit is None and key not in seen and key not in self.inflight and not self._probe_covers(key):
                    seen.add(key)
                    new.append(key)
                    if guessing:
                        guessed.add(key)
                    if len(new) >= want:
                        self.plan_located = located
                        return new, chain
                    if self.cap_nsamples is not None and read_geometry(key[0])[2] + BLOCKLEN > self.cap_nsamples:
                        self.plan_located = located
                        self.plan_complete = True
                        return new, chain     # this read's last block passes the capture end (EOF)
                    if limit is not None and loader_tell(self.fmt, read_geometry(key[0])[2], self.cap_bytes) > limit:
                        past_limit += 1
                        if past_limit > 3:
                            self.plan_located = located
                            self.plan_complete = True
                            return new, chain
                if hit is not None:
                    chain.append(key)
                    if not guessing:
                        located += 1
                    info = hit[1]
                    if info.status == native.FS_EOF or info.status == native.FS_CRASH:
                        self.plan_located = located
                        self.plan_complete = True
                        return new, chain
                    nxt = self._next_known(key[0], info)
                    valid = info.status == native.FS_VALID
                    istop = bool(info.istop) if valid else None
                    fnr = info.vbi_framenr if valid and info.vbi_framenr != native.VBI_NONE else None
                    clv = bool(info.vbi_isclv) if valid else isclv
                else:
                    h = self._hint(key[0])
                    if h is not None and h[1].status == native.FS_VALID:
                        # a decoded read of the same field: its next start, parity and VBI
                        if not guessing:
                            located += 1
                        nxt, hinfo = h
                        valid = True
                        istop = bool(hinfo.istop)
                        fnr = hinfo.vbi_framenr if hinfo.vbi_framenr != native.VBI_NONE else None
                        clv = bool(hinfo.vbi_isclv)
                    elif (not guessing and self.boot_ahead and len(hist) < self.period + 2
                          and (ha := self._hint_ahead(key[0])) is not None):
                        # boot: a decoded read later in this field (one of the boot launch's
                        # guesses at the nominal field spacing) already saw where the next
                        # field starts
                        located += 1
                        nxt = ha
                        valid = True
                        istop = (not prev_top) if prev_top is not None else self.sysp.topfirst
                        fnr = (fr + 1) if (fr is not None and not isclv) else None
                        clv = isclv
                    else:
                        guessing = True
                        if h is not None:
                            nxt = h[0]
                        elif len(starts) >= self.period - 1:
                            # r_{k+1} = r_{k+1-mP} + mD: P fields span D samples exactly
                            nxt = self._grid_next(starts)
                        else:
                            nxt = key[0] + self.field_nom
                        valid = True
                        istop = (not prev_top) if prev_top is not None else self.sysp.topfirst
                        fnr = (fr + 1) if (fr is not None and not isclv) else None
                        clv = isclv
                sample = nxt
                if not valid:
                    continue
                starts.append(key[0])          # valid field starts only (the periodic ones)
                prev_top = istop
                if istop == self.sysp.topfirst:
                    fieldcount = 1
                elif fieldcount == 1:
                    fieldcount = 2
                last = (fnr, clv)
                if self.trace is not None:
                    hk = None if hit is not None else self._hint_key(key[0])
                    self.trace.append((key, hit is not None, istop, fnr, fieldcount, nxt, hk))
            if last is None:
                break
            nframes += 1
            fnr, clv = last
            isclv = clv
            if fnr is not None:
                fr = fnr
                if not clv:
                    newmtf = 1 - (fnr / 10000)
                    if newmtf < 0:
                        newmtf = 0
                    cur_mtf = newmtf
            firstframe = False
        self.plan_located = located
        self.plan_complete = frames_left is not None and nframes >= frames_left
        return new, chain

    def _grid_next(self, starts, votes=None):
        """The next read start on the capture's field grid, r_{k+1} = r_{k+1-mP} + mD, voted
        over m = 1..votes (the most common value; ties go to the smallest m).  A read start
        is the absolute position of a sync peak found by argmax on a noisy channel
        (lddecode_core.py:1204, Field.nextfieldoffset): grid + an independent +-1..2 sample
        jitter (PAL: r[k+2] - r[k] = 1,600,000 +- 1 about one step in ten).  m = 1 alone
        carries one jittered start into every P-th prediction after it (half of a 96-read
        PAL launch wasted, profiles/r04_c_pal_waste_10s.txt); the vote keeps it to that read."""
        P, D = self.period, self.period_samples
        votes = votes or self.grid_votes
        if votes == 1:
            return starts[-(P - 1)] + D         # the planner's hot path (once per guessed read)
        counts, best, bestc = {}, None, 0
        for m in range(1, votes + 1):
            j = m * P - 1
            if j > len(starts):
                break
            c = starts[-j] + m * D
            counts[c] = counts.get(c, 0) + 1
            if counts[c] > bestc:
                best, bestc = c, counts[c]
        return best

    def _launch(self, keys, protect):
        """Decode `keys` now (launch and wait for everything outstanding)."""
        while not self._launch_async(keys, protect):
            self._launch_wait()
        while self.pending:
            self._launch_wait()

    def _launch_async(self, keys, protect):
        """Start decoding `keys` into free slots, evicting least-recently-used cache
        entries not in `protect` (the reads the replay is about to consume) as
        needed; _launch_wait() adds the records of the oldest launch to the cache.
        Slots of launches still in flight are never reused."""
        if self.stream:
            keys = self._stream_fit(keys)
            if not keys:
                if self.pending:
                    return False            # the ring moves on once the replay releases
                raise RuntimeError('stream: a read does not fit the ring (ring too small for one read)')
        used = {v[0] for v in self.cache.values()}
        for _, sl in self.pending:
            used.update(sl)
        free = [s for s in range(self.capacity) if s not in used]
        if len(free) < len(keys):
            ss = self._staged_slots
            for k in [k for k in self.cache if k not in protect and self.cache[k][0] not in ss][:len(keys) - len(free)]:
                free.append(self.cache.pop(k)[0])      # oldest first (insertion / touch order)
            keys = keys[:len(free)]
        if not keys:
            if self.pending:
                return False                # every free slot is spoken for: wait for a launch first
            raise RuntimeError('read cache full (capacity %d)' % self.capacity)
        slots = free[:len(keys)]
        t0 = time.perf_counter()
        if self.probe_mode == 'auto' and not self.probe:
            j = self.stats.get('jitter_misses', 0)
            self.probe = j > 3 and j > 0.01 * self.stats['reads_used']
        # (not the very first launch: its guesses at the nominal field spacing are not near
        # field starts, they only locate the first fields)
        probe = self.probe and bool(self.plan_guessed) and bool(self._hint_keys)
        full = None
        if self.full_keys or probe:
            full = [(native.READ_FULL if k in self.full_keys else 0) |
                    (native.READ_PROBE if probe and k in self.plan_guessed and k not in self.full_keys else 0)
                    for k in keys]
        back = self.ctx.decode_reads_async([k[0] for k in keys], [k[1] for k in keys], slots, full)
        if back is not None:
            full = back
        if probe:
            # only the reads the library actually probed (a probe block outside the
            # resident capture is skipped, its flag cleared)
            import bisect
            for k, f in zip(keys, full):
                if f & native.READ_PROBE:
                    bisect.insort(self._probe_starts, k)
                    self.stats['probes'] = self.stats.get('probes', 0) + 1
        self.stats['gpu_s'] += time.perf_counter() - t0
        if self.htrace is not None:
            self.htrace.append((t0, 'launch', len(keys)))
        self.stats['batches'] += 1
        self.stats['reads'] += len(keys)
        self.pending.append((keys, slots))
        self.inflight.update(keys)
        return True

    def _launch_wait(self):
        if not self.pending:
            return
        dh = self.stats.setdefault('inflight_at_wait', {})
        dh[len(self.pending)] = dh.get(len(self.pending), 0) + 1
        keys, slots = self.pending.pop(0)
        t0 = time.perf_counter()
        infos = self.ctx.decode_reads_wait()
        self.stats['wait_s'] = self.stats.get('wait_s', 0.0) + time.perf_counter() - t0
        if self.htrace is not None:
            self.htrace.append((t0, 'wait', len(keys)))
            self.htrace.append((time.perf_counter(), 'waited', len(keys)))
        self.inflight.difference_update(keys)
        import bisect
        if self._probe_starts:
            for k in keys:
                i = bisect.bisect_left(self._probe_starts, k)
                if i < len(self._probe_starts) and self._probe_starts[i] == k:
                    del self._probe_starts[i]
        for k, sl, inf in zip(keys, slots, infos):
            if inf.readsample != k[0]:
                # its probe moved it: the read is the one at its actual start
                self.stats['probe_moved'] = self.stats.get('probe_moved', 0) + 1
                k = (int(inf.readsample), k[1])
                if k in self.cache:
                    continue                # decoded already (this slot stays free)
            if inf.status == native.FS_MIGRATED:
                # the demod's park was overwritten under it (compute-wave save/restore on a
                # shared GPU): the read is void and stays undecoded; the replay's miss decodes it again
                self.stats['migrated'] = self.stats.get('migrated', 0) + 1
                continue
            if inf.status == native.FS_VCUT:
                # its field reaches past the video cut: void, and decoded again in full
                self.stats['vcut_redo'] = self.stats.get('vcut_redo', 0) + 1
                self.full_keys.add(k)
                continue
            self.cache[k] = (sl, inf)
            if inf.status in (native.FS_VALID, native.FS_SHORT):
                if k[0] not in self.hints:
                    bisect.insort(self._hint_keys, k[0])
                self.hints[k[0]] = (k[0] + inf.nextfieldoffset, inf)
        if len(self._hint_keys) > 4096:           # keep the hint index bounded
            for s in self._hint_keys[:-2048]:
                self.hints.pop(s, None)
            self._hint_keys = self._hint_keys[-2048:]

    def _probe_covers(self, key):
        """A probed read in flight will land on this start if it is the sync peak within
        the probe's window of that read's predicted start (same MTF)."""
        ps = self._probe_starts
        if not ps:
            return False
        import bisect
        w = self.probe_win
        i = bisect.bisect_left(ps, (key[0] - w, float('-inf')))
        while i < len(ps) and ps[i][0] <= key[0] + w:
            if ps[i][1] == key[1]:
                return True
            i += 1
        return False

    def _note_miss(self, key):
        """Diagnostics: how far the nearest decoded read was from the one the replay needed."""
        self.stats['misses'] = self.stats.get('misses', 0) + 1
        best = None
        for (s, m) in self.cache:
            d = s - key[0]
            if abs(d) <= 200000 and (best is None or abs(d) < abs(best[0])):
                best = (d, m == key[1])
        if best is not None and best[1] and 0 < abs(best[0]) <= self.probe_win:
            # a read of this field was decoded a few samples off: the start jitters
            self.stats['jitter_misses'] = self.stats.get('jitter_misses', 0) + 1
        h = self.stats.setdefault('miss_log', [])
        if len(h) < 64:
            h.append(best)

    def demod_isolated(self, iters=10, variants=(0,), reads=None):
        """(reads, ms per launch) of the demod alone over `reads` (default `batch`) decoded reads,
        `iters` launches back to back (the benchmark's roofline leg).  The reads are the
        most recent cached reads whose field decoded (FS_VALID): every block of such a
        read lies inside the resident capture, so each launch demodulates whole reads
        (a sharded rank's speculative reads past its window are FS_EOF and their
        workgroups would return at once; the library refuses them).  The reads' demod
        outputs are recomputed in place, so the read cache is dropped.  `variants`
        (native.Context.demod_isolated) run in turn over the same reads; with more than
        one the ms figure is a list in that order."""
        slots = [sl for sl, inf in reversed(list(self.cache.values())) if inf.status == native.FS_VALID]
        want = self.batch if reads is None else min(int(reads), self.batch)
        slots = slots[:want]
        if len(slots) < want:
            raise RuntimeError('demod_isolated: %d decoded reads cached, %d needed' % (len(slots), want))
        try:
            ms = [self.ctx.demod_isolated(slots, iters, v) for v in variants]
        finally:
            self._reset_cache()
        return len(slots), (ms[0] if len(ms) == 1 else ms)

    # ---- reference control flow --------------------------------------------------
    def _get(self, readsample, mtf, audio_offset):
        key = (int(readsample), mtf)
        self.requested.append(key)
        hit = self.cache.get(key)
        if hit is None:
            raise Miss(key)
        self.cache[key] = self.cache.pop(key)         # LRU touch
        slot, info = hit
        if info.status == native.FS_CRASH:
            raise ReferenceCrash('reference would raise at read %d' % readsample)
        if info.status == native.FS_EOF and self.stream:
            if read_geometry(key[0])[2] + BLOCKLEN <= self.cap_nsamples:
                raise RuntimeError('stream: read %d came back FS_EOF inside the capture' % key[0])
        if info.status == native.FS_EOF and self.window is not None:
            s0, _, last = read_geometry(key[0])
            if s0 < self.window[0] or last + BLOCKLEN > self.window[1]:
                if last + BLOCKLEN <= self.cap_nsamples:
                    raise WindowMiss('read %d needs samples outside the window %s' % (key[0], self.window))
        f = GPUField(info, slot, int(readsample), mtf, audio_offset, self.sysp, None)
        f.tidx = len(self.transitions)       # audio-offset transitions before this field
        return f

    def readfield(self, sample):
        """lddecode_core.py:1194-1223."""
        readsample = sample
        while True:
            f = self._get(readsample, self.mtf_level, self.audio_offset)
            self.last_read = readsample
            if f.status == native.FS_EOF:
                return None, None, None
            nextsample = readsample + f.nextfieldoffset
            if not f.valid:
                if f.npeaks < 100:
                    nextsample = readsample + (self.rf.freq_hz * 10)
                elif f.nvsync == 0:
                    nextsample = readsample + (self.rf.freq_hz * 1)
            f.nextsample = nextsample
            self.field_log.append(f)
            if not f.valid:
                readsample = nextsample
            else:
                return f, readsample, nextsample

    def mergevbi(self, fields):
        merged = dict(fields[0].vbi)
        for k in merged:
            if fields[1].vbi[k] is not None:
                merged[k] = fields[1].vbi[k]
        if merged['seconds'] is not None:
            fps = self.sysp.clvfps
            merged['framenr'] = merged['minutes'] * 60 * fps + merged['seconds'] * fps + merged['clvframe']
        return merged

    def readframe(self, sample, firstframe=False, cav=False):
        """lddecode_core.py:1254-1311 (formatoutput/audio deferred to the batch flush).
        cav: the reference's CAV framing (:1273-1275), used by findframe."""
        fieldcount = 0
        fields = [None, None]
        audio = []
        f = None
        while fieldcount < 2:
            f, readsample, nextsample = self.readfield(sample)
            if f is not None:
                if f.istop:
                    fields[0] = f
                else:
                    fields[1] = f
                if ((not cav and (f.istop == self.sysp.topfirst)) or
                        (cav and (f.vbi['framenr'] or f.vbi['minutes']))):
                    fieldcount = 1
                elif fieldcount == 1:
                    fieldcount = 2
                if fieldcount or not firstframe:
                    audio.append(f)
            elif readsample is None:
                return None
            sample = nextsample
        if len(audio):
            self.audio_offset = f.audio_next_offset
            self.transitions.append(int(f.linecount))   # offset -> next(offset, linecount)
        vbi = self.mergevbi(fields)
        self.vbi = vbi
        fv = f.vbi
        self.last_isclv = bool(fv['isclv'])
        fnr = fv['framenr']
        if fnr is not None:
            self.last_framenr = fnr
        if not fv['isclv'] and fnr is not None:
            newmtf = 1 - (fnr / 10000)
            if newmtf < 0:
                newmtf = 0
            oldmtf = self.mtf_level
            self.mtf_level = newmtf
            if abs(newmtf - oldmtf) > .1:
                return self.readframe(sample, firstframe, cav)
        return FrameOut(top=fields[0], bottom=fields[1], audio_fields=audio, vbi=vbi, nextsample=sample)

    # ---- seek (lddecode_core.py:1338-1378) -----------------------------------------
    _STATE = ('mtf_level', 'audio_offset', 'last_framenr', 'last_isclv', 'last_read', 'vbi')

    def _resolve(self, fn, max_launches=64):
        """Run a replay step; decode whatever reads it misses (a few speculative reads
        ahead of each) and re-run it from the same state until it completes."""
        for _ in range(max_launches):
            saved = {k: getattr(self, k, None) for k in self._STATE}
            nt = len(self.transitions)
            self.requested, self.field_log = [], []
            try:
                return fn()
            except Miss as m:
                for k, v in saved.items():
                    setattr(self, k, v)
                del self.transitions[nt:]
                keys, _ = self._plan(m.key[0], m.key[1], self.last_framenr, self.last_isclv, False, 4, [])
                if m.key not in keys:
                    keys = [m.key] + keys[:3]
                self._launch(keys, set(self.requested))
        raise RuntimeError('replay step did not converge after %d launches' % max_launches)

    def findframe(self, target, nextsample=0, log=print):
        """Sample number of frame `target` (lddecode_core.py:1338-1378), on a fresh
        framer (mtf 1, audio offset 0).  Returns None where the reference does."""
        spf = int(self.rf.freq_hz / self.sysp.fps)
        self.mtf_level, self.audio_offset = 1, 0
        self.last_framenr, self.last_isclv, self.last_read = None, False, None
        self.vbi = {'framenr': None}
        self.transitions = []
        iscav = False
        tolerance = 0
        rv = None
        retry = 5
        while self.vbi['framenr'] is None and retry:
            rv = self._resolve(lambda: self.readframe(nextsample, False, cav=False))
            if rv is None:
                raise ReferenceCrash('findframe: end of capture (reference: TypeError on rv[2])')
            log(rv.nextsample, self.vbi)
            if self.vbi['isclv']:
                tolerance = 1
            else:
                tolerance = 0
                iscav = True
            nextsample = rv.nextsample + (self.rf.freq_hz * 10)
            retry -= 1
        if retry == 0 and self.vbi['framenr'] is None:
            log("SEEK ERROR: Unable to find a usable frame")
            return None
        retry = 5
        while np.abs(target - self.vbi['framenr']) > tolerance and retry:
            offset = (spf * (target - 1 - self.vbi['framenr']))
            nextsample = rv.nextsample + offset
            rv = self._resolve(lambda: self.readframe(nextsample, False, cav=iscav))
            if rv is None:
                raise ReferenceCrash('findframe: end of capture (reference: TypeError on rv[2])')
            log(self.vbi)
            retry -= 1
        if np.abs(target - self.vbi['framenr']) > tolerance:
            log("SEEK WARNING: seeked to frame {0} instead of {1}".format(self.vbi['framenr'], target))
        return nextsample

    # ---- main loop (lddecode.py:39-107) ------------------------------------------
    def _tell(self):
        if self.last_read is None:
            return 0
        return loader_tell(self.fmt, read_geometry(self.last_read)[2], self.cap_bytes)

    def decode(self, start_frame=0, length=None, sink=None, comb=False, comb_sink=None, start_sample=None,
               stop_sample=None, keep_from=None, firstframe=True, archive=False, init_state=None, comb3d=None,
               resume=False):
        """Decode frames; sink(frame_u16, pcm_i16, meta) per frame (None: frames stay in HBM).
        The frame (and comb_sink's rgb48) handed to the sinks is a view of a pinned output
        buffer that a later batch reuses: copy it to keep it past the call.

        comb: also run the 2D NTSC comb (comb-ntsc.cxx dim=2) on every frame, in
        order, as one comb process; comb_sink(rgb48) receives each 480x744x3
        frame (None with sink=None: the rgb frames stay in HBM).  comb3d = (core_ire,
        range_ire) runs the 3D comb without optical flow instead (comb-ntsc -d 3 -F;
        negative values: the -F defaults); it outputs every frame but the first and
        the last, one frame late, and needs a sink.
        Field-group sharding (ldgpu/shard.py) hooks: start at start_sample; stop
        before a frame that would start at or after stop_sample; frames starting
        before keep_from are decoded (they lock the read / MTF chains) but not
        output; firstframe: whether the first frame is the capture's first
        (lddecode.py:90); archive: keep each output field's audio inputs in the
        field archive instead of computing its 48 kHz audio (the shard's audio
        time offset is known only after the exchange), see self.shard_frames.
        resume: continue the previous decode (same archive / shard_frames / audio-offset
        transitions / comb state / fd.tell()) from start_sample, with the chain state in
        init_state -- a shard extending its range past its nominal end (ShardedDecode.extend).
        Returns the number of frames decoded."""
        self.comb, self.comb_sink, self.comb3d = comb, comb_sink, (comb3d if comb else None)
        if self.comb3d is not None and sink is None:
            raise ValueError('the 3D comb runs on host frames (a sink is required)')
        if not resume:
            self.archive, self.arch_next, self.shard_frames = archive, 0, []
            self.transitions = []
            if comb:
                self.ctx.comb_reset()
        spf = self.rf.samples_per_frame
        bpf = spf * 5 // 4                     # (sic) 10-bit packing assumed, lddecode.py:42
        size = self.cap_bytes
        if (size // bpf - start_frame) < 2:
            raise ValueError('start frame is past end of file')
        num_frames = length if length is not None else size // bpf - start_frame
        if not resume:
            self.mtf_level, self.audio_offset = 1, 0
            self.last_framenr, self.last_isclv, self.last_read = None, False, None
            self.frame_numbers, self.pcm_samples, self.last_meta = [], 0, None
        for k, v in (init_state or {}).items():        # chain state handed over by a previous shard
            setattr(self, k, v)
        nextsample = start_frame * spf if start_sample is None else start_sample
        # Python's cyclic collector off for the decode: a full (oldest-generation)
        # collection over the read cache and hint index stalls the host for
        # 10-25 ms, during which the GPU runs dry (measured: one such gap per
        # 60 s decode, ~5% of a 2-step bench).  The loop collects the young
        # generations itself every few batches, so cyclic garbage stays bounded.
        gc_on = gc.isenabled()
        gc.disable()
        # Everything alive before the decode (the interpreter's, torch's and numpy's
        # objects: most of the heap) goes to the permanent generation for the call,
        # so the loop's rare oldest-generation collection scans only what the decode
        # made: it took ~36 ms with the whole heap (one step in 16 of the bench, which
        # runs 32 launches per step, r04_zj's checks.step_ms), the demod idle meanwhile
        froze = gc.get_freeze_count() == 0 and os.environ.get('LDG_GC_FREEZE', '1') == '1'
        if froze:
            gc.freeze()
        try:
            return self._decode_loop(start_frame, num_frames, nextsample, spf, bpf, size, sink, stop_sample,
                                     keep_from, firstframe)
        finally:
            try:
                while self.pending:             # no launch outlives the call (an exception included)
                    self._launch_wait()
                try:
                    self._finish_flush()
                    self._emit_pending()
                finally:
                    self._out_pending = None
                    self._staged, self._staged_slots = None, set()
                    self.ctx.sync()
                    if self.before_ring_reuse is not None:
                        self.before_ring_reuse()   # the sink's writes from the rings are done
                    for ring in self._obufs or ():
                        for b in ring:
                            b.release_retired()
            finally:
                if froze:
                    gc.unfreeze()
                if gc_on:
                    gc.enable()

    def _decode_loop(self, start_frame, num_frames, nextsample, spf, bpf, size, sink, stop_sample, keep_from,
                     firstframe):
        done = 0
        nframes_read = 0
        hist = []
        plan_idle = False
        W, H = self.sysp.outlinelen, self.sysp.frame_lines

        def more(ns):
            return stop_sample is None or ns < stop_sample

        while done < num_frames and self._tell() + bpf * 1.05 <= size and more(nextsample):
            # nothing known about this capture yet: learn the first fields' parity,
            # VBI and sync positions from a small launch before speculating wide
            # (until P + 2 field starts are known the period extrapolation has nothing to use).
            # In steady state keep `depth` launches in flight: the newer one is planned
            # through the older one's predicted outcomes, so its demod runs on the GPU
            # while the older one's field kernels finish and the host replays.
            steady = len(hist) >= self.period + 2
            if self.boot_wide and not steady:
                # once the last plan walked P + 2 fields on decoded reads (cache hits or
                # hints within 4096 samples), the next fields are located exactly and the
                # period extrapolation is seeded: go wide before the replay catches up.
                # (Counting hints alone went wide on the boot launch's nominal-spacing
                # guesses for PAL, P + 2 = 4, and wasted two whole batches.)
                steady = self.plan_located >= self.period + 2
            depth = self.depth if steady else 1
            launched = 0
            # a walk that found nothing new and reached the decode's end finds nothing new
            # until the replay misses (a read the plan got wrong): skip re-walking the whole
            # decoded chain then (the last batches' drain, ~0.4 ms of host time per batch)
            while len(self.pending) < depth and not plan_idle:
                # boot: the first launch holds P + 2 reads (the first read and P + 1 guesses at the
                # nominal field spacing, whose decoded records locate the next fields exactly when
                # the capture starts near a field start); later boot plans are walked wide and
                # launched wide when this very walk located P + 2 fields on decoded reads, else
                # cut to the narrow size (a walk's first keys do not depend on how far it goes)
                narrow = min(self.batch, 8 if self._hint_keys else self.period + 2)
                probe_wide = not steady and self.boot_wide and bool(self._hint_keys)
                want = self.batch if (steady or probe_wide) else narrow
                tp = time.perf_counter()
                plan, chain = self._plan(nextsample, self.mtf_level, self.last_framenr, self.last_isclv, done == 0,
                                         want, hist, frames_left=num_frames - done + 2)
                if probe_wide:
                    if self.plan_located >= self.period + 2:
                        steady, depth = True, self.depth
                    else:
                        plan = plan[:narrow]
                self.stats['plan_s'] = self.stats.get('plan_s', 0.0) + time.perf_counter() - tp
                if not plan:
                    plan_idle = steady and self.plan_complete and self.plan_idle_skip
                    break
                if not self._launch_async(plan, set(chain)):
                    break
                launched += 1
            self._finish_flush()
            frames = []
            eof = False
            missed = None
            window_miss = None
            t0 = time.perf_counter()
            self.requested = []
            while done + len(frames) < num_frames and self._tell() + bpf * 1.05 <= size and more(nextsample):
                cp = (nextsample, self.mtf_level, self.audio_offset, self.last_framenr, self.last_isclv,
                      self.last_read, len(self.transitions), nframes_read)
                self.field_log = []
                try:
                    fr = self.readframe(nextsample, firstframe and nframes_read == 0)
                except Miss as m:
                    missed = m.key
                    self._note_miss(m.key)
                    (nextsample, self.mtf_level, self.audio_offset, self.last_framenr, self.last_isclv,
                     self.last_read, nt, nframes_read) = cp
                    del self.transitions[nt:]
                    break
                except WindowMiss as wm:
                    # no launch can fix this one: back to the frame's checkpoint, emit the
                    # frames before it, then raise with the resume point
                    (nextsample, self.mtf_level, self.audio_offset, self.last_framenr, self.last_isclv,
                     self.last_read, nt, nframes_read) = cp
                    del self.transitions[nt:]
                    window_miss = WindowMiss(str(wm), resume_at=int(nextsample))
                    break
                if fr is None:
                    eof = True
                    break
                nframes_read += 1
                fr.start = nextsample
                fr.tstart = cp[6]
                fr.mtf0 = cp[1]                 # the MTF this frame's readframe began with (the chain state)
                # the framer's state after this frame (the next decode's init: shard.py end_state)
                fr.end = (self.mtf_level, self.last_framenr, self.last_isclv, self.last_read, len(self.transitions))
                nextsample = fr.nextsample
                if keep_from is not None and fr.start < keep_from:
                    continue                    # warm-up frame: chains only
                fr.field_objs = self.field_log
                fr.log = field_log_lines(self.field_log, self.sysp.name == 'NTSC') if self.frame_log else None
                fr.index = done + len(frames)
                frames.append(fr)
                hist = (hist + [x.readsample for x in self.field_log if x.valid])[-self.hist_len:]
            self.stats['replay_s'] += time.perf_counter() - t0
            if missed is not None or window_miss is not None:
                plan_idle = False
            if self.stream:
                # the replay never reads before its checkpoint again: the reader may refill that
                self.ctx.stream_release(nextsample - STREAM_MARGIN)
            if self.stats['batches'] % 32 == 0:
                gc.collect(1)
            if self.stats['batches'] % 512 == 0:
                gc.collect(2)                    # the oldest generation too, rarely (long captures)
            tf = time.perf_counter()
            if self.htrace is not None:
                self.htrace.append((t0, 'replay', len(frames)))
                self.htrace.append((tf, 'flush', len(frames)))
            self._flush(frames, W, H, sink)
            self.stats['flush_s'] = self.stats.get('flush_s', 0.0) + time.perf_counter() - tf
            if self.htrace is not None:
                self.htrace.append((time.perf_counter(), 'flushed', len(frames)))
            done += len(frames)
            self.stats['reads_used'] += sum(len(f.field_objs) for f in frames)
            if window_miss is not None:
                raise window_miss
            if eof or (not frames and not launched and not self.pending):
                break
            self._launch_wait()                 # the oldest launch: the replay continues into it
            # the replay stopped at a read a newer launch holds: it cannot move before
            # that launch lands, so wait for it rather than plan further ahead (each such
            # plan pins another batch of cached reads; a long capture once filled the cache)
            while (self.miss_drain and missed is not None and (missed in self.inflight or self._probe_covers(missed))
                   and self.pending):
                self.stats['drain_waits'] = self.stats.get('drain_waits', 0) + 1
                self._launch_wait()
                while (self.drain_refill and steady and (missed in self.inflight or self._probe_covers(missed))
                       and len(self.pending) < depth):
                    plan, chain = self._plan(nextsample, self.mtf_level, self.last_framenr, self.last_isclv,
                                             done == 0, self.batch, hist, frames_left=num_frames - done + 2)
                    if not plan or not self._launch_async(plan, set(chain)):
                        break
                    self.stats['drain_refills'] = self.stats.get('drain_refills', 0) + 1
        return done

    def _flush(self, frames, W, H, sink):
        if not frames:
            return
        tops = [f.top.slot for f in frames]
        bots = [f.bottom.slot for f in frames]
        if sink is None:
            # benchmark mode: .tbc frames (and their comb output) stay in HBM
            self.ctx.assemble_frames_device(tops, bots)
            pics = None
            if self.comb:
                self.ctx.comb_async(len(frames))          # overlaps the next batch's decode
        elif not self.comb or self.comb3d is None:
            # frames (and the fused 2D comb) go to pinned host buffers asynchronously on the
            # output stream (ldg_output_async); the sink sees them at the next flush, after
            # ldg_output_wait -- no host round trip of the frames through the comb
            rh, rw = (576, 1057) if self.sysp.name == 'PAL' else (self.ctx.comb_lines, self.ctx.comb_width)
            if self._obufs is None:
                # two rings; one that grows keeps its old memory until the decode ends
                # (the sink's views of it stay valid: PinnedBuffer.release_retired)
                from .native import PinnedBuffer
                self._obufs = [(PinnedBuffer(), PinnedBuffer()) for _ in range(2)]
            tb, rb = self._obufs[self._oring]
            self._oring ^= 1
            n = len(frames)
            if self.before_ring_reuse is not None:
                self.before_ring_reuse()           # (a sink that writes its frames later, lddecode.py Writer)
            pics = tb.view(n * H * W).reshape(n, H * W)
            rgb = rb.view(n * rh * rw * 3).reshape(n, rh, rw, 3) if self.comb else None
            self.ctx.output_async(tops, bots, pics, rgb)
            pics = (pics, rgb)
        else:
            pics = self.ctx.assemble_frames(tops, bots, W, H)
            if self.comb:
                if self.sysp.name == 'PAL':
                    rgb = self.ctx.comb_pal(pics)             # build-defined PAL Y/C (row F2)
                elif self.comb3d is None:
                    rgb = self.ctx.comb_ntsc(pics)
                else:
                    rgb = self.ctx.comb_ntsc3d(pics, *self.comb3d)
                if self.comb_sink:
                    for r in rgb:
                        self.comb_sink(r)
        af = [(fr_i, x) for fr_i, fr in enumerate(frames) for x in fr.audio_fields]
        if self.archive:
            # audio deferred: archive the fields' audio inputs, record the chain positions
            if af:
                self.ctx.archive_fields([x.slot for _, x in af], self.arch_next)
            by_frame = [[] for _ in frames]
            for j, (fi, x) in enumerate(af):
                by_frame[fi].append((self.arch_next + j, x.tidx))
            for i, fr in enumerate(frames):
                ents = by_frame[i]
                self.shard_frames.append({'index': fr.index, 'start': int(fr.start), 'tstart': fr.tstart,
                                          'nextsample': int(fr.nextsample),
                                          'audio': ents, 'vbi': dict(fr.vbi), 'fields': fr.fields,
                                          'mtf': float(fr.top.mtf_level), 'mtf0': float(fr.mtf0), 'end': fr.end})
            self.arch_next += len(af)
            af = []
        # the audio runs while the host plans and replays the next batch: this batch's
        # frames go to the sink at the next flush (or at the end of the decode)
        self._staged = (frames, pics, af, sink)
        if self.defer_flush:
            self._staged_slots = set(tops) | set(bots) | {x.slot for _, x in af}
        else:
            self._finish_flush()

    def _finish_flush(self):
        """Hand the previous batch to the sink (waiting for its audio and output) and
        launch the staged batch's audio."""
        if self._staged is None:
            return
        staged, self._staged = self._staged, None
        self._emit_pending()
        af = staged[2]
        self.ctx.field_audio_async([x.slot for _, x in af], [x.audio_offset for _, x in af])
        self._staged_slots = set()
        self._out_pending = staged

    def _emit_pending(self):
        """Collect the outstanding batch's audio and hand its frames to the sink."""
        if self._out_pending is None:
            return
        frames, pics, af, sink = self._out_pending
        self._out_pending = None
        pcm, counts, _ = self.ctx.field_audio_collect()
        if isinstance(pics, tuple):
            self.ctx.output_wait()                # this batch's frames / rgb48 are on the host now
            pics, rgb = pics
            if rgb is not None and self.comb_sink:
                for r in rgb:
                    self.comb_sink(r)
        per_frame = [[] for _ in frames]
        for j, (fr_i, x) in enumerate(af):
            if counts[j] < 0:
                raise ReferenceCrash('audio index error (reference: field invalid)')
            per_frame[fr_i].append(pcm[j, :2 * counts[j]])
        def meta_of(fr):
            return {'frame': fr.index, 'vbi': dict(fr.vbi), 'nextsample': int(fr.nextsample), 'fields': fr.fields}
        for i, fr in enumerate(frames):
            self.frame_numbers.append(fr.vbi['framenr'])
            if fr.log:
                self.frame_log(fr.log)
            if sink:
                audio = np.concatenate(per_frame[i]) if per_frame[i] else np.zeros(0, dtype=np.int16)
                meta = meta_of(fr)
                self.last_meta = meta
                sink(pics[i], audio, meta)
            else:
                self.pcm_samples += sum(a.size for a in per_frame[i])
        if frames and not sink:
            self.last_meta = meta_of(frames[-1])     # (no sink: only the last frame's metadata is read)
