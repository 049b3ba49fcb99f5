"""CPU tests of the decoder's speculative planner and replay (ldgpu/decoder.py) on a
model capture: the GPU context is replaced by a fake whose "decode" of a read is
a closed-form NTSC field model, so thousands of frames run in seconds without a GPU.

The model: field k starts at P_k (the steady-state NTSC read chain at 40 MSPS,
3 frames = 4,004,000 samples exactly); a read within 4096 samples of P_k decodes
field k (top when k is even, picture number 2 + k // 2 on both fields) and its
next-field offset lands on P_{k+1} -- plus one sample for some read starts, so the
chain is signal-locked but not every prediction is exact (the case that once
pinned the whole read cache, see test_long_decode_with_mispredictions).  The
reference control flow (Framer.readfield / readframe, lddecode_core.py:1194-1311;
the EOF guard and frame count, lddecode.py:41-49,88-98) is replayed here
sequentially as the expected result.
"""
import numpy as np
import pytest

from ldgpu import decoder as D
from ldgpu import native

P0 = 1052829
CUM = [0, 668605, 1334667, 2003272, 2669334, 3337938]     # field starts within 3 frames
PERIOD = 4004000


def field_start(k):
    return P0 + (k // 6) * PERIOD + CUM[k % 6]


def nearest_field(s):
    k = max(0, int((s - P0) * 6 // PERIOD))
    for j in (k - 1, k, k + 1, k + 2):
        if j >= 0 and abs(field_start(j) - s) <= 4096:
            return j
    return None


def field_jitter(k):
    """jitter='field': field k's start as the chain finds it is off the grid by -2..2
    samples, a property of the signal (PAL's sync peaks, profiles/r04_f_pal_chain.json):
    every read of field k - 1 reports the same start, whatever its own start."""
    return (k * 37) % 5 - 2


def chain_start(k, jitter):
    return field_start(k) + (field_jitter(k) if jitter == 'field' else 0)


def model_read(s, nsamples, jitter):
    """(status, istop, nextfieldoffset, framenr, linecount) of a read starting at s."""
    if s + 1000001 + 16384 > nsamples:
        return native.FS_EOF, 0, 0, None, 0
    k = nearest_field(s)
    if k is None:
        # before the first field: not valid; its next-field offset points at the next field
        j = 0
        while field_start(j) < s:
            j += 1
        return native.FS_NO_VSYNC, 0, field_start(j) - s, None, 0
    if jitter == 'field':
        nfo = chain_start(k + 1, jitter) - s
    else:
        nfo = field_start(k + 1) - s + (1 if jitter and (s % 7 == 3) else 0)
    return native.FS_VALID, int(k % 2 == 0), nfo, 2 + k // 2, 263 if k % 2 == 0 else 262


class FakeCtx:
    """The parts of native.Context the decode loop uses, with model_read as the decode."""
    nsamples = 0
    jitter = False

    def __init__(self, system, device, max_reads=0, max_frames=0):
        self.max_reads = max_reads
        self._pending = []
        self._audio = 0
        self.reads = []
        self.probed = 0

    def set_filters(self, *a):
        pass

    def set_video_cut(self, out_samples):
        pass

    def decode_reads_async(self, starts, mtfs, slots, full=None):
        assert len(set(slots)) == len(slots) and all(0 <= s < self.max_reads for s in slots)
        busy = {s for p in self._pending for s in p[0]}
        assert not busy.intersection(slots), 'slot reused while in flight'
        infos = []
        for i, s in enumerate(starts):
            s = int(s)
            if full is not None and full[i] & native.READ_PROBE:
                # the GPU's start probe: the sync peak (the chain's start) within 0.3 lines
                j = nearest_field(s)
                if j is not None and abs(chain_start(j, self.jitter) - s) <= 760:
                    s = chain_start(j, self.jitter)
                self.probed += 1
            self.reads.append(s)
            st, top, nfo, fnr, lc = model_read(s, self.nsamples, self.jitter)
            f = native.FieldInfo()
            f.readsample = s
            f.status, f.istop, f.nextfieldoffset, f.linecount = st, top, nfo, lc
            f.npeaks, f.nvsync = (400, 2) if st == native.FS_VALID else (400, 1)
            for name in ('vbi_minutes', 'vbi_seconds', 'vbi_clvframe', 'vbi_status'):
                setattr(f, name, native.VBI_NONE)
            f.vbi_framenr = native.VBI_NONE if fnr is None else fnr
            f.vbi_isclv = 0
            infos.append(f)
        self._pending.append((list(slots), infos))

    def decode_reads_wait(self):
        _, infos = self._pending.pop(0)
        return infos

    def assemble_frames_device(self, tops, bots):
        pass

    def comb_reset(self):
        pass

    def field_audio_async(self, slots, offsets):
        self._audio = len(slots)

    def field_audio_collect(self):
        n = self._audio
        return np.zeros((n, 1602), np.int16), [801] * n, [0.0] * n

    def sync(self):
        pass


def reference_chain(nsamples):
    """The reference control flow, sequentially: frames (framenr, first read) until the EOF guard."""
    spf = 1334668                                     # int(40e6 / (30000 / 1001)) + 1
    bpf = spf * 5 // 4
    size = nsamples                                   # u8: one byte per sample
    num_frames = size // bpf
    sample, frames = 0, []
    tell = 0
    while len(frames) < num_frames and tell + bpf * 1.05 <= size:
        fieldcount, first, fnr = 0, None, None
        while fieldcount < 2:
            rs = sample
            while True:
                st, top, nfo, fr, _ = model_read(rs, nsamples, FakeCtx.jitter)
                if st == native.FS_EOF:
                    return frames
                tell = D.loader_tell(0, D.read_geometry(rs)[2], size)
                nxt = rs + nfo
                if st == native.FS_VALID:
                    break
                rs = nxt
            first = rs if first is None else first
            if top:
                fieldcount = 1
            elif fieldcount == 1:
                fieldcount = 2
            fnr = fr
            sample = nxt
        frames.append((fnr, sample))
    return frames


def run_decode(monkeypatch, frames, batch, jitter):
    nsamples = int(field_start(2 * frames + 4)) + 2_000_000
    FakeCtx.nsamples, FakeCtx.jitter = nsamples, jitter
    monkeypatch.setattr(native, 'Context', FakeCtx)
    dec = D.GPUDecoder(system='NTSC', device=0, batch=batch)
    dec.use_resident_capture(0, nsamples)
    n = dec.decode(sink=None)
    return dec, n, nsamples


@pytest.mark.parametrize('jitter,votes', [(False, 1), (True, 1), (True, 8)])
def test_replay_matches_sequential_reference(monkeypatch, jitter, votes):
    """Batched speculative decode == the reference's sequential read chain (frames, numbers, end),
    with the planner's period prediction from the last period (votes 1) or voted over 8."""
    monkeypatch.setenv('LDG_GRID_VOTES', str(votes))
    monkeypatch.setenv('LDG_PROBE', '0')
    dec, n, nsamples = run_decode(monkeypatch, 300, batch=16, jitter=jitter)
    ref = reference_chain(nsamples)
    assert n == len(ref)
    assert dec.frame_numbers == [f for f, _ in ref]
    assert dec.last_meta['nextsample'] == ref[-1][1]
    # every frame after the first two reads is a top + bottom pair of consecutive fields
    assert all(b == a + 1 for a, b in zip(dec.frame_numbers, dec.frame_numbers[1:]))


@pytest.mark.parametrize('refill', ['0', '1'])
def test_long_decode_with_mispredictions(monkeypatch, refill):
    """A long decode whose predictions are sometimes a sample off keeps going: the
    planner waits for the launch holding the read the replay stopped at instead of
    pinning the whole read cache with ever further reads (round-2 fix; before it,
    240 s captures died with 'read cache full' after ~3000 frames).  With the drain
    refill (LDG_DRAIN_REFILL=1) it keeps `depth` launches in flight meanwhile, still
    within the cache."""
    monkeypatch.setenv('LDG_DRAIN_REFILL', refill)
    dec, n, nsamples = run_decode(monkeypatch, 2500, batch=8, jitter=True)
    ref = reference_chain(nsamples)
    assert n == len(ref) and dec.frame_numbers == [f for f, _ in ref]
    assert dec.stats['reads'] < 1.3 * dec.stats['reads_used']


@pytest.mark.parametrize('probe', ['0', '1', 'auto'])
def test_start_probes_follow_a_jittering_chain(monkeypatch, probe):
    """Field starts off the period grid by a couple of samples (a property of the
    signal): without probes every such prediction is decoded twice; with them
    (LDG_PROBE=1, ldg_decode_reads_async2 READ_PROBE) the predicted reads move to the
    chain's starts and nearly every read decoded is used -- and the frames are the
    sequential reference chain's either way."""
    monkeypatch.setenv('LDG_PROBE', probe)
    dec, n, nsamples = run_decode(monkeypatch, 600, batch=16, jitter='field')
    ref = reference_chain(nsamples)
    assert n == len(ref) and dec.frame_numbers == [f for f, _ in ref]
    assert dec.last_meta['nextsample'] == ref[-1][1]
    ratio = dec.stats['reads'] / dec.stats['reads_used']
    if probe == '1':
        assert dec.ctx.probed > 0 and dec.stats.get('probe_moved', 0) > 0
        assert ratio < 1.05, ratio
    elif probe == 'auto':
        # off until the waste passes 5%, then on for the rest of the decode
        assert dec.ctx.probed > 0 and ratio < 1.2, ratio
    else:
        assert ratio > 1.3, ratio


def test_demod_isolated_read_count(monkeypatch):
    """bench.py's roofline leg: `reads` picks how many decoded reads one isolated launch
    demodulates (96 whatever the pipeline's batch), default the batch; too few refuse."""
    monkeypatch.setenv('LDG_PROBE', '0')
    dec, _, _ = run_decode(monkeypatch, 60, batch=16, jitter=False)
    seen = []
    monkeypatch.setattr(dec.ctx, 'demod_isolated', lambda slots, iters, v: seen.append(list(slots)) or 1.0,
                        raising=False)
    cached = dict(dec.cache)
    assert dec.demod_isolated(3, reads=8) == (8, 1.0)
    assert len(seen[-1]) == 8 and len(set(seen[-1])) == 8
    dec.cache.update(cached)
    assert dec.demod_isolated(3, (0, 1)) == (16, [1.0, 1.0])
    assert [len(s) for s in seen[-2:]] == [16, 16]
    with pytest.raises(RuntimeError):
        dec.demod_isolated(3, reads=8)              # the read cache was dropped


def test_frame_metadata_with_and_without_a_sink(monkeypatch):
    """Each frame's metadata lists the fields its readframe read, chained read to read
    (nextsample of one = readsample of the next); the records are built on first use, and
    a decode without a sink keeps only the last frame's metadata -- the same dict as the
    sink run's last one."""
    monkeypatch.setenv('LDG_PROBE', '0')
    frames = 200
    nsamples = int(field_start(2 * frames + 4)) + 2_000_000
    FakeCtx.nsamples, FakeCtx.jitter = nsamples, False
    monkeypatch.setattr(native, 'Context', FakeCtx)
    class HostBuf:                                     # PinnedBuffer without ldg_host_alloc
        def view(self, count):
            return np.zeros(count, np.uint16)

        def release_retired(self):
            pass
    monkeypatch.setattr(native, 'PinnedBuffer', HostBuf)
    dec = D.GPUDecoder(system='NTSC', device=0, batch=16)
    dec.use_resident_capture(0, nsamples)
    dec.ctx.output_async = lambda tops, bots, tbc, rgb=None: None
    dec.ctx.output_wait = lambda: None
    dec.ctx.comb_lines, dec.ctx.comb_width = 480, 744
    metas = []
    n = dec.decode(sink=lambda fr, au, meta: metas.append(meta))
    assert n == len(metas) > 100
    prev = None
    for m in metas:
        assert len(m['fields']) >= 2
        for f in m['fields']:
            if prev is not None:
                assert f['readsample'] == prev['nextsample']
            prev = f
        assert m['nextsample'] == m['fields'][-1]['nextsample']
    last = metas[-1]
    dec.use_resident_capture(0, nsamples)
    assert dec.decode(sink=None) == n
    assert dec.last_meta == last
