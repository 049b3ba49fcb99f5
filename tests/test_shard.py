"""Field-group sharding of one capture (ldgpu/shard.py).

CPU: the exchange step over a real torch.distributed gloo group of 2 ranks
(all_gather_object of the per-rank summaries -> chain check, audio-offset
replay, frame index prefix sums).  GPU: ranks run one after another on one
device must reproduce a single decode of the whole capture exactly.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from ldgpu.formats import FMT_LDS, FMT_R30, FMT_U8, bytes_for_samples
from ldgpu.shard import (audio_next, check_chain, decode_bounds, exchange_halo, frame_offsets, halo_plan, replay_offsets,
                         sample_byte, shard_bounds, shard_windows, start_offsets)

LINE_PERIOD = 63.5555555556


def _summaries():
    # three shards of a regular NTSC stream: last field of every frame is the 262-line bottom
    return [{'rank': 0, 'n': 4, 'first_start': 385743, 'first_mtf': 1, 'last_next': 5725434, 'end_mtf': 0.9995,
             'transitions': [262] * 4, 't0': 0},
            {'rank': 1, 'n': 5, 'first_start': 5725434, 'first_mtf': 0.9995, 'last_next': 12399101, 'end_mtf': 0.999,
             'transitions': [262] * 5, 't0': 3},
            {'rank': 2, 'n': 0, 'first_start': None, 'first_mtf': None, 'last_next': None, 'end_mtf': 0.999,
             'transitions': [], 't0': 0}]


def test_offsets_equal_sequential_replay():
    s = _summaries()
    seq = replay_offsets(0.0, [lc for x in s for lc in x['transitions']], LINE_PERIOD)
    assert start_offsets(s, LINE_PERIOD) == [seq[0], seq[4], seq[9]]
    assert frame_offsets(s) == [0, 4, 9]
    assert check_chain(s) == []
    bad = [dict(x) for x in s]
    bad[1]['first_start'] += 1
    assert check_chain(bad) == [1]
    bad = [dict(x) for x in s]
    bad[1]['first_mtf'] = 1.0
    assert check_chain(bad) == [1]


class _FakeDec:
    """The state ShardedDecode.summary reads from a GPUDecoder after a shard's decode."""

    def __init__(self, frames, mtf_level):
        self.shard_frames, self.mtf_level = frames, mtf_level
        self.transitions, self.last_framenr, self.last_isclv = [262] * len(frames), 12000, False
        self.last_read = None


def test_chain_check_uses_the_mtf_before_a_reread():
    """A CAV picture number >= 10000 clamps the MTF to 0 (lddecode_core.py:1300-1309).
    The warm-up frames of shard 1 carry no picture number, so its first kept frame
    begins with MTF 1 and re-reads itself at MTF 0, while the single decode (and
    shard 0, whose end MTF is 0) reads it at MTF 0 once.  The frame's fields then
    carry MTF 0 either way: the check must compare the MTF the frame's readframe
    began with, and flag the shard."""
    from ldgpu.shard import ShardedDecode
    sd = ShardedDecode.__new__(ShardedDecode)
    sd.rank = 1
    sd.dec = _FakeDec([{'start': 5725434, 'tstart': 0, 'nextsample': 7060101, 'mtf': 0.0, 'mtf0': 1.0,
                        'audio': [], 'vbi': {}, 'fields': []}], 0.0)
    s1 = sd.summary()
    s0 = {'rank': 0, 'n': 4, 'first_start': 385743, 'first_mtf': 0.0, 'last_next': 5725434, 'end_mtf': 0.0,
          'transitions': [262] * 4, 't0': 0}
    assert s1['first_mtf'] == 1.0 and check_chain([s0, s1]) == [1]
    sd.dec.shard_frames[0]['mtf0'] = 0.0          # began at the handed-over MTF: no re-read, chain exact
    assert check_chain([s0, sd.summary()]) == []


def test_frame_spill_round_trip(tmp_path):
    """A shard's frames wait on storage (bounded host memory) and read back unchanged."""
    from ldgpu.shard import FrameSpill, comb_burst_levels
    rng = np.random.default_rng(3)
    frames = rng.integers(0, 65535, (5, 525, 910)).astype(np.uint16)
    sp = FrameSpill(str(tmp_path))
    sp.reset()
    for f in frames:
        sp.append(f)
    assert len(sp) == 5 and np.array_equal(sp[3], frames[3]) and np.array_equal(np.stack(list(sp)), frames)
    assert np.array_equal(comb_burst_levels(sp, chunk=2), comb_burst_levels(list(frames)))
    sp.reset()                                    # a re-decode starts a fresh file
    assert len(sp) == 0
    sp.close()


def test_shard_bounds_cover_the_capture():
    spf = 1334668
    b = shard_bounds(0, 2_400_000_000, spf, 8)
    assert b[0] == 0 and b[-1] == 2_400_000_000
    assert all((x % spf) == 0 for x in b[:-1]) and all(x < y for x, y in zip(b, b[1:]))


def test_decode_bounds_stop_at_the_frame_limit():
    """The shards split only the samples the frame limit reaches: a 60 s u8 capture's
    10-bit EOF guard keeps 1438 of its ~1798 frames, so the last shard ends two frames
    past frame 1438, not at the end of the capture; -l shortens it further."""
    spf = 1334667
    n = 2_400_000_000
    b, limit, start = decode_bounds(n, n, spf, 4)
    assert limit == n // (spf * 5 // 4) == 1438 and start == 0
    assert b[-1] == (limit + 2) * spf < n and b[0] == 0 and all(x < y for x, y in zip(b, b[1:]))
    b2, limit2, start2 = decode_bounds(n, n, spf, 2, start_frame=10, length=100)
    assert limit2 == 100 and start2 == 10 * spf and b2[-1] == start2 + 102 * spf
    # a short capture: the end stays the capture's
    b3, _, _ = decode_bounds(5 * spf, 5 * spf, spf, 2, length=100)
    assert b3[-1] == 5 * spf


def test_audio_next_is_downscale_audio_recurrence():
    o = 0.0
    for _ in range(3):
        o2 = audio_next(o, 262, LINE_PERIOD)
        frametime = LINE_PERIOD * 262 / 1e6
        ticks = np.arange(o, frametime + 1 / 48000.0, 1 / 48000.0)
        assert o2 == ticks[-1] - frametime and 0 <= o2 < 1 / 48000.0 + 1e-12
        o = o2


@pytest.mark.parametrize('line_period', [LINE_PERIOD, 64.0])
def test_audio_next_closed_form_equals_np_arange(line_period):
    """audio_next's closed form == np.arange(...)[-1] - frametime bit for bit, over the
    chain's own offsets and over arbitrary ones (short and empty ranges included)."""
    rng = np.random.default_rng(7)
    o = 0.0
    for i in range(20000):
        lc = int(rng.choice([262, 263, 312, 313])) if i % 3 else int(rng.integers(1, 700))
        off = o if i % 2 else float(rng.uniform(-2e-3, 2e-3))
        frametime = line_period * lc / 1e6
        ticks = np.arange(off, frametime + 1 / 48000.0, 1 / 48000.0)
        if ticks.size == 0:
            with pytest.raises(IndexError):
                audio_next(off, lc, line_period)
            continue
        got = audio_next(off, lc, line_period)
        assert got == ticks[-1] - frametime
        assert replay_offsets(off, [lc], line_period)[1] == got      # the library's chain (C)
        o = got


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    mine = _summaries()[rank]
    got = [None] * world
    dist.all_gather_object(got, mine)
    res = (check_chain(got + _summaries()[world:]), start_offsets(got, LINE_PERIOD), frame_offsets(got))
    q.put((rank, res))
    dist.destroy_process_group()


def test_exchange_over_gloo_world2():
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert out[0] == out[1]
    bad, offs, fo = out[0]
    s = _summaries()[:2]
    assert bad == [] and fo == [0, 4] and offs == start_offsets(s, LINE_PERIOD)


SPF = 1334668


def test_shard_windows_cover_every_shards_reads():
    n = 60_000_000
    b = shard_bounds(0, n, SPF, 4)
    w = shard_windows(b, SPF, n)
    assert halo_plan(w) == [True] * 3
    for k, (lo, cut, hi) in enumerate(w):
        assert lo % 12 == 0 and lo <= max(0, b[k] - 2 * SPF - 1024)
        if k < 3:
            assert cut <= b[k + 1] < cut + 12 and hi >= b[k + 1] + 2 * SPF + 1000001
            assert w[k + 1][0] <= cut            # the next rank holds the halo in its own part
        else:
            assert cut == hi == n


def test_last_window_ends_with_the_decode_not_the_capture():
    """An epoch of a long capture (the frame limit ends far before the capture) keeps the
    last rank's window O(epoch) too; a read past it widens around the read."""
    from ldgpu.shard import READ_SPAN, widen_window
    n = 3600 * 40_000_000                                  # an hour of u8 RF
    b, limit, _ = decode_bounds(n, n, SPF, 4, start_frame=5000, length=9)
    w = shard_windows(b, SPF, n)
    assert limit == 9
    for lo, cut, hi in w:
        assert hi - lo <= (9 // 4 + 2 + 2 + 2 + 1) * SPF + READ_SPAN + 1024 + 24
    assert w[-1][1] == w[-1][2] < n
    lo, hi = widen_window(w[-1][2] + 5 * SPF, SPF, n)
    assert lo <= w[-1][2] + 4 * SPF - 1024 and hi >= w[-1][2] + 13 * SPF + READ_SPAN and hi - lo < 11 * SPF
    assert widen_window(n - 100, SPF, n)[1] == n


def _halo_worker(rank, world, port, fmt, q):
    import torch
    from ldgpu.shard import torch_p2p
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    n = 14_000_000
    data = (np.arange(bytes_for_samples(fmt, n), dtype=np.uint64) * 2654435761 >> 13).astype(np.uint8)
    w = shard_windows(shard_bounds(0, n, SPF, world), SPF, n)
    lo, cut, hi = w[rank]
    end = lambda s: data.size if s >= n else sample_byte(fmt, s)   # noqa: E731
    bl, bc, bh = sample_byte(fmt, lo), end(cut), end(hi)
    buf = torch.zeros(bh - bl, dtype=torch.uint8)
    buf[:bc - bl].numpy()[:] = data[bl:bc]              # this rank's own part, from "storage"
    got = exchange_halo(buf, rank, w, fmt, torch_p2p)
    q.put((rank, got, bool(np.array_equal(buf.numpy(), data[bl:bh]))))
    dist.destroy_process_group()


@pytest.mark.parametrize('world,fmt', [(2, FMT_U8), (3, FMT_R30), (2, FMT_LDS)])
def test_halo_exchange_over_gloo(world, fmt):
    """Each rank's capture window = its own storage part + the halo from the next rank."""
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    ps = [ctx.Process(target=_halo_worker, args=(r, world, port, fmt, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = dict((r, (g, ok)) for r, g, ok in (q.get(timeout=120) for _ in ps))
    for p in ps:
        p.join(timeout=60)
    for r in range(world):
        assert out[r][1], r
        assert out[r][0] == (r < world - 1)


@pytest.mark.gpu
@pytest.mark.parametrize('world,windowed', [(2, False), (3, False), (2, True), (3, True)])
def test_sharded_decode_equals_single_decode(world, windowed):
    from ldgpu.decoder import GPUDecoder
    from ldgpu.shard import ShardedDecode
    from ldgpu.synth import make_capture
    data = make_capture(int(40e6 * 0.6), 'u8', first_frame=1200, seed=21)
    ref = GPUDecoder(system='NTSC', batch=8)
    ref.set_capture(data, 0)
    want = []
    ref.decode(sink=lambda fr, au, m: want.append((fr.copy(), au.copy(), m)))
    decs = [GPUDecoder(system='NTSC', batch=8) for _ in range(world)]
    raw = np.frombuffer(data, np.uint8)
    n = raw.size
    spf = decs[0].rf.samples_per_frame          # the windows production computes (lddecode.load_window)
    w = shard_windows(decode_bounds(n, n, spf, world)[0], spf, n)
    sds = []
    for r, d in enumerate(decs):
        if windowed:
            # the window a rank holds after the halo exchange (the exchange itself: test_halo_exchange_over_gloo)
            lo, cut, hi = w[r]
            d.set_capture(raw[lo:hi], 0, first_sample=lo, total_bytes=n)
        else:
            d.set_capture(data, 0)
        sds.append(ShardedDecode(d, r, world, whole_capture=lambda d=d: d.set_capture(data, 0)))
    summ = [sd.local() for sd in sds]
    assert check_chain(summ) == []
    got = []
    for sd in sds:
        got += [(pic, a, m) for (g, a, m), pic in zip(sd.finish(summ), sd.frames)]
    assert len(got) == len(want) and all(s['n'] > 0 for s in summ)
    for i, ((gf, ga, gm), (wf, wa, wm)) in enumerate(zip(got, want)):
        assert gm == wm, i
        d = np.flatnonzero(np.asarray(gf) != wf)
        if d.size:
            # which side is off: a second single decode of the same capture
            again = []
            ref2 = GPUDecoder(system='NTSC', batch=8)
            ref2.set_capture(data, 0)
            ref2.decode(sink=lambda fr, au, m: again.append(fr.copy()))
            side = ('the first single decode is off' if np.array_equal(again[i], gf) else
                    'the sharded decode is off' if np.array_equal(again[i], wf) else 'all three differ')
            assert False, ('frame %d of %d (ranks %s): %d samples differ at %s, max |diff| %d; by a second '
                           'single decode, %s' % (
                               i, len(got), [s['n'] for s in summ], d.size,
                               sorted({(int(x) // 910, int(x) % 910) for x in d})[:6],
                               np.abs(np.asarray(gf, dtype=np.int64) - wf)[d].max(), side))
        assert np.array_equal(ga, wa), i
    if windowed:
        assert all(sd.window_misses == 0 for sd in sds)


@pytest.mark.gpu
def test_sharded_window_miss_falls_back_to_whole_capture():
    """A window too small for the reads (no halo) is detected (WindowMiss) and the rank
    re-decodes from the whole capture: the result still equals the single decode."""
    from ldgpu.decoder import GPUDecoder
    from ldgpu.shard import ShardedDecode
    from ldgpu.synth import make_capture
    data = make_capture(int(40e6 * 0.6), 'u8', first_frame=1200, seed=21)
    raw = np.frombuffer(data, np.uint8)
    n = raw.size
    ref = GPUDecoder(system='NTSC', batch=8)
    ref.set_capture(data, 0)
    want = []
    ref.decode(sink=lambda fr, au, m: want.append((fr.copy(), au.copy(), m)))
    decs = [GPUDecoder(system='NTSC', batch=8) for _ in range(2)]
    spf = decs[0].rf.samples_per_frame
    w = shard_windows(decode_bounds(n, n, spf, 2)[0], spf, n, halo_frames=0)
    sds = []
    for r, d in enumerate(decs):
        lo, cut, _ = w[r]
        d.set_capture(raw[lo:cut], 0, first_sample=lo, total_bytes=n)      # no halo at all
        sds.append(ShardedDecode(d, r, 2, whole_capture=lambda d=d: d.set_capture(data, 0)))
    summ = [sd.local() for sd in sds]
    got = []
    for sd in sds:
        got += [(pic, a, m) for (g, a, m), pic in zip(sd.finish(summ), sd.frames)]
    assert sds[0].window_misses == 1
    assert len(got) == len(want)
    for (gf, ga, gm), (wf, wa, wm) in zip(got, want):
        assert gm == wm and np.array_equal(gf, wf) and np.array_equal(ga, wa)


def run_ranks(sds):
    """decode_sharded's phases for every rank of one process, one rank after another
    (local decode -> chain check / refix -> the last rank's extension -> finish).
    Returns [(global index, frame, pcm, meta)] in order and the summaries."""
    summ = [sd.local() for sd in sds]
    for _ in range(len(sds)):
        bad = check_chain(summ)
        if not bad:
            break
        summ = [sd.refix(summ) if r in bad else summ[r] for r, sd in enumerate(sds)]
    assert check_chain(summ) == []
    summ = [sd.extend(summ) or s for sd, s in zip(sds, summ)]
    out = []
    for sd in sds:
        res = sd.finish(summ)
        out += [(g, pic, a, m) for (g, a, m), pic in zip(res, sd.frames)]
    return out, summ


def windowed_decoders(data, fmt, system, world, batch=8, length=None):
    """One GPUDecoder per rank holding the capture window shard_windows gives it (what
    load_window leaves in HBM after the halo exchange), each with the whole-capture fallback."""
    from ldgpu.decoder import GPUDecoder
    from ldgpu.formats import samples_in_bytes
    from ldgpu.shard import ShardedDecode
    raw = np.frombuffer(bytes(data), np.uint8)
    decs = [GPUDecoder(system=system, batch=batch) for _ in range(world)]
    n = samples_in_bytes(fmt, raw.size)
    spf = decs[0].rf.samples_per_frame
    w = shard_windows(decode_bounds(n, raw.size, spf, world, length=length)[0], spf, n)
    from ldgpu.shard import widen_window

    def load(d, lo, hi):
        b0 = sample_byte(fmt, lo)
        b1 = raw.size if hi >= n else sample_byte(fmt, hi)
        d.set_capture(raw[b0:b1], fmt, first_sample=lo, total_bytes=raw.size)

    sds = []
    for r, d in enumerate(decs):
        lo, cut, hi = w[r]
        load(d, lo, hi)
        # the last rank's extension past its window widens it (lddecode.py widen_window)
        sds.append(ShardedDecode(d, r, world, length=length,
                                 whole_capture=lambda d=d: d.set_capture(raw, fmt),
                                 widen=lambda s, d=d: load(d, *widen_window(s, spf, n))))
    return sds


def assert_matches_oracle(got, frames, pcm, meta, pcm_sha=None):
    """.tbc within +-1 LSB, .pcm bit-exact, metadata exact, frame for frame."""
    import hashlib
    assert [g for g, _, _, _ in got] == list(range(len(got)))
    assert len(got) == len(frames), (len(got), len(frames))
    for i, ((g, pic, a, m), f, p, om) in enumerate(zip(got, frames, pcm, meta)):
        assert m == om, i
        d = np.abs(np.asarray(pic, dtype=np.int64).reshape(-1) - f.astype(np.int64))
        assert d.max() <= 1, (i, int(d.max()))
        assert np.array_equal(a, p), i
        if pcm_sha is not None:
            assert hashlib.sha256(a.tobytes()).hexdigest() == pcm_sha[i]


_ORACLE_1S = {}


def _clv_1s():
    """~1 s of NTSC CLV u8 RF and the oracle's decode of it (once per session)."""
    if not _ORACLE_1S:
        from ldgpu.synth import make_capture
        from oracle.capture import FMT_U8
        from oracle.framer import decode_capture
        data = make_capture(int(40e6 * 1.0), 'u8', first_frame=3020, clv=True, seed=44)
        _ORACLE_1S['v'] = (data,) + decode_capture(data, FMT_U8)
    return _ORACLE_1S['v']


@pytest.mark.gpu
@pytest.mark.parametrize('world', [2, 3, 4])
@pytest.mark.parametrize('case', ['ntsc_clv_u8_0p2s', 'clv_1s',
                                  # the MTF chain across rank boundaries: every rank after the
                                  # first starts from a fresh framer (MTF 1), so its warm-up frame
                                  # re-reads at MTF 0.88 / 0.0002, and the clamp to 0 falls on a
                                  # later rank (lddecode_core.py:1300-1309)
                                  'ntsc_cav_u8_mtf_0p3s', 'ntsc_cav_u8_mtf0_0p3s',
                                  # PAL: the same field-group windows and chains
                                  'pal_clv_u8_0p2s', 'pal_cav_u8_mtf_0p3s'])
def test_sharded_decode_vs_oracle(case, world):
    """Config 5's decode (field-group sharded, capture windows, ranks one after another on
    one device) against the ORACLE's single decode of the same capture -- not against
    another GPU decode: .tbc +-1 LSB, .pcm bit-exact, per-frame metadata exact.  The golden
    case's oracle output is itself pinned to the committed fixture's SHA-256s.  The chains
    carried across the rank boundaries: read position, MTF, audio offset
    (lddecode_core.py:1204,1289,1300-1309)."""
    if case == 'clv_1s':
        data, frames, pcm, meta = _clv_1s()
        sys_, fmt, sha = 'NTSC', FMT_U8, None
    else:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from test_gpu_parity import oracle_decode
        from ldgpu.formats import NAME_TO_FMT
        data, gold, frames, pcm, meta = oracle_decode(case)
        sys_, fmt = gold['settings']['system'], NAME_TO_FMT[gold['settings']['fmt']]
        sha = [g['pcm_sha256'] for g in gold['frames']]
    sds = windowed_decoders(data, fmt, sys_, world)
    got, summ = run_ranks(sds)
    assert sum(1 for s in summ if s['n']) >= 2, [s['n'] for s in summ]     # really split
    assert all(sd.window_misses == 0 for sd in sds)
    assert_matches_oracle(got, frames, pcm, meta, sha)


@pytest.mark.gpu
@pytest.mark.parametrize('world', [2, 3])
def test_sharded_skipped_fields_extend_the_last_rank(world):
    """Fields the reference skips ("no/corrupt VSYNC found, jumping forward", 'not valid')
    push the limit's last frame past the nominal split (the frame limit -l 5 here ends at
    sample ~13.1 M, the split at 7 frames = 9.34 M): the last rank reads on past its
    boundary, so the sharded decode still emits the reference's 5 frames."""
    from ldgpu.synth import make_capture
    from oracle.capture import FMT_U8
    from oracle.framer import decode_capture
    starts = [1052829 + int(k * 667333.5) for k in range(12)]
    data = make_capture(int(40e6 * 0.5), 'u8', first_frame=300, seed=41,
                        dropouts=tuple((s + 30000, 15000) for s in starts[2:10:2]))
    frames, pcm, meta = decode_capture(data, FMT_U8, length=5)
    spf = 1334668
    assert len(frames) == 5 and meta[-1]['nextsample'] > 7 * spf      # past the nominal split
    sds = windowed_decoders(data, FMT_U8, 'NTSC', world, length=5)
    got, summ = run_ranks(sds)
    assert sds[-1].extended > 0
    assert sds[-1].widened > 0          # the extension read past the last rank's capped window
    assert_matches_oracle(got, frames, pcm, meta)


@pytest.mark.gpu
def test_sharded_300s_clv_8way_property():
    """Config 5 at size (a 300 s CLV capture, 12 GB u8, field-sharded 8 ways on one device,
    capture windows): consecutive CLV frame numbers across every rank boundary, the frame
    count the reference's 10-bit EOF guard gives (lddecode.py:42,49,89), no chain re-fix
    and no window miss."""
    import torch
    from ldgpu.decoder import GPUDecoder
    from ldgpu.shard import ShardedDecode
    n, world = int(40e6 * 300), 8
    src = GPUDecoder(system='NTSC', batch=8)
    src.ctx.synth(n, fmt=0, first_frame=1, clv=True, seed=23)
    spf = src.rf.samples_per_frame
    w = shard_windows(decode_bounds(n, n, spf, world)[0], spf, n)
    sds, bufs = [], []
    for r in range(world):
        lo, cut, hi = w[r]
        buf = torch.empty(hi - lo, dtype=torch.uint8, device='cuda')
        src.ctx.capture_copy_to_device(buf.data_ptr(), lo, hi - lo)
        torch.cuda.synchronize()
        d = GPUDecoder(system='NTSC', batch=32)
        d.set_capture(None, 0, device_ptr=buf.data_ptr(), nsamples=hi - lo, first_sample=lo, total_bytes=n)
        bufs.append(buf)
        sds.append(ShardedDecode(d, r, world, resident=True))
    src.ctx.close()
    summ = [sd.local() for sd in sds]
    assert check_chain(summ) == []                     # no re-fix needed
    summ = [sd.extend(summ) or s for sd, s in zip(sds, summ)]
    nrs = []
    for sd in sds:
        res = sd.finish(summ)
        nrs += [m['vbi']['framenr'] for _, _, m in res]
        assert sd.window_misses == 0
    bpf = spf * 5 // 4
    assert len(nrs) == n // bpf, (len(nrs), n // bpf)
    assert all(b == a + 1 for a, b in zip(nrs, nrs[1:]))
    assert all(s['n'] > 0 for s in summ)


def test_comb_start_state_matches_one_chain():
    """The comb state a shard starts from is the single chain's state at that frame."""
    from ldgpu.shard import comb_burst_levels, comb_chain, comb_start_state
    rng = np.random.default_rng(6)
    frames = rng.integers(0, 65535, (5, 525, 910)).astype(np.uint16)
    frames[:, :, 1] = rng.integers(0, 20 * 358, (5, 525))          # burst levels 0..20 IRE
    frames[0, :100, 1] = 0                                         # the chain starts late
    lv = [comb_burst_levels(frames[:2]), comb_burst_levels(frames[2:3]), comb_burst_levels(frames[3:])]
    whole = comb_chain(-1.0, comb_burst_levels(frames[:3]))
    assert comb_start_state(lv, 2) == whole
    assert comb_start_state(lv, 0) == -1.0


def test_comb_summaries_give_the_exact_start_state():
    """The comb exchange of chain summaries (first COMB_PREFIX levels + the speculative
    states) gives every rank the same start state as the full chain over all earlier
    frames; a rank whose prefix has too few bursts to converge is reported (None)."""
    from ldgpu.shard import (COMB_PREFIX, comb_chain, comb_redo_frames, comb_start_from_summaries,
                             comb_start_state, comb_summary)
    rng = np.random.default_rng(12)
    lv = [rng.uniform(2.0, 25.0, n) for n in (3 * 487, 20 * 487, 15 * 487, 4 * 487)]
    summ = [comb_summary(x) for x in lv]
    for r in range(len(lv)):
        assert comb_start_from_summaries(summ, r) == comb_start_state(lv, r)
    quiet = np.concatenate([np.zeros(COMB_PREFIX + 10), rng.uniform(5, 20, 5000)])   # no burst at first
    s2 = [summ[0], comb_summary(quiet), summ[2]]
    assert comb_start_from_summaries(s2, 2) is None
    # frames to re-comb: until the speculative chain (from "not initialised") meets the exact one
    a0 = comb_start_state(lv, 2)
    k = comb_redo_frames(a0, lv[2], 487)
    assert 0 < k < 15
    ex, sp = a0, -1.0
    for f in range(15):
        part = lv[2][f * 487:(f + 1) * 487]
        if f >= k:
            assert ex == sp
        ex, sp = comb_chain(ex, part), comb_chain(sp, part)
    assert comb_redo_frames(-1.0, lv[2], 487) == 0


class _FakeComb3D:
    """comb_ntsc3d's contract on a host (no GPU): history of the last two inputs, one output
    per frame with both neighbours, the burst-level EMA chained over the outputs' frames.
    An output is (the frame's label, the EMA entering it, its two neighbours' labels)."""
    comb_lines, max_frames = 480, 3

    def __init__(self):
        self.hist, self.state = [], -1.0

    def comb_reset(self):
        self.hist, self.state = [], -1.0

    def comb_set_state(self, a):
        self.state = float(a)

    def comb_ntsc3d(self, frames, core, rng):
        from ldgpu.shard import comb_burst_levels, comb_chain
        out = []
        for f in frames:
            self.hist = (self.hist + [np.asarray(f)])[-3:]
            if len(self.hist) == 3:
                p, c, n = self.hist
                out.append(np.array([c[0], self.state, p[0], n[0]], dtype=np.float64))
                self.state = comb_chain(self.state, comb_burst_levels([c]))
        return out


def test_comb3d_sharded_equals_one_process_over_any_split():
    """ldgpu/shard.py comb3d_sharded: the ranks' 3D-comb outputs, put together by their
    output index, are the single process's -- every frame but the first and last, each
    with its true neighbours and the exact burst-level EMA (ranks with no frames too)."""
    import threading
    from ldgpu.shard import comb3d_sharded
    rng = np.random.default_rng(5)
    N = 11
    frames = []
    for g in range(N):
        f = np.zeros(525 * 910, dtype=np.uint16)
        f[0] = 1000 + g                                          # the frame's label
        lv = rng.integers(0, 4000, 525)
        lv[rng.random(525) < 0.3] = 0                            # lines without burst
        f[np.arange(525) * 910 + 1] = lv
        frames.append(f)

    class Dec:
        def __init__(self):
            self.ctx = _FakeComb3D()
    one = Dec()
    want = [(i, o) for i, o in enumerate(one.ctx.comb_ntsc3d(frames, -1, -1))]
    for split in ([0, 4, 7, 11], [0, 1, 2, 11], [0, 5, 5, 11], [0, 11, 11, 11], [0, 3, 10, 11]):
        world = len(split) - 1
        bar = threading.Barrier(world)
        slots = [None] * world
        got = [None] * world

        def run(r):
            def ag(obj):
                slots[r] = obj
                bar.wait()
                res = list(slots)
                bar.wait()
                return res
            got[r] = comb3d_sharded(Dec(), r, ag, frames[split[r]:split[r + 1]], split[r])
        th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        allout = sorted((k, tuple(o)) for part in got for k, o in part)
        assert allout == [(k, tuple(o)) for k, o in want], split
