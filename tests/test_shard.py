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
