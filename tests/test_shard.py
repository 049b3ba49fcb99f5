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

from ldgpu.shard import audio_next, check_chain, frame_offsets, replay_offsets, shard_bounds, start_offsets

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


def test_shard_bounds_cover_the_capture():
    spf = 1334668
    b = shard_bounds(0, 2_400_000_000, spf, 8)
    assert b[0] == 0 and b[-1] == 2_400_000_000
    assert all((x % spf) == 0 for x in b[:-1]) and all(x < y for x, y in zip(b, b[1:]))


def test_audio_next_is_downscale_audio_recurrence():
    o = 0.0
    for _ in range(3):
        o2 = audio_next(o, 262, LINE_PERIOD)
        frametime = LINE_PERIOD * 262 / 1e6
        ticks = np.arange(o, frametime + 1 / 48000.0, 1 / 48000.0)
        assert o2 == ticks[-1] - frametime and 0 <= o2 < 1 / 48000.0 + 1e-12
        o = o2


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


@pytest.mark.gpu
@pytest.mark.parametrize('world', [2, 3])
def test_sharded_decode_equals_single_decode(world):
    from ldgpu.decoder import GPUDecoder
    from ldgpu.shard import ShardedDecode
    from ldgpu.synth import make_capture
    data = make_capture(int(40e6 * 0.6), 'u8', first_frame=1200, seed=21)
    ref = GPUDecoder(system='NTSC', batch=8)
    ref.set_capture(data, 0)
    want = []
    ref.decode(sink=lambda fr, au, m: want.append((fr.copy(), au.copy(), m)))
    decs = [GPUDecoder(system='NTSC', batch=8) for _ in range(world)]
    sds = []
    for r, d in enumerate(decs):
        d.set_capture(data, 0)
        sds.append(ShardedDecode(d, r, world))
    summ = [sd.local() for sd in sds]
    assert check_chain(summ) == []
    got = []
    for sd in sds:
        got += [(pic, a, m) for (g, a, m), pic in zip(sd.finish(summ), sd.frames)]
    assert len(got) == len(want) and all(s['n'] > 0 for s in summ)
    for (gf, ga, gm), (wf, wa, wm) in zip(got, want):
        assert gm == wm
        assert np.array_equal(gf, wf)
        assert np.array_equal(ga, wa)
