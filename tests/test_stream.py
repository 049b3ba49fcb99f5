"""Streamed capture (ldg_stream_*, GPUDecoder.open_stream): the capture reaches the GPU
from its file through a fixed ring in HBM, as the reference's loader reads it block by
block (lddecode_core.py:373-392, lddutils.py:131-229) -- device memory independent of the
capture's length.  Bar: the decode through a ring much smaller than the capture is
byte-identical to the decode of the whole capture resident in HBM (frames, audio,
metadata), on every golden case and on 60 s of RF."""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CLI = os.path.join(ROOT, 'ld-decode_amd', 'lddecode.py')
EXT = {'u8': 'u8', 's16': 'r16', 'r30': 'r30', 'lds': 'lds'}


def _decode(dec, **kw):
    got = []
    dec.decode(sink=lambda fr, au, meta: got.append((fr.copy(), au.copy(), meta)), **kw)
    return got


# ---- host logic (no GPU): the planner's fit of a launch to the ring -----------------------

class _FakeStreamCtx:
    def __init__(self, lo, reach):
        self.win = [lo, reach]
        self.seeks = []

    def stream_window(self):
        return self.win[0], self.win[1], 0, 10 ** 9

    def stream_seek(self, s):
        self.seeks.append(s)
        self.win = [s - s % 12, s - s % 12 + (self.win[1] - self.win[0])]


def _fit(lo, reach, keys, pending=()):
    from ldgpu.decoder import GPUDecoder
    d = GPUDecoder.__new__(GPUDecoder)
    d.ctx = _FakeStreamCtx(lo, reach)
    d.pending = list(pending)
    d.cap_nsamples = 10 ** 9
    d.stats = {}
    return d, d._stream_fit(keys)


def test_stream_fit_keeps_the_reads_inside_the_ring():
    from ldgpu.decoder import BLOCKCUT, read_geometry
    keys = [(1000000 + 667000 * i, 1.0) for i in range(10)]
    last_end = lambda k: read_geometry(k[0])[2] + 16384           # noqa: E731
    reach = last_end(keys[4])
    d, fit = _fit(0, reach, keys)
    assert fit == keys[:5] and not d.ctx.seeks
    # a read whose first block lies below the released point is not launched
    d, fit = _fit(keys[0][0] - BLOCKCUT + 1, reach, keys, pending=[1])
    assert fit == [] and not d.ctx.seeks


def test_stream_fit_restarts_the_stream_at_a_jump():
    from ldgpu.decoder import STREAM_MARGIN, read_geometry
    far = [(400000000, 1.0), (400667000, 1.0)]
    d, fit = _fit(0, 50000000, far)          # nothing in flight: the stream moves to the read
    assert d.ctx.seeks == [read_geometry(far[0][0])[0] - STREAM_MARGIN]
    assert fit == far and d.stats['stream_seeks'] == 1
    d, fit = _fit(0, 50000000, far, pending=[1])   # in flight: wait for the replay instead
    assert fit == [] and not d.ctx.seeks


def test_stream_abi_declared():
    src = open(os.path.join(ROOT, 'include', 'ldgpu.h')).read()
    for f in ('ldg_stream_open', 'ldg_stream_release', 'ldg_stream_seek', 'ldg_stream_window',
              'ldg_stream_stats', 'ldg_stream_close'):
        assert f + '(' in src


# ---- GPU --------------------------------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize('case,ring_mb', [('ntsc_cav_u8_0p2s', 2), ('ntsc_cav_s16_0p15s', 3),
                                          ('ntsc_cav_s16_0p15s', 6),
                                          ('ntsc_cav_r30_0p15s', 2), ('ntsc_cav_lds_0p15s', 2),
                                          ('pal_clv_u8_0p2s', 2), ('ntsc_cav_u8_mtf_0p3s', 4),
                                          ('ntsc_cav_u8_mid_0p2s', 2)])
def test_stream_decode_equals_resident(case, ring_mb, tmp_path):
    """Every golden case through a ring of a few MiB (the capture slides through it many
    times over; u8 2 MiB = 3 fields) gives exactly the resident decode, which the golden
    fixture pins (metadata exact, .pcm SHA-256)."""
    sys.path.insert(0, os.path.join(HERE, 'golden'))
    import make_golden
    from ldgpu.decoder import GPUDecoder
    from ldgpu.formats import NAME_TO_FMT
    with open(os.path.join(HERE, 'golden', case + '.json')) as fh:
        gold = json.load(fh)
    c = gold['settings']
    data = make_golden.build_capture(case)
    fmt = NAME_TO_FMT[c['fmt']]
    path = tmp_path / ('cap.' + EXT[c['fmt']])
    path.write_bytes(bytes(data))
    dec = GPUDecoder(system=c['system'], batch=16)
    dec.set_capture(data, fmt)
    want = _decode(dec)
    dec.open_stream(str(path), fmt, ring_mb << 20)
    got = _decode(dec)
    st = dec.ctx.stream_stats()
    assert len(got) == len(want) == len(gold['frames'])
    for (f1, a1, m1), (f2, a2, m2), g in zip(got, want, gold['frames']):
        assert m1 == m2 == g['meta']
        assert np.array_equal(f1, f2)
        assert np.array_equal(a1, a2)
        assert hashlib.sha256(a1.tobytes()).hexdigest() == g['pcm_sha256']
    assert st['bytes_read'] >= len(data) * 0.9 and st['ring_bytes'] <= ring_mb << 20
    print('%s: ring %d MiB, %d chunks, %d launch waits, %d seeks' % (case, ring_mb, st['chunks'],
                                                                     st['launch_waits'], st['seeks']))
    dec.ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize('copies', ['1', '3'])
def test_stream_copy_streams_and_ring_reuse(copies, tmp_path, monkeypatch):
    """The chunks' copies rotate over LDG_STREAM_COPIES streams (default 4): with 1 and 3
    (a count that does not divide the ring's chunks) the decode through a 2 MiB ring is the
    resident one; a second file opened at the same ring size reuses the ring (no new
    device memory) and decodes to its own golden output."""
    sys.path.insert(0, os.path.join(HERE, 'golden'))
    import make_golden
    from ldgpu.decoder import GPUDecoder
    from ldgpu.native import device_memory
    monkeypatch.setenv('LDG_STREAM_COPIES', copies)
    dec = GPUDecoder(system='NTSC', batch=16)
    for i, case in enumerate(('ntsc_cav_u8_0p2s', 'ntsc_cav_u8_mid_0p2s')):
        with open(os.path.join(HERE, 'golden', case + '.json')) as fh:
            gold = json.load(fh)
        data = make_golden.build_capture(case)
        path = tmp_path / ('cap%d.u8' % i)
        path.write_bytes(bytes(data))
        free0 = device_memory(0)[0]
        dec.open_stream(str(path), 0, 2 << 20)
        if i:
            assert abs(device_memory(0)[0] - free0) < 1 << 20     # the same ring, reused
        got = _decode(dec)
        assert len(got) == len(gold['frames'])
        for (f1, a1, m1), g in zip(got, gold['frames']):
            assert m1 == g['meta']
            assert hashlib.sha256(a1.tobytes()).hexdigest() == g['pcm_sha256']
        if i == 0:
            dec.set_capture(data, 0)
            want = _decode(dec)
            assert all(np.array_equal(a[0], b[0]) for a, b in zip(got, want))
            dec.open_stream(str(path), 0, 2 << 20)      # (set_capture closed the stream)
    dec.ctx.close()


@pytest.mark.gpu
def test_stream_edge_files(tmp_path):
    """A missing file fails loudly at the open; a file shorter than two frames is refused
    by the decode exactly as the resident capture is ('start frame is past end of file',
    lddecode.py:49 with the 10-bit frame size); the stream then still decodes a good file."""
    sys.path.insert(0, os.path.join(HERE, 'golden'))
    import make_golden
    from ldgpu.decoder import GPUDecoder
    from ldgpu.native import LDGError
    dec = GPUDecoder(system='NTSC', batch=16)
    with pytest.raises(LDGError, match='cannot open'):
        dec.open_stream(str(tmp_path / 'missing.u8'), 0, 2 << 20)
    short = bytes(make_golden.build_capture('ntsc_cav_u8_0p2s'))[:1000000]
    path = tmp_path / 'short.u8'
    path.write_bytes(short)
    errs = []
    for opener in (lambda: dec.set_capture(short, 0), lambda: dec.open_stream(str(path), 0, 2 << 20)):
        opener()
        with pytest.raises(ValueError) as e:
            dec.decode(sink=lambda *a: None)
        errs.append(str(e.value))
    assert errs[0] == errs[1] == 'start frame is past end of file'
    with open(os.path.join(HERE, 'golden', 'ntsc_cav_u8_0p2s.json')) as fh:
        gold = json.load(fh)
    good = tmp_path / 'good.u8'
    good.write_bytes(bytes(make_golden.build_capture('ntsc_cav_u8_0p2s')))
    dec.open_stream(str(good), 0, 2 << 20)
    got = _decode(dec)
    assert [m for _, _, m in got] == [g['meta'] for g in gold['frames']]
    dec.ctx.close()


@pytest.mark.gpu
def test_stream_open_and_seek_refused_with_decodes_outstanding(tmp_path):
    """ldg_stream_open / ldg_stream_seek need no decode outstanding (they rewrite the ring a
    launched demod may still read): LDG_ESTATE while a call is in flight, fine after its
    wait."""
    sys.path.insert(0, os.path.join(HERE, 'golden'))
    import make_golden
    from ldgpu.decoder import GPUDecoder
    from ldgpu.native import LDGError
    data = bytes(make_golden.build_capture('ntsc_cav_u8_0p2s'))
    path = tmp_path / 'cap.u8'
    path.write_bytes(data)
    dec = GPUDecoder(system='NTSC', batch=16)
    dec.open_stream(str(path), 0, 2 << 20)
    dec.ctx.decode_reads_async([0], [1.0], [0])
    with pytest.raises(LDGError, match='outstanding'):
        dec.ctx.stream_open(str(path), 0, 2 << 20)
    with pytest.raises(LDGError, match='outstanding'):
        dec.ctx.stream_seek(0)
    dec.ctx.decode_reads_wait()
    dec.open_stream(str(path), 0, 2 << 20)
    with open(os.path.join(HERE, 'golden', 'ntsc_cav_u8_0p2s.json')) as fh:
        gold = json.load(fh)
    assert [m for _, _, m in _decode(dec)] == [g['meta'] for g in gold['frames']]
    dec.ctx.close()


def _run_cli(*args):
    return subprocess.run([sys.executable, CLI, *map(str, args)], capture_output=True, text=True, timeout=600)


@pytest.mark.gpu
def test_cli_stream_equals_whole_capture(tmp_path):
    """lddecode.py through a 2 MiB ring (--window-mb 2) writes the same .tbc / .pcm / .json
    and prints the same lines as with the capture uploaded whole (--window-mb 0), on a
    capture with dropouts (invalid fields, jumps) and with -s / -l."""
    from ldgpu.synth import make_capture
    from test_cli import DROPOUT_CAPTURE
    cap = tmp_path / 'cap.u8'
    cap.write_bytes(bytes(make_capture(int(40e6 * 0.3), 'u8', **DROPOUT_CAPTURE)))
    for extra in ([], ['-s', '1', '-l', '3']):
        outs = []
        for w in (0, 2):
            out = tmp_path / ('o%d_%d' % (w, len(extra)))
            r = _run_cli(*extra, '--window-mb', w, cap, out)
            assert r.returncode == 0, r.stderr[-3000:]
            outs.append((r.stdout.splitlines()[1:], [open(str(out) + e, 'rb').read() for e in ('.tbc', '.pcm', '.json')]))
        assert outs[0] == outs[1]
        assert len(outs[0][1][0]) >= 2 * 955500


@pytest.mark.gpu
def test_stream_60s_equals_resident_and_memory_is_flat(tmp_path):
    """60 s of NTSC CAV RF (2.4 GB u8, 1,438 frames) through a 64 MiB ring: every frame,
    the audio and the metadata equal the decode of the whole capture resident in HBM, and
    the stream's device memory is the ring, not the capture."""
    from ldgpu.decoder import GPUDecoder
    from ldgpu.native import device_memory
    n = int(40e6 * 60)
    dec = GPUDecoder(system='NTSC', batch=128)
    dec.ctx.synth(n, fmt=0, first_frame=1, seed=20181016)
    path = tmp_path / 'cap60.u8'
    with open(path, 'wb') as fh:
        step = 1 << 28
        for off in range(0, n, step):
            fh.write(dec.ctx.capture_download(off, min(step, n - off)).tobytes())
    dec.use_resident_capture(0, n)

    def run():
        h = [hashlib.sha256(), hashlib.sha256()]
        metas = []

        def sink(fr, au, meta):
            h[0].update(fr)
            h[1].update(au)
            metas.append(meta)
        frames = dec.decode(sink=sink)
        return frames, h[0].hexdigest(), h[1].hexdigest(), metas
    want = run()
    dec.open_stream(str(path), 0, 64 << 20)          # (frees the resident capture)
    free_open = device_memory(0)[0]
    dec.ctx.stream_close()
    used = device_memory(0)[0] - free_open          # what the open stream holds
    dec.open_stream(str(path), 0, 64 << 20)
    got = run()
    st = dec.ctx.stream_stats()
    assert want[0] == got[0] >= 1400
    assert got[1:3] == want[1:3]
    assert got[3] == want[3]
    assert 0 < used < 96 << 20, used             # the ring (+ slack), not 2.4 GB
    assert st['bytes_read'] >= got[3][-1]['nextsample']      # (the 10-bit EOF guard stops at ~1.9e9)
    print('60 s: %d frames; ring 64 MiB used %.1f MiB of HBM; read %.2f GB in %.2f s; launch waits %d (%.3f s); '
          'reader waited %.2f s for space' % (got[0], used / 2 ** 20, st['bytes_read'] / 1e9, st['read_s'],
                                              st['launch_waits'], st['launch_wait_s'], st['space_wait_s']))
    dec.ctx.close()
