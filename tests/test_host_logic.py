"""CPU tests of the product's host-side logic against the oracle (no GPU)."""
import numpy as np
import pytest

from ldgpu import decoder as D
from ldgpu.formats import FMT_LDS, FMT_R30, FMT_S16, FMT_U8, pack_lds, pack_r30
from ldgpu.rfparams import RFTables
from oracle.capture import pack_lds as o_pack_lds, pack_r30 as o_pack_r30
from oracle.demod import RFDemod
from oracle.field import downscale_audio
from oracle.framer import TrackedCapture


@pytest.mark.parametrize('system', ['NTSC', 'PAL'])
def test_filter_tables_match_oracle(system):
    """Host tables (ldgpu.rfparams) == oracle RFDecode tables, bit for bit."""
    t = RFTables(system)
    o = RFDemod(system=system).Filters
    pairs = {'rfvideo': 'RFVideo', 'mtf': 'MTF', 'fvideo': 'FVideo', 'fvideo05': 'FVideo05',
             'fvideoburst': 'FVideoBurst', 'fpsync': 'FPsync', 'audio_lfilt': 'audio_lfilt',
             'audio_rfilt': 'audio_rfilt', 'audio_lpf2': 'audio_lpf2'}
    if system == 'PAL':
        pairs['fvideopilot'] = 'FVideoPilot'
    for k, ok in pairs.items():
        assert np.array_equal(t.tables[k], o[ok]), k
    p = t.params()
    orf = RFDemod(system=system)
    assert p['audio_lowfreq'] == o['audio_lowfreq'] and p['freq_arf'] == o['freq_arf']
    assert p['linelen'] == orf.linelen and p['outlinelen'] == orf.SysParams['outlinelen']
    assert p['sync_lo'] == orf.iretohz(-55) and p['sync_hi'] == orf.iretohz(-25)


@pytest.mark.parametrize('start', [0, 500, 1024, 1025, 385743, 10 ** 9 + 7])
def test_read_geometry_matches_demod_grid(start):
    rf = RFDemod(system='NTSC')
    s0, end, starts = rf.block_starts(start, 1000000)
    g = D.read_geometry(start)
    assert g == (s0, end, starts[-1])
    assert len(starts) <= 66


@pytest.mark.parametrize('fmt', [FMT_U8, FMT_S16, FMT_R30, FMT_LDS])
def test_loader_tell_matches_reference_read(fmt):
    n = 300000
    vals = (np.arange(n) % 1000).astype(np.uint16)
    if fmt == FMT_U8:
        raw = (vals % 256).astype(np.uint8).tobytes()
    elif fmt == FMT_S16:
        raw = vals.astype('<i2').tobytes()
    elif fmt == FMT_R30:
        raw = pack_r30(vals)
    else:
        raw = pack_lds(vals)
    cap = TrackedCapture(raw, fmt)
    for s in (0, 12345, 200000, n - 20000, n - 1000):
        try:
            cap.load(s, 16384)
        except Exception:
            pass
        assert D.loader_tell(fmt, s, len(raw)) == cap.pos


def test_pack_helpers_agree():
    v = np.random.default_rng(1).integers(0, 1024, 999).astype(np.uint16)
    assert pack_r30(v) == o_pack_r30(v)
    assert pack_lds(v) == o_pack_lds(v)


@pytest.mark.parametrize('lc,offset', [(262, 0.0), (263, 1.5111111111111575e-05), (263, 2.07e-5)])
def test_audio_offset_chain_matches_downscale_audio(lc, offset):
    """GPUField's host-side next offset == downscale_audio's (lddecode_core.py:484)."""
    class FakeInfo:
        status = 0; istop = 1; linecount = lc; nextfieldoffset = 0; npeaks = 400; nvsync = 2; tbcstart = 0
        vbi_minutes = vbi_seconds = vbi_clvframe = vbi_framenr = vbi_status = -2147483648
        vbi_isclv = 0; linecode_ok = [0, 0, 0]; linecode = [[0] * 6] * 3
    t = RFTables('NTSC')
    f = D.GPUField(FakeInfo(), 0, 0, 1, offset, t.system, None)
    rf = RFDemod(system='NTSC')
    ll = np.arange(lc + 4) * 2542.0 + 1000
    audio = {'audio_left': np.full(20000, 2.3e6), 'audio_right': np.full(20000, 2.8e6)}
    _, nxt = downscale_audio(audio, ll, rf, lc, offset)
    assert f.audio_next_offset == nxt


def test_predictor_is_exact_for_stable_ntsc():
    """r[k] = r[k-6] + 4,004,000 (3 NTSC frames at 40 MSPS is an integer number of samples)."""
    t = RFTables('NTSC')
    assert t.freq_hz * 3 / t.system.fps == pytest.approx(4004000, abs=1e-6)


def test_arange_last_matches_numpy():
    """GPUField's audio offset recurrence uses np.arange(...)[-1] without the array
    (downscale_audio, lddecode_core.py:432-437, 484): bit-identical to numpy."""
    from ldgpu.decoder import arange_last
    rng = np.random.default_rng(7)
    gap = 1 / 48000.0
    for i in range(20000):
        start = float(rng.uniform(0, gap))
        lc = int(rng.integers(250, 320))
        ft = (63.5555555556 * lc) / 1000000
        assert arange_last(start, ft + gap, gap) == np.arange(start, ft + gap, gap, dtype=np.double)[-1]
    for i in range(5000):
        st = float(rng.uniform(-5, 5))
        step = float(rng.uniform(1e-4, 1))
        stop = st + float(rng.uniform(step, 100 * step))
        assert arange_last(st, stop, step) == np.arange(st, stop, step)[-1]


def _bench():
    import importlib.util
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location('ldg_bench', os.path.join(root, 'bench.py'))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_demod_issue_lag_classifies_launches():
    """bench.py checks.demod_issue: a launch is host-late when no demod was executing
    before it started (gap > 5 us) and the host issued it after the last one ended."""
    b = _bench()
    # (start, end, host issue, host ms): #1 queued early (overlaps #0), #2 issued late into an
    # idle GPU, #3 issued early but started after a gap (GPU-side), #4 a launch with no workgroup
    tab = np.array([[0.0, 2.0, -1.0, 0.0], [1.5, 4.0, -0.5, 0.0], [4.3, 6.0, 4.2, 0.0],
                    [6.4, 8.0, 3.0, 0.0], [np.nan, np.nan, 7.0, 0.0]])
    r = b.demod_issue_lag(tab)
    assert r['launches'] == 3 and r['idle_gaps'] == 2 and r['host_late'] == 1
    assert abs(r['host_late_ms'] - 0.2) < 1e-9 and abs(r['idle_ms'] - 0.7) < 1e-9
    assert b.demod_issue_lag(tab[:1]) is None
