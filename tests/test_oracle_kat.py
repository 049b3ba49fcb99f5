"""Known-answer tests pinning the oracle restatement to the reference source formulas.

The reference ships no tests, fixtures or golden vectors and may
not be executed here, so each KAT below derives its expected
value analytically from the cited reference lines.
"""
import numpy as np
import pytest

from oracle.capture import FMT_LDS, FMT_R30, FMT_S16, FMT_U8, Capture, pack_lds, pack_r30
from oracle.demod import RFDemod, inrange, unwrap_hilbert
from oracle.field import calczc, scale
from oracle.params import HILBERT_FIR, FilterSet, system_params


# ---- loaders: lddutils.py:131-229 ---------------------------------------------------
def test_loader_u8_s16():
    raw = bytes(range(256)) * 4
    c = Capture(raw, FMT_U8)
    assert np.array_equal(c.load(10, 5), np.arange(10, 15, dtype=np.uint8))
    assert c.load(1020, 100).size == 4           # short read at EOF
    s = (np.arange(-50, 50, dtype='<i2')).tobytes()
    c = Capture(s, FMT_S16)
    assert np.array_equal(c.load(3, 4), np.array([-47, -46, -45, -44], dtype=np.int16))


def test_loader_r30_bitfields():
    # word = a | b << 10 | c << 20  (lddutils.py:166-171); sample offsets mod 3
    vals = np.array([1, 1023, 512, 7, 300, 0, 999, 5, 6], dtype=np.uint16)
    c = Capture(pack_r30(vals), FMT_R30)
    assert np.array_equal(c.load(0, 9), vals.astype(np.int16))
    assert np.array_equal(c.load(4, 3), vals[4:7].astype(np.int16))
    w = np.frombuffer(pack_r30(vals[:3]), '<u4')[0]
    assert w == 1 | (1023 << 10) | (512 << 20)


def test_loader_lds_bitfields():
    # 5 bytes -> 4 samples, MSB-first (lddutils.py:213-227)
    b = bytes([0b10101010, 0b11001100, 0b11110000, 0b00001111, 0b01010101])
    c = Capture(b * 3, FMT_LDS)
    s = c.load(0, 4)
    assert s[0] == (0b10101010 << 2) | (0b11001100 >> 6)
    assert s[1] == ((0b11001100 & 0x3f) << 4) | (0b11110000 >> 4)
    assert s[2] == ((0b11110000 & 0xf) << 6) | (0b00001111 >> 2)
    assert s[3] == ((0b00001111 & 3) << 8) | 0b01010101
    vals = np.arange(0, 1024, 7, dtype=np.uint16)[:100]
    c = Capture(pack_lds(vals), FMT_LDS)
    assert np.array_equal(c.load(5, 48), vals[5:53])
    # the reference's broadcasting raises for read lengths that are not a multiple of 4
    from oracle.capture import LoaderShapeError
    with pytest.raises(LoaderShapeError):
        c.load(5, 50)


# ---- system constants: lddecode_core.py:30-117 ---------------------------------------
def test_system_constants():
    sp, _ = system_params('NTSC')
    assert sp['outlinelen'] == 910
    assert abs(sp['line_period'] - 63.55555555555556) < 1e-12
    rf = FilterSet(system='NTSC')
    assert rf.linelen == 2542
    assert rf.iretohz(0) == 8100000 and abs(rf.iretohz(100) - 9314285.714285715) < 1e-6
    sp, _ = system_params('PAL')
    assert sp['outlinelen'] == 1135
    assert FilterSet(system='PAL').linelen == 2560


def test_audio_slices():
    rf = FilterSet(system='NTSC')
    F = rf.Filters
    assert F['audio_fdslice_lo'] == slice(791, 1303) and F['audio_fdslice_hi'] == slice(15081, 15593)
    assert F['audio_lowfreq'] == 1931818.0
    assert F['freq_arf'] == 2500000.0


def test_hilbert_fir_is_one_sided():
    h = np.fft.fft(HILBERT_FIR, 16384)
    pos, neg = np.abs(h[100:8000]).mean(), np.abs(h[8400:16300]).mean()
    assert pos > 0.9 and neg < 0.1


# ---- FM demod: lddutils.py:320-334 -----------------------------------------------------
def test_unwrap_hilbert_constant_tone():
    fs, f0 = 40e6, 8.1e6
    n = np.arange(4096)
    h = np.exp(2j * np.pi * f0 * n / fs)
    d = unwrap_hilbert(h, fs)
    assert d[0] == 0
    assert np.allclose(d[1:], f0, rtol=0, atol=1e-5)


def test_unwrap_hilbert_negative_frequency_folds():
    fs = 40e6
    n = np.arange(256)
    h = np.exp(-2j * np.pi * 1e6 * n / fs)        # -1 MHz folds to fs - 1 MHz
    d = unwrap_hilbert(h, fs)
    assert np.allclose(d[1:], fs - 1e6, atol=1e-5)


def test_demodblock_recovers_fm_carrier():
    rf = RFDemod(system='NTSC')
    n = np.arange(16384)
    x = 100 + 90 * np.cos(2 * np.pi * rf.iretohz(50) * n / 40e6)
    video, _ = rf.demodblock(x, 0)
    mid = video['demod'][2000:14000]
    assert abs(np.median(mid) - rf.iretohz(50)) < 200


# ---- threshold crossing: lddutils.py:265-303 ---------------------------------------------
def test_calczc_linear_interpolation():
    d = np.array([0.0, 1.0, 2.0, 3.0, 4.0])
    assert calczc(d, 0, 2.5) == pytest.approx(2.5)
    assert calczc(d, 0, 10.0) is None
    f = d[::-1].copy()
    assert calczc(f, 0, 1.25) == pytest.approx(2.75)


# ---- spline resample: lddutils.py:83-97 ----------------------------------------------------
def test_scale_reproduces_cubic_exactly():
    x = np.arange(3000, dtype=float)
    y = 1e-6 * (x - 1500) ** 3 + 3 * x + 7         # a cubic: not-a-knot spline is exact
    out = scale(y, 100.25, 2642.75, 910)
    xs = np.linspace(0.25, 2542.5 + 0.25, 911)[:-1] + 100
    assert np.allclose(out, 1e-6 * (xs - 1500) ** 3 + 3 * xs + 7, rtol=0, atol=1e-7)


# ---- IRE -> uint16: lddecode_core.py:1139-1142 ------------------------------------------------
def test_ire_to_u16_mapping():
    sp, _ = system_params('NTSC')
    for ire in (-40, 0, 7.5, 100):
        hz = sp['ire0'] + sp['hz_ire'] * ire
        red = (hz - sp['ire0']) / sp['hz_ire'] - sp['vsync_ire']
        val = np.uint16(np.clip(red * (50176 / 140) + 1024, 0, 65535) + 0.5)
        assert val == int((ire + 40) * 358.4 + 1024 + .5)


def test_inrange():
    assert inrange(np.array([1.0, 2.0, 3.0]), 1.5, 3.0).tolist() == [False, True, True]
