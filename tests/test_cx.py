"""CX expander (row F4, cx-expander.cxx): the library's host implementation
(ldg_cx_process) against the pure-Python oracle (oracle/cx.py), which is pinned
by closed-form answers.  No GPU involved: the chain is sequential host code."""
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import cx as ocx

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, 'ld-decode_amd'))


def tone(n, amp, f=1000.0, fs=48000.0, phase=0.0):
    t = np.arange(n)
    v = amp * np.sin(2 * np.pi * f * t / fs + phase)
    return (np.round(v) + 32768).astype(np.uint16)


def stereo(l, r):
    return np.stack([l, r], axis=1)


def amp(x):
    """peak of the last 20 ms (steady state) around the 32768 offset"""
    return np.abs(x[-960:].astype(np.float64) - 32768).max()


def test_oracle_silence_is_midscale():
    out = np.array(ocx.CX().process([(32768, 32768)] * 2000))
    assert (out == 32768).all()


def test_oracle_unity_region_below_threshold():
    """Peaks after the 500 Hz high-pass below 6500 * m14db = 1297 give val = 0: the
    output is 0.4 * m14db * HP40(x), a 1 kHz tone scaled by 0.0798 (HP40 ~ 1 there)."""
    a = 400.0
    x = tone(9600, a)
    out = np.array(ocx.CX().process(stereo(x, x).tolist()))
    assert amp(out[:, 0]) == pytest.approx(0.4 * ocx.M14DB * a, rel=0.02)


def test_oracle_two_to_one_expansion():
    """Far above the threshold the gain is peak / 1297: output amplitude grows as the
    square of the input's (x2 in -> x4 out)."""
    outs = []
    for a in (6000.0, 12000.0):
        x = tone(48000, a)
        outs.append(amp(np.array(ocx.CX().process(stereo(x, x).tolist()))[:, 0]))
    assert outs[1] / outs[0] == pytest.approx(4.0, rel=0.05)


def test_native_matches_oracle_bit_exact():
    from ldgpu.native import CXExpander
    rng = np.random.default_rng(9)
    n = 12000
    l = (tone(n, 9000.0) .astype(np.int64) + rng.integers(-2000, 2000, n))
    r = tone(n, 3000.0, f=440.0, phase=1.0).astype(np.int64)
    r[5000:5200] = 65535                                   # clipping
    x = stereo(np.clip(l, 0, 65535), np.clip(r, 0, 65535)).astype(np.uint16)
    cx = CXExpander()
    got = np.concatenate([cx.process(x[:777]), cx.process(x[777:5000]), cx.process(x[5000:])])
    exp = np.array(ocx.CX().process(x.tolist()), dtype=np.uint16)
    assert np.array_equal(got, exp)


def test_cli_drops_partial_block():
    rng = np.random.default_rng(2)
    x = stereo(tone(3 * 1024, 7000.0), tone(3 * 1024, 2000.0, f=700.0)).astype('<u2')
    data = x.tobytes() + rng.integers(0, 256, 1000, dtype=np.uint8).tobytes()
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'ld-decode_amd', 'cx_expander.py')], input=data,
                       capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    got = np.frombuffer(r.stdout, dtype='<u2').reshape(-1, 2)
    assert got.shape == (3 * 1024, 2)
    assert np.array_equal(got, ocx.stream(data))


@pytest.mark.gpu
def test_native_matches_oracle_bit_exact_on_gpu_box():
    """The same check in the GPU box's run (libldgpu.so as shipped there: the driver's
    record of row F4); the expander itself is host code in the library."""
    test_native_matches_oracle_bit_exact()
    test_cli_drops_partial_block()
