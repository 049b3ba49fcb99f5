"""Read-start probes (csrc/demod.hip ldg_k_demod_probe / ldg_k_probe_pick, LDG_READ_PROBE):
they choose where speculative reads start, never what a decode outputs.

GPU: a PAL capture whose field starts wander a sample or two off the period grid
(the synthetic capture's first seconds, profiles/r04_f_pal_chain.json) decoded with
probes and without: the probes move predicted reads (fewer reads decoded), and every
frame, its audio and its metadata are identical.  The model-level checks (a chain
with signal-borne start jitter, the auto mode) are in test_planner.py.
"""
import json

import numpy as np
import pytest

from ldgpu.decoder import GPUDecoder
from ldgpu.synth import make_capture


def _decode(monkeypatch, data, probe):
    monkeypatch.setenv('LDG_PROBE', probe)
    dec = GPUDecoder(system='PAL', batch=32)
    dec.set_capture(data, 0)
    out = []
    dec.decode(sink=lambda fr, au, m: out.append((np.array(fr, copy=True), np.array(au, copy=True), m)))
    return out, dec.stats


@pytest.mark.gpu
def test_probes_move_reads_not_results(monkeypatch):
    data = np.frombuffer(make_capture(int(40e6 * 1.5), 'u8', system='PAL', clv=True, first_frame=3000,
                                      seed=20181018), np.uint8)
    off, s0 = _decode(monkeypatch, data, '0')
    on, s1 = _decode(monkeypatch, data, '1')
    assert s1.get('probes', 0) > 0 and s1.get('probe_moved', 0) > 0
    assert s1['reads'] < s0['reads'], (s1['reads'], s0['reads'])
    assert len(on) == len(off) > 20
    for (f0, a0, m0), (f1, a1, m1) in zip(off, on):
        assert np.array_equal(f0, f1)
        assert np.array_equal(a0, a1)
        assert json.dumps(m0, sort_keys=True, default=str) == json.dumps(m1, sort_keys=True, default=str)
