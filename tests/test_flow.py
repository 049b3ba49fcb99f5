"""The 3D comb with optical flow (comb-ntsc -d 3; comb-ntsc.cxx:600-662,851-858).

BUILD-DEFINED, PARITY UNPINNED: the reference's flow is OpenCV's
calcOpticalFlowFarneback, absent here; oracle/farneback.py restates it (steps,
parameters, borders) in float64.  CPU: closed-form known answers pin that
restatement (no motion gives no flow, a translated pattern gives its shift, the
weight map's formula).  GPU: csrc/flow.hip through the comb within +-1 LSB of
the oracle's comb (oracle/comb.py Comb3DFlow).
"""
import numpy as np
import pytest

from oracle import farneback as fb


def pattern(seed=1, shape=(252, 840)):
    """A smooth random texture (8-pixel blocks blurred): the flow has structure to lock on."""
    from scipy.ndimage import gaussian_filter
    rng = np.random.default_rng(seed)
    a = np.kron(rng.uniform(0, 60000, (shape[0] // 8 + 1, shape[1] // 8 + 1)), np.ones((8, 8)))[:shape[0], :shape[1]]
    return gaussian_filter(a, 3)


def test_no_motion_gives_no_flow():
    a = pattern()
    f = fb.farneback(a, a)
    # exactly 0 away from the edges; the edge rows / columns (OpenCV's 'outside' branch of
    # UpdateMatrices) leave a small residue within the 61-pixel box
    assert np.abs(f).max() < 0.05
    assert np.abs(f[64:-64, 128:-128]).max() < 1e-3


@pytest.mark.parametrize('dy,dx', [(0, 3), (-2, 0), (1, -2)])
def test_translation_gives_its_shift(dy, dx):
    """calcOpticalFlowFarneback(prev, next): prev(y, x) = next(y + fy, x + fx); a pattern
    moved by (dy, dx) from next to prev gives flow (-dx, -dy) in the interior."""
    a = pattern(seed=2)
    b = np.roll(a, (dy, dx), axis=(0, 1))
    f = fb.farneback(b, a)
    inner = f[48:-48, 96:-96]
    assert np.median(inner[..., 0]) == pytest.approx(-dx, abs=1e-3)
    assert np.median(inner[..., 1]) == pytest.approx(-dy, abs=1e-3)


def test_initial_flow_converges_to_the_same_shift():
    a = pattern(seed=3)
    b = np.roll(a, 2, axis=1)
    f0 = fb.farneback(b, a)
    f1 = fb.farneback(b, a, f0)           # OPTFLOW_USE_INITIAL_FLOW (the reference's third call on)
    assert np.median(f1[48:-48, 96:-96, 0]) == pytest.approx(-2, abs=1e-3)


def test_weight_map_formula():
    """c = 1 - clamp((|(fy, 2 fx)| - core) / range, 0, 1), the smaller field, rows 2y / 2y+1,
    columns 70..909 (comb-ntsc.cxx:633-650); 0 elsewhere."""
    f0 = np.zeros((252, 840, 2))
    f1 = np.zeros((252, 840, 2))
    f0[..., 0] = 30.0                   # |(0, 60)| = 60
    f1[..., 1] = 20.0                   # |(20, 0)| = 20
    k = fb.combk_from_flow(f0, f1, 0.0, 179.2)
    assert k.shape == (525, 910)
    assert k[0, 70] == pytest.approx(1 - 60 / 179.2) and k[503, 909] == k[0, 70]
    assert (k[504:] == 0).all() and (k[:, :70] == 0).all()


def test_gaussian_kernels():
    assert fb.gaussian_kernel(3, 0).tolist() == [0.25, 0.5, 0.25]
    k = fb.gaussian_kernel(9, 1.5)
    assert k.sum() == pytest.approx(1.0) and k[4] == k.max() and np.allclose(k, k[::-1])


@pytest.mark.gpu
@pytest.mark.parametrize('opts', [dict(), dict(black_ire=0.0, nr_c=1.0)])
def test_gpu_comb3d_optical_flow_matches_oracle(gpu_ctx_ntsc, opts):
    """The GPU flow (csrc/flow.hip) inside the 3D comb against the oracle's, +-1 LSB, in calls
    of 2 and 3 frames (the flow and the held frames cross the call boundary)."""
    import sys
    import os
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_comb import frames_3d
    from oracle.comb import Comb3DFlow
    ctx, _ = gpu_ctx_ntsc
    fr = frames_3d(seed=19, n=5)
    ctx.comb_set_opts(opticalflow=True, **opts)
    try:
        ctx.comb_reset()
        g = np.concatenate([ctx.comb_ntsc3d(fr[:2]), ctx.comb_ntsc3d(fr[2:])])
        o = Comb3DFlow(**opts).process(fr)
        assert g.shape == o.shape == (3, 480, 744, 3)
        d = np.abs(g.astype(np.int64) - o.astype(np.int64))
        assert d.max() <= 1, (d.max(), np.argwhere(d > 1)[:5])
    finally:
        ctx.comb_set_opts()
        ctx.comb_reset()
