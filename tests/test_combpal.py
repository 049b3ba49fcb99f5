"""PAL Y/C decoder (SURVEY §8 f row F2; BUILD-DEFINED, parity with the reference
unpinned -- it has no PAL comb for the 1135x625 geometry): the oracle
(oracle/combpal.cpp, an adaptation of attic2/comb-pal.cxx's dim=2 path) pinned
by closed-form answers, and the GPU kernels against it (+-1 LSB)."""
import numpy as np
import pytest

from oracle.comb import CombPAL

IRESCALE = 376.32
M = 240.0 * 255 / 100
NR_B = [1.141291975113614e-04, -1.857019211291029e-03, -4.499636864042073e-03, -5.577680979937061e-03,
        -4.423694440267179e-04, 1.309163063177155e-02, 2.861211356202848e-02, 3.029931283148555e-02,
        1.098965697652802e-03, -6.398130386469833e-02, -1.492080690537196e-01, -2.223459379380252e-01,
        7.479077367478024e-01, -2.223459379380252e-01, -1.492080690537196e-01, -6.398130386469833e-02,
        1.098965697652803e-03, 3.029931283148557e-02, 2.861211356202848e-02, 1.309163063177156e-02,
        -4.423694440267185e-04, -5.577680979937061e-03, -4.499636864042074e-03, -1.857019211291030e-03,
        1.141291975113614e-04]


def ire_to_u16(ire):
    return int(np.clip((ire + 43.122874) * IRESCALE, 1, 65535))


def pal_frame(y_ire, a=0, b=0):
    """1135x625 frame: luma plus a 4fsc chroma pattern (a, b, -a, -b) that inverts every 4
    frame rows (2 lines of a field: 567.5 subcarrier cycles), in the picture and the burst."""
    base = ire_to_u16(y_ire)
    fr = np.zeros((625, 1135), dtype=np.int64)
    c = np.array([a, b, -a, -b], dtype=np.int64)
    for l in range(625):
        s = 1 if (l // 4) % 2 == 0 else -1
        fr[l, :] = base + s * c[np.arange(1135) % 4]
        fr[l, 0] = 32768                     # not the NTSC 16384 phase flag
    return fr.astype(np.uint16)


def expected(y_ire, u=0.0, v=0.0):
    y = float(ire_to_u16(y_ire))
    a = float(np.clip(sum(t * y for t in NR_B), -IRESCALE, IRESCALE))
    yi = -43.122874 + int(y - a) / IRESCALE
    r = yi + 1.13983 * v
    g = yi - 0.58060 * v - u * 0.39465
    b = yi + u * 2.032
    return np.clip(np.array([r, g, b]) * M, 0, 65535)


def test_oracle_pal_flat_grey_kat():
    out = CombPAL().process(pal_frame(50.0)[None])[0].astype(np.float64)
    core = out[10:560, 20:1000].reshape(-1, 3)
    assert np.abs(core - np.floor(expected(50.0))).max() <= 1


@pytest.mark.parametrize('y_ire,a,b', [(40.0, 1500, -900), (60.0, -700, 1200)])
def test_oracle_pal_solid_colour_kat(y_ire, a, b):
    """Burst and picture carry the same chroma: each line is rotated so its burst sits
    at 135 degrees, so every pixel decodes to U = -V = -|c| * 10/8 / irescale / sqrt 2
    (the V-switch flip (U, V) -> (-V, -U) leaves that vector unchanged)."""
    out = CombPAL().process(pal_frame(y_ire, a, b)[None])[0].astype(np.float64)
    mag = np.hypot(a, b) * (10 / 8.0) / IRESCALE
    exp = expected(y_ire, -mag / np.sqrt(2), mag / np.sqrt(2))
    core = out[10:560, 60:950].reshape(-1, 3)
    assert np.abs(core - np.floor(exp)).max() <= 1
    assert np.ptp(core.mean(0)) > 100


def test_oracle_pal_state_carries_across_calls():
    fr = np.stack([pal_frame(30.0 + 10 * k, 800, 400) for k in range(3)])
    one = CombPAL().process(fr)
    c = CombPAL()
    two = np.concatenate([c.process(fr[:1]), c.process(fr[1:])])
    assert np.array_equal(one, two)


def pal_frames_noisy(seed=4, n=3):
    rng = np.random.default_rng(seed)
    out = []
    for k in range(n):
        fr = pal_frame(45.0 + 5 * k, 1100 - 300 * k, -600 + 200 * k).astype(np.int64)
        fr[:, 300 + 50 * k:380 + 50 * k] += 7000
        fr += rng.integers(-250, 250, (625, 1135))
        fr[:, 0] = 32768
        out.append(np.clip(fr, 0, 65535).astype(np.uint16))
    return np.stack(out)


@pytest.mark.gpu
def test_gpu_comb_pal_matches_oracle(gpu_ctx_ntsc):
    ctx, _ = gpu_ctx_ntsc
    fr = np.concatenate([pal_frames_noisy(), pal_frame(40.0, 1500, -900)[None], pal_frame(50.0)[None]])
    ctx.comb_reset()
    g = np.concatenate([ctx.comb_pal(fr[:2]), ctx.comb_pal(fr[2:])])
    o = CombPAL().process(fr)
    d = np.abs(g.astype(np.int64) - o.astype(np.int64))
    assert d.max() <= 1, d.max()
    assert (d > 0).mean() < 1e-3
    ctx.comb_reset()


@pytest.mark.gpu
@pytest.mark.parametrize('wide', [False, True])
def test_comb_pal_cli_stream(wide):
    """comb_pal.py as encode-pal's `comb-pal -d 2 -` stream filter: 974-wide rgb48 frames
    (attic2/comb-pal.cxx:883-884's geometry, what encode-pal's ffmpeg -s 974x576 reads), or
    the whole 1057 columns with -W; against the oracle on the same frames (+-1 LSB)."""
    import os
    import subprocess
    import sys
    from oracle.comb import CombPAL
    cli = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'ld-decode_amd', 'comb_pal.py')
    fr = pal_frames_noisy(seed=6, n=3)
    r = subprocess.run([sys.executable, cli, '-d', '2', '--chunk', '2'] + (['-W'] if wide else []) + ['-'],
                       input=fr.tobytes() + b'\x00' * 100, capture_output=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    exp = CombPAL().process(fr)
    if not wide:
        exp = exp[:, :, :974]
    got = np.frombuffer(r.stdout, dtype=np.uint16).reshape(exp.shape)
    assert np.abs(got.astype(np.int64) - exp.astype(np.int64)).max() <= 1
