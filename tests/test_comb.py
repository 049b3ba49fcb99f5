"""2D NTSC comb (comb-ntsc.cxx dim=2): oracle known-answer tests (CPU) and GPU parity.

The oracle is oracle/comb2d.cpp, a C++ restatement of the reference comb's
default path (PARITY UNPINNED against the reference binary, which cannot run
here: SURVEY §8 C1/C2).  It is pinned here by closed-form answers:
  * a flat grey field has no chroma: RGB = (IRE - 7.5) * 100/92.5 * 604.16;
  * a solid-colour 4fsc field with NTSC line-to-line phase inversion decodes to
    the I/Q it was built from (the 2D comb, the hold, AdjustY and the colour
    LPF all have unit gain at DC);
  * the burst-level EMA of a constant burst is that constant.
GPU results must match the oracle within +-1 LSB.
"""
import numpy as np
import pytest

from oracle.comb import Comb2D

IRESCALE, IREBASE = 358.4, 1024.0
M = 236.0 * 256 / 100


def ire_to_u16(ire):
    return int(np.clip(((ire + 40) * IRESCALE) + IREBASE, 1, 65535))


def frame_solid(y_ire, a=0, b=0, burst_ire=20.0):
    """910x525 frame: luma y_ire plus a 4fsc chroma pattern c[h % 4] = (a, b, -a, -b),
    sign flipping on every line of a field (frame rows l and l+2), burst flag/level in px 0/1."""
    base = ire_to_u16(y_ire)
    fr = np.zeros((525, 910), dtype=np.int64)
    c = np.array([a, b, -a, -b], dtype=np.int64)
    for l in range(525):
        s = 1 if (l // 2) % 2 == 0 else -1
        fr[l, :] = base + s * c[np.arange(910) % 4]
        fr[l, 0] = 16384 if s > 0 else 32768
        fr[l, 1] = int(burst_ire * IRESCALE)
    return fr.astype(np.uint16)


# deemp.h f_nr taps (DoYNR's high pass); its DC gain is not exactly 0, so a flat
# field loses y * sum(taps) (clipped to +-1 IRE) -- the reference's behaviour.
NR_B = [1.141291975113614e-04, -1.857019211291029e-03, -4.499636864042073e-03, -5.577680979937061e-03,
        -4.423694440267179e-04, 1.309163063177155e-02, 2.861211356202848e-02, 3.029931283148555e-02,
        1.098965697652802e-03, -6.398130386469833e-02, -1.492080690537196e-01, -2.223459379380252e-01,
        7.479077367478024e-01, -2.223459379380252e-01, -1.492080690537196e-01, -6.398130386469833e-02,
        1.098965697652803e-03, 3.029931283148557e-02, 2.861211356202848e-02, 1.309163063177156e-02,
        -4.423694440267185e-04, -5.577680979937061e-03, -4.499636864042074e-03, -1.857019211291030e-03,
        1.141291975113614e-04]


def ynr(y_u16):
    a = 0.0
    for t in NR_B:
        a += t * y_u16
    return y_u16 - float(np.clip(a, -IRESCALE, IRESCALE))


def expected_rgb(y_ire, i_val=0.0, q_val=0.0, burst_ire=20.0):
    """RGB::conv (comb-ntsc.cxx:124-147) of y (u16, after DoYNR) and I/Q samples scaled by 10/aburstlev."""
    yu = int(ynr(float(ire_to_u16(y_ire))))
    y = -40 + (yu - IREBASE) / IRESCALE
    y = (y - 7.5) * (100 / 92.5)
    k = 10 / burst_ire
    q = i_val * k / IRESCALE
    i = q_val * k / IRESCALE
    r = y + .956 * i + .621 * q
    g = y - .272 * i - .647 * q
    b = y - 1.106 * i + 1.703 * q
    return np.clip(np.array([r, g, b]) * M, 0, 65535)


def test_oracle_flat_grey_kat():
    c = Comb2D()
    out = c.process(frame_solid(50.0)[None])[0]
    exp = expected_rgb(50.0)
    core = out[20:460, 40:700].reshape(-1, 3).astype(np.float64)
    assert np.abs(core - np.floor(exp)).max() <= 1
    assert c.aburstlev == pytest.approx(20.0, rel=1e-12)


@pytest.mark.parametrize('y_ire,a,b', [(40.0, 1500, -900), (60.0, -700, 1200), (25.0, 400, 400)])
def test_oracle_solid_colour_kat(y_ire, a, b):
    """A pattern c[h % 4] = (a, b, -a, -b) on rows flagged 16384 (the sign flipping
    line to line within a field) decodes to the held samples I = -a, Q = b:
    SplitIQ's phase table (:446-452) on the 2D comb output -c (:341-343)."""
    out = Comb2D().process(frame_solid(y_ire, a, b)[None])[0].astype(np.float64)
    core = out[40:440, 100:700].reshape(-1, 3)
    assert np.abs(core - np.floor(expected_rgb(y_ire, -a, b))).max() <= 1
    assert np.ptp(core.mean(0)) > 100          # a colour, not grey


def test_oracle_state_carries_across_calls():
    fr = np.stack([frame_solid(30.0, 800, 400, burst_ire=b) for b in (10.0, 25.0, 40.0)])
    one = Comb2D().process(fr)
    c = Comb2D()
    two = np.concatenate([c.process(fr[:1]), c.process(fr[1:])])
    assert np.array_equal(one, two)


@pytest.mark.gpu
def test_gpu_comb_matches_oracle(gpu_ctx_ntsc):
    ctx, _ = gpu_ctx_ntsc
    rng = np.random.default_rng(7)
    frames = [frame_solid(40.0, 1500, -900), frame_solid(60.0, -700, 1200, burst_ire=30.0)]
    noisy = frame_solid(50.0, 1000, 300).astype(np.int64) + rng.integers(-300, 300, (525, 910))
    noisy[:, :2] = frame_solid(50.0)[:, :2]
    frames.append(np.clip(noisy, 0, 65535).astype(np.uint16))
    fr = np.stack(frames)
    ctx.comb_reset()
    g = np.concatenate([ctx.comb_ntsc(fr[:2]), ctx.comb_ntsc(fr[2:])])
    o = Comb2D().process(fr)
    d = np.abs(g.astype(np.int64) - o.astype(np.int64))
    assert d.max() <= 1, d.max()
    assert (d > 0).mean() < 1e-3


@pytest.mark.gpu
def test_gpu_comb_default_kernels_equal_option_kernels(monkeypatch):
    """At comb-ntsc's defaults the library runs one fused row kernel with the options folded
    in as constants, from a persistent grid (LDG_COMB_ROWS workgroups; 3: many rows each,
    0: one workgroup per row); its FilterIQ fallback, the three-kernel path
    (LDG_COMB_UNFUSED=1) and the option-taking kernels (LDG_COMB_GENERIC=1; all read at
    context creation) must give the same rgb48 bit for bit."""
    from ldgpu import native
    from ldgpu.rfparams import RFTables
    rf = RFTables('NTSC')
    rng = np.random.default_rng(11)
    noisy = frame_solid(45.0, 900, -400).astype(np.int64) + rng.integers(-400, 400, (525, 910))
    noisy[:, :2] = frame_solid(45.0)[:, :2]
    fr = np.stack([frame_solid(40.0, 1500, -900), np.clip(noisy, 0, 65535).astype(np.uint16)])
    out = []
    # the fused row kernel (default), its FilterIQ fallback forced (no exact warm-up after the
    # scan seed: lanes' checks fail), the three default kernels, the option-taking kernels
    for env in ({}, {'LDG_COMB_ROWS': '3'}, {'LDG_COMB_ROWS': '0'}, {'LDG_COMB_IQW': '0'}, {'LDG_COMB_UNFUSED': '1'},
                {'LDG_COMB_GENERIC': '1'}):
        for k in ('LDG_COMB_ROWS', 'LDG_COMB_IQW', 'LDG_COMB_UNFUSED', 'LDG_COMB_GENERIC'):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        ctx = native.Context('NTSC', 0, max_reads=8)
        ctx.set_filters(rf.params(), rf.tables)
        ctx.comb_reset()
        out.append(ctx.comb_ntsc(fr))
        ctx.close()
    for o in out[1:]:
        assert np.array_equal(out[0], o)


@pytest.mark.gpu
def test_gpu_comb_on_decoded_frames():
    """RF -> .tbc on the GPU -> 2D comb on the GPU, against the oracle comb of the same
    frames (+-1 LSB) and the committed golden comb hashes (bit-exact frames reported)."""
    import hashlib
    import json
    import os
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, 'golden'))
    import make_golden
    from ldgpu.decoder import GPUDecoder
    case = 'ntsc_cav_u8_0p2s'
    with open(os.path.join(here, 'golden', case + '.json')) as fh:
        gold = json.load(fh)
    dec = GPUDecoder(system='NTSC', batch=8)
    dec.set_capture(make_golden.build_capture(case), 0)
    frames = []
    dec.decode(sink=lambda fr, au, m: frames.append(fr.copy()))
    fr = np.stack(frames).reshape(-1, 525, 910)
    dec.ctx.comb_reset()
    g = dec.ctx.comb_ntsc(fr)
    o = Comb2D().process(fr)
    assert np.abs(g.astype(np.int64) - o.astype(np.int64)).max() <= 1
    exact = sum(hashlib.sha256(x.tobytes()).hexdigest() == e['comb_rgb48_sha256'] for x, e in zip(g, gold['frames']))
    print('comb: %d/%d frames bit-identical to golden' % (exact, len(g)))


# ---- 3D comb without optical flow (comb-ntsc -d 3 -F) ---------------------------------

from oracle.comb import Comb3D  # noqa: E402


def test_oracle3d_frame_delay_and_chunking():
    """Process with f = 1 (:837,860-868): nothing for the first two frames, frame k once
    frame k+1 is in; the held frames carry across calls like one process."""
    rng = np.random.default_rng(3)
    fr = np.stack([np.clip(frame_solid(40.0 + 5 * k, 900, -500).astype(np.int64)
                           + rng.integers(-200, 200, (525, 910)), 0, 65535).astype(np.uint16) for k in range(6)])
    fr[:, :, :2] = frame_solid(40.0)[:, :2]
    one = Comb3D().process(fr)
    assert one.shape[0] == 4
    c = Comb3D()
    parts = [c.process(fr[:1]), c.process(fr[1:2]), c.process(fr[2:5]), c.process(fr[5:])]
    assert [p.shape[0] for p in parts] == [0, 0, 3, 1]
    assert np.array_equal(one, np.concatenate(parts))
    # the first output is frame 1 combed with frames 0 and 2
    assert np.array_equal(one[0], Comb3D().process(fr[:3])[0])


@pytest.mark.parametrize('y_ire,a,b', [(40.0, 1500, -900), (60.0, -700, 1200)])
def test_oracle3d_solid_colour_kat(y_ire, a, b):
    """Real NTSC: the 4fsc chroma inverts from frame to frame.  With the neighbours
    inverted, |next - prev| = 0, so combk2 = 1 and the temporal estimate
    (prev + next)/2 - cur = -2c alone decodes the same I = -a, Q = b as the 2D KAT."""
    f, g = frame_solid(y_ire, a, b), frame_solid(y_ire, -a, -b)
    out = Comb3D().process(np.stack([g, f, g]))[0].astype(np.float64)
    core = out[40:440, 100:700].reshape(-1, 3)
    assert np.abs(core - np.floor(expected_rgb(y_ire, -a, b))).max() <= 1


def test_oracle3d_static_scene_has_no_chroma():
    """A frame repeated without the frame-to-frame inversion: the temporal estimate
    is 0 with full weight, so I = Q = 0 and every output pixel is grey."""
    f = frame_solid(50.0, 1200, 600)
    out = Comb3D().process(np.stack([f, f, f]))[0].astype(np.int64)
    core = out[10:470, 20:720]
    assert (core[..., 0] == core[..., 1]).all() and (core[..., 1] == core[..., 2]).all()


def test_oracle3d_motion_falls_back_to_2d():
    """Neighbours that differ by far more than p_3dcore + p_3drange give combk2 = 0 and
    combk1 = 1: away from the line ends the 3D output is the 2D output."""
    f = frame_solid(50.0, 1000, -400)
    prev, nxt = frame_solid(0.0, -1000, 400), frame_solid(100.0, -1000, 400)
    three = Comb3D().process(np.stack([prev, f, nxt]))[0].astype(np.int64)
    two = Comb2D().process(f[None])[0].astype(np.int64)
    assert np.abs(three[:, 40:700] - two[:, 40:700]).max() <= 1


def frames_3d(seed=11, n=7):
    """Alternating-phase colour frames with noise, a moving luma edge and a cut."""
    rng = np.random.default_rng(seed)
    out = []
    for k in range(n):
        s = 1 if k % 2 == 0 else -1
        fr = frame_solid(45.0 + (30.0 if k == 4 else 0.0), s * 1100, -s * 600).astype(np.int64)
        fr[:, 200 + 40 * k:260 + 40 * k] += 9000
        fr += rng.integers(-250, 250, (525, 910))
        fr[:, :2] = frame_solid(45.0, burst_ire=20.0 + k)[:, :2]
        out.append(np.clip(fr, 0, 65535).astype(np.uint16))
    return np.stack(out)


@pytest.mark.gpu
def test_gpu_comb3d_matches_oracle(gpu_ctx_ntsc):
    ctx, _ = gpu_ctx_ntsc
    fr = frames_3d()
    ctx.comb_reset()
    parts = [ctx.comb_ntsc3d(fr[:1]), ctx.comb_ntsc3d(fr[1:4]), ctx.comb_ntsc3d(fr[4:])]
    assert [p.shape[0] for p in parts] == [0, 2, 3]
    g = np.concatenate(parts)
    o = Comb3D().process(fr)
    assert g.shape == o.shape
    d = np.abs(g.astype(np.int64) - o.astype(np.int64))
    assert d.max() <= 1, d.max()
    assert (d > 0).mean() < 1e-3
    # non-default -c / -r
    ctx.comb_reset()
    g2 = ctx.comb_ntsc3d(fr, 0.5, 2.0)
    o2 = Comb3D(0.5, 2.0).process(fr)
    assert np.abs(g2.astype(np.int64) - o2.astype(np.int64)).max() <= 1
    ctx.comb_reset()


@pytest.mark.gpu
def test_gpu_comb3d_on_decoded_frames():
    """RF -> .tbc on the GPU -> 3D comb on the GPU, against the oracle's 3D comb of the
    same frames (+-1 LSB)."""
    import os
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, 'golden'))
    import make_golden
    from ldgpu.decoder import GPUDecoder
    dec = GPUDecoder(system='NTSC', batch=8)
    dec.set_capture(make_golden.build_capture('ntsc_cav_u8_0p2s'), 0)
    frames = []
    dec.decode(sink=lambda fr, au, m: frames.append(fr.copy()))
    fr = np.stack(frames).reshape(-1, 525, 910)
    assert fr.shape[0] >= 3
    dec.ctx.comb_reset()
    g = dec.ctx.comb_ntsc3d(fr)
    o = Comb3D().process(fr)
    assert g.shape[0] == fr.shape[0] - 2
    assert np.abs(g.astype(np.int64) - o.astype(np.int64)).max() <= 1


@pytest.mark.gpu
def test_gpu_comb_set_state_continues_the_chain(gpu_ctx_ntsc):
    """ldg_comb_set_state with the host chain's state over the first frames makes the
    comb of the rest equal to the uninterrupted run (the sharded --comb handover)."""
    from ldgpu.shard import comb_burst_levels, comb_chain
    ctx, _ = gpu_ctx_ntsc
    fr = frames_3d(seed=12, n=5)
    ctx.comb_reset()
    full = ctx.comb_ntsc(fr)
    ctx.comb_set_state(comb_chain(-1.0, comb_burst_levels(fr[:2])))
    part = ctx.comb_ntsc(fr[2:])
    assert np.array_equal(full[2:], part)
    ctx.comb_reset()


# ---- the burst-level EMA chain (ldg_k_comb_burst: speculative chunks + exact check) ----

def _burst_frames(n, seed):
    """n frames whose line burst levels (px 1) are random: 15-30 IRE, with ~20% of lines
    at or below the 3 IRE qualification (the EMA holds there) and the first 700 lines of
    the sequence unqualified (the chain starts uninitialised)."""
    rng = np.random.default_rng(seed)
    fr = np.repeat(frame_solid(50.0, 800, -400)[None], n, axis=0)
    lv = rng.uniform(15.0, 30.0, (n, 525))
    lv[rng.random((n, 525)) < 0.2] = rng.uniform(0.0, 3.0)
    lv.reshape(-1)[:700] = 1.0
    fr[:, :, 1] = (lv * IRESCALE).astype(np.uint16)
    return fr


def _chain_values(a, frames):
    """The reference's EMA (comb-ntsc.cxx:560-566) over lines 38..524, value per line."""
    out = []
    for b in (frames[:, 38:525, 1].astype(np.float64) / IRESCALE).reshape(-1).tolist():
        if b > 3:
            if a < 0:
                a = b
            a = (a * .99) + (b * .01)
        out.append(a)
    return np.array(out), a


@pytest.mark.gpu
@pytest.mark.parametrize('warm', [None, 16])
def test_gpu_comb_burst_chain_bit_exact(warm, monkeypatch):
    """The parallel EMA kernel equals the sequential chain bit for bit: over a call of 100
    frames (two LDS pieces, 48,700 lines), after a short call that initialised the state,
    with the default run-in (the speculative chunks meet the true chain) and with
    LDG_COMB_WARM=16 (almost every chunk fails its check: the serial fix-up path)."""
    from ldgpu import native
    from ldgpu.rfparams import RFTables
    if warm is not None:
        monkeypatch.setenv('LDG_COMB_WARM', str(warm))
    rf = RFTables('NTSC')
    ctx = native.Context('NTSC', 0, max_reads=4, max_frames=100)
    ctx.set_filters(rf.params(), rf.tables)
    fr = _burst_frames(103, seed=31 if warm is None else 32)
    ctx.comb_reset()
    ref, a = _chain_values(-1.0, fr[:3])
    ctx.comb_ntsc(fr[:3])
    got = ctx.debug(0, 50, np.float64, 3 * 487)
    assert np.array_equal(got.view(np.int64), ref.view(np.int64))
    ref, a = _chain_values(a, fr[3:])
    ctx.comb_ntsc(fr[3:])
    got = ctx.debug(0, 50, np.float64, 100 * 487)
    st = ctx.debug(0, 51, np.float64, 1)
    assert got.size == ref.size
    assert np.array_equal(got.view(np.int64), ref.view(np.int64)), np.flatnonzero(got != ref)[:10]
    assert st[0] == a


# ---- comb-ntsc's options (main's getopt, comb-ntsc.cxx:972-1091) -------------------------

def expected_grey(y_ire, black_ire=7.5, brightness=236.0, nr=True):
    """RGB::conv of a flat field (no chroma) with -I black_ire / -b brightness."""
    yu = int(ynr(float(ire_to_u16(y_ire)))) if nr else ire_to_u16(y_ire)
    y = -40 + (yu - IREBASE) / IRESCALE
    y = (y - black_ire) * (100 / (100 - black_ire))
    return float(np.clip(y * brightness * 256 / 100, 0, 65535))


@pytest.mark.parametrize('black,bright', [(0.0, 236.0), (7.5, 200.0), (0.0, 120.0)])
def test_oracle_black_level_and_brightness_kat(black, bright):
    """-I (encode-ntsc / encode-ralf run `comb -d 3 -I 0`) and -b on a flat grey field."""
    out = Comb2D(black_ire=black, brightness=bright).process(frame_solid(50.0)[None])[0]
    core = out[20:460, 40:700].reshape(-1, 3).astype(np.float64)
    assert np.abs(core - np.floor(expected_grey(50.0, black, bright))).max() <= 1


def test_oracle_ynr_off_kat():
    """-n 0: DoYNR returns before feeding (comb-ntsc.cxx:527-529): the flat field keeps its level."""
    out = Comb2D(nr_y=0.0).process(frame_solid(50.0)[None])[0]
    core = out[20:460, 40:700].reshape(-1, 3).astype(np.float64)
    assert np.abs(core - np.floor(expected_grey(50.0, nr=False))).max() <= 1


def test_oracle_bw_has_no_chroma():
    """-B: SplitIQ zeroes I and Q (:463-465), so a coloured field comes out grey."""
    out = Comb2D(bw=True).process(frame_solid(40.0, 1500, -900)[None])[0].astype(np.int64)
    core = out[10:470, 20:720]
    assert (core[..., 0] == core[..., 1]).all() and (core[..., 1] == core[..., 2]).all()


@pytest.mark.parametrize('opts', [dict(colorlpf=False), dict(colorlpf_hq=False), dict(adaptive2d=False)])
def test_oracle_solid_colour_options_kat(opts):
    """The colour LPF (either filter) has unit gain at DC and the fixed 2D weights give the
    adaptive ones' result on a uniform field: a solid colour decodes to the same I = -a, Q = b."""
    out = Comb2D(**opts).process(frame_solid(40.0, 1500, -900)[None])[0].astype(np.float64)
    core = out[40:440, 100:700].reshape(-1, 3)
    assert np.abs(core - np.floor(expected_rgb(40.0, 1500 * -1, -900))).max() <= 1


# deemp.h f_nrc (DoCNR's 17-tap high pass): DC gain sum(taps) = 0.5403, not 0
NRC_SUM = sum([-3.148569668063267e-03, -4.941974513425438e-03, -9.929538598536455e-03, -1.787793973911701e-02,
               -2.783702315543740e-02, -3.829928032339736e-02, -4.750186865627083e-02, -5.380281552534787e-02,
               9.469899799540406e-01, -5.380281552534787e-02, -4.750186865627083e-02, -3.829928032339737e-02,
               -2.783702315543740e-02, -1.787793973911701e-02, -9.929538598536455e-03, -4.941974513425442e-03,
               -3.148569668063267e-03])


@pytest.mark.parametrize('nr_c', [0.5, 2.0, 5.0])
def test_oracle_cnr_kat(nr_c):
    """-N: DoCNR (:485-521) subtracts its high pass, clipped to +-nr_c IRE, from I and Q; on
    a solid colour the high pass is NRC_SUM * I (Q), so I' = I - clip(NRC_SUM * I)."""
    clip = nr_c * IRESCALE
    i0, q0 = -1500.0, -900.0
    i1 = i0 - float(np.clip(NRC_SUM * i0, -clip, clip))
    q1 = q0 - float(np.clip(NRC_SUM * q0, -clip, clip))
    out = Comb2D(nr_c=nr_c).process(frame_solid(40.0, 1500, -900)[None])[0].astype(np.float64)
    core = out[40:440, 100:700].reshape(-1, 3)
    assert np.abs(core - np.floor(expected_rgb(40.0, i1, q1))).max() <= 1


def test_oracle_525_lines_and_debug_line():
    """-v: 525 rows from line 20 (:486,1013); rows 0..3 show the VBI copy of raw lines 40..43
    (:876-882), rows 4..15 (lines 24..35, outside SplitIQ) are black, the last 20 rows are
    never written (0); -l 100 blacks out line 125 (:586-589)."""
    fr = frame_solid(30.0)
    fr[40:44, 2:] = ire_to_u16(80.0)
    out = Comb2D(linesout=525, debugline=100).process(fr[None])[0].astype(np.int64)
    assert out.shape == (525, 744, 3)
    assert (out[505:] == 0).all()
    assert (out[4:16] == 0).all()
    assert np.abs(out[0:4, 100:700] - np.floor(expected_grey(80.0))).max() <= 1
    assert (out[125 - 20] == 0).all() and out[124 - 20].min() > 0
    dflt = Comb2D(debugline=100).process(fr[None])[0]
    assert (dflt[125 - 38] == 0).all()


COMB_OPTION_CASES = [dict(black_ire=0.0), dict(black_ire=0.0, brightness=200.0), dict(nr_y=0.0), dict(nr_y=3.0),
                     dict(nr_c=2.0), dict(nr_c=0.5, nr_y=0.5), dict(bw=True), dict(linesout=525),
                     dict(colorlpf=False), dict(colorlpf_hq=False), dict(adaptive2d=False), dict(debug_line=100),
                     dict(wide=True), dict(wide=True, linesout=525, nr_c=1.0), dict(wide=True, nr_y=3.0)]


def _opts_for_oracle(o):
    return {('debugline' if k == 'debug_line' else k): v for k, v in o.items()}


@pytest.mark.gpu
@pytest.mark.parametrize('opts', COMB_OPTION_CASES)
def test_gpu_comb_options_match_oracle(gpu_ctx_ntsc, opts):
    """The GPU comb with comb-ntsc's options (ldg_comb_set_opts) against the oracle: +-1 LSB
    on noisy colour frames, 2D and 3D (-d 3 -F)."""
    ctx, _ = gpu_ctx_ntsc
    fr = frames_3d(seed=17, n=5)
    ctx.comb_set_opts(**opts)
    try:
        ctx.comb_reset()
        g = ctx.comb_ntsc(fr)
        o = Comb2D(**_opts_for_oracle(opts)).process(fr)
        assert g.shape == o.shape
        d = np.abs(g.astype(np.int64) - o.astype(np.int64))
        assert d.max() <= 1, d.max()
        ctx.comb_reset()
        g3 = ctx.comb_ntsc3d(fr)
        o3 = Comb3D(**_opts_for_oracle(opts)).process(fr)
        assert g3.shape == o3.shape
        assert np.abs(g3.astype(np.int64) - o3.astype(np.int64)).max() <= 1
    finally:
        ctx.comb_set_opts()
        ctx.comb_reset()


def test_oracle_wide_kat():
    """-W (comb-ntsc.cxx:898-899, 974-976): 910-wide rows from x 0.  Columns 78..821 are the
    744-wide output exactly; columns 0, 1 and 842..909 are black (AdjustY and SplitIQ leave
    them 0 in cbuf, u16_to_ire(0) = -100 IRE, clamped to 0); DoYNR's cross-line history
    reaches x 40..51 only: a different previous frame changes nothing else."""
    fr = frames_3d(seed=21, n=3)
    w = Comb2D(wide=True).process(fr)
    n = Comb2D().process(fr)
    assert w.shape == (3, 480, 910, 3)
    assert np.array_equal(w[:, :, 78:822], n)
    assert (w[:, :, 0:2] == 0).all() and (w[:, :, 842:] == 0).all()
    # the history: the same frame after two different predecessors with the same burst
    # levels (px 1: the global aburstlev chain stays the same)
    # and a bright tail on its line 524; a wide Y-NR clip (-n 100) so the FIR's output shows
    p1 = fr[0].copy()
    p1[524, 820:840] = 60000
    a = Comb2D(wide=True, nr_y=100.0).process(np.stack([fr[0], fr[2]]))[1]
    b = Comb2D(wide=True, nr_y=100.0).process(np.stack([p1, fr[2]]))[1]
    rows, cols = np.nonzero((a != b).any(axis=2))
    assert cols.size and set(rows) == {0} and cols.min() >= 40 and cols.max() <= 51


@pytest.mark.gpu
def test_gpu_comb_wide_history_across_calls(gpu_ctx_ntsc):
    """-W on the GPU in calls of 2 and 3 frames equals one oracle process over all 5 (+-1
    LSB): DoYNR's history at x 40..51 enters from the previous frame, across the call
    boundary through the context; 3D too."""
    ctx, _ = gpu_ctx_ntsc
    fr = frames_3d(seed=23, n=5)
    fr[1, 524, 820:840] = 60000              # a bright tail the next frame's first row sees (x 40..51)
    fr[2, 524, 820:840] = 60000
    ctx.comb_set_opts(wide=True, nr_y=100.0)
    try:
        ctx.comb_reset()
        g = np.concatenate([ctx.comb_ntsc(fr[:2]), ctx.comb_ntsc(fr[2:])])
        o = Comb2D(wide=True, nr_y=100.0).process(fr)
        assert g.shape == o.shape == (5, 480, 910, 3)
        assert np.abs(g.astype(np.int64) - o.astype(np.int64)).max() <= 1
        ctx.comb_reset()
        g3 = np.concatenate([ctx.comb_ntsc3d(fr[:3]), ctx.comb_ntsc3d(fr[3:])])
        o3 = Comb3D(wide=True, nr_y=100.0).process(fr)
        assert g3.shape == o3.shape
        assert np.abs(g3.astype(np.int64) - o3.astype(np.int64)).max() <= 1
    finally:
        ctx.comb_set_opts()
        ctx.comb_reset()
