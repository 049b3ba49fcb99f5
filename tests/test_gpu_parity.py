"""HIP path vs oracle parity (runs through libldgpu.so on an MI355X).

Bars (DESIGN.md "Parity"): demod channels within 1e-9 relative (FP64; FFT
round-off differs from pocketfft); peak lists, vsyncs, nextfieldoffset,
VBI and all per-field metadata exactly equal; line locations within 1e-6
samples; .tbc samples within +-1 LSB; .pcm samples within +-1.
"""
import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope='module')
def cav_capture():
    import sys
    sys.path.insert(0, os.path.join(HERE, 'golden'))
    import make_golden
    return make_golden, make_golden.build_capture('ntsc_cav_u8_0p2s')


READS = [(0, 1), (385743, 1), (1052829, 0.9999)]


@pytest.fixture(scope='module')
def decoded(cav_capture, gpu_ctx_ntsc):
    _, data = cav_capture
    ctx, rf = gpu_ctx_ntsc
    buf = np.frombuffer(data, np.uint8)
    ctx.set_capture(buf, buf.size, 0, 0)
    infos = ctx.decode_reads([r[0] for r in READS], [r[1] for r in READS])
    from oracle.capture import FMT_U8, Capture
    from oracle.demod import RFDemod
    from oracle.field import FieldNTSC
    orf = RFDemod(system='NTSC')
    cap = Capture(data, FMT_U8)
    ref = []
    for s, m in READS:
        raw = orf.demod(cap, s, 1000000, m)
        ref.append((raw, FieldNTSC(orf, raw, 0, audio_offset=0)))
    return ctx, infos, ref


def test_demod_channels(decoded):
    ctx, infos, ref = decoded
    for slot, (raw, _) in enumerate(ref):
        for ci, ch in enumerate(['demod', 'demod_05', 'demod_sync', 'demod_burst']):
            o = raw[0][ch]
            g = ctx.debug(slot, ci, np.float64, o.size)
            assert g.size == o.size
            scale = max(np.abs(o).max(), 1.0)
            assert np.abs(g - o).max() / scale < 1e-9, ch
        for ci, ch in enumerate(['audio_left', 'audio_right']):
            o = raw[1][ch]
            g = ctx.debug(slot, 10 + ci, np.float64, o.size)
            assert np.abs(g - o).max() < 1e-3, ch


MTF_LEVELS = [0.88, 0.5, 0.0]


@pytest.mark.parametrize('system', ['NTSC', 'PAL'])
def test_rf_table_mtf_levels(system, gpu_ctx_ntsc, gpu_ctx_pal):
    """The demod's RF filter at MTF levels away from 1 (lddecode_core.py:290-293): the
    ldg_k_rf_table path exp(m log|MTF|) cis(m arg MTF) against numpy's complex power
    RFVideo * MTF**m of the oracle's filter set, and RFVideo alone at m = 0 (demodblock
    skips the product there)."""
    from oracle.demod import RFDemod
    ctx, _ = gpu_ctx_ntsc if system == 'NTSC' else gpu_ctx_pal
    F = RFDemod(system=system).Filters
    for m in MTF_LEVELS + [1.0]:
        got = ctx.rf_table(m)
        ref = F['RFVideo'] * (F['MTF'] ** m) if m != 0 else F['RFVideo']
        scale = np.abs(ref).max()
        assert np.abs(got - ref).max() / scale < 1e-14, m
    assert np.array_equal(ctx.rf_table(0.0), F['RFVideo'])


@pytest.mark.parametrize('mtf', MTF_LEVELS)
def test_demod_channels_at_mtf(mtf, cav_capture, gpu_ctx_ntsc):
    """One field read demodulated at MTF 0.88, 0.5 and 0 (the m = 0 skip): channels within
    1e-9 relative of the oracle's demod at the same level, peaks exact."""
    _, data = cav_capture
    ctx, rf = gpu_ctx_ntsc
    buf = np.frombuffer(data, np.uint8)
    ctx.set_capture(buf, buf.size, 0, 0)
    infos = ctx.decode_reads([1052829], [mtf], slots=[7])     # slot 7: the module's fixtures use 0..3
    from oracle.capture import FMT_U8, Capture
    from oracle.demod import RFDemod
    from oracle.field import FieldNTSC
    orf = RFDemod(system='NTSC')
    raw = orf.demod(Capture(data, FMT_U8), 1052829, 1000000, mtf)
    f = FieldNTSC(orf, raw, 0, audio_offset=0)
    for ci, ch in enumerate(['demod', 'demod_05', 'demod_sync', 'demod_burst']):
        o = raw[0][ch]
        g = ctx.debug(7, ci, np.float64, o.size)
        assert g.size == o.size
        assert np.abs(g - o).max() / max(np.abs(o).max(), 1.0) < 1e-9, (mtf, ch)
    assert infos[0].npeaks == len(f.peaklist)
    assert np.array_equal(ctx.debug(7, 41, np.int32, infos[0].npeaks), np.asarray(f.peaklist))
    assert infos[0].nextfieldoffset == f.nextfieldoffset


def test_field_records(decoded):
    ctx, infos, ref = decoded
    for slot, (raw, f) in enumerate(ref):
        inf = infos[slot]
        assert inf.npeaks == len(f.peaklist)
        assert np.array_equal(ctx.debug(slot, 41, np.int32, inf.npeaks), np.array(f.peaklist))
        assert inf.nvsync == len(f.vsyncs)
        assert inf.nextfieldoffset == f.nextfieldoffset
        assert (inf.status == 0) == bool(f.valid)
        if not f.valid:
            continue
        assert inf.istop == int(f.istop) and inf.linecount == f.linecount
        for q in range(inf.nvsync):
            assert list(inf.vsync[q]) == [int(x) for x in f.vsyncs[q]]
        assert inf.vbi_framenr == f.vbi['framenr']
        assert inf.vbi_status == f.vbi['status']
        nl = f.linecount + 4
        for what, arr in ((20, f.linelocs1), (21, f.linelocs2), (22, f.linelocs3), (23, f.linelocs4),
                          (24, f.linelocs)):
            g = ctx.debug(slot, what, np.float64, nl)
            assert np.abs(g - np.asarray(arr, dtype=np.float64)).max() < 1e-6
        assert np.array_equal(ctx.debug(slot, 30, np.float32, nl), f.burstlevel)


def test_tbc_lines_and_audio(decoded):
    ctx, infos, ref = decoded
    for slot, (raw, f) in enumerate(ref):
        if not f.valid:
            continue
        pic = ctx.debug(slot, 40, np.uint16, f.linecount * 910)
        d = np.abs(pic.astype(np.int64) - f.dspicture.astype(np.int64))
        assert d.max() <= 1
        pcm, counts, nxt = ctx.field_audio([slot], [0.0])
        assert counts[0] * 2 == f.dsaudio.size
        assert np.abs(pcm[0, :2 * counts[0]].astype(np.int64) - f.dsaudio.astype(np.int64)).max() <= 1
        assert nxt[0] == f.audio_next_offset


PAL_READS = [(0, 1), (508767, 1), (1311073, 1), (2109792, 1)]   # the PAL golden's reads (the last one sample off)


@pytest.fixture(scope='module')
def decoded_pal(gpu_ctx_pal):
    import sys
    sys.path.insert(0, os.path.join(HERE, 'golden'))
    import make_golden
    data = make_golden.build_capture('pal_clv_u8_0p2s')
    ctx, rf = gpu_ctx_pal
    buf = np.frombuffer(data, np.uint8)
    ctx.set_capture(buf, buf.size, 0, 0)
    infos = ctx.decode_reads([r[0] for r in PAL_READS], [r[1] for r in PAL_READS])
    from oracle.capture import FMT_U8, Capture
    from oracle.demod import RFDemod
    from oracle.field import FieldPAL
    orf = RFDemod(system='PAL')
    cap = Capture(data, FMT_U8)
    ref = []
    for s, m in PAL_READS:
        raw = orf.demod(cap, s, 1000000, m)
        ref.append((raw, FieldPAL(orf, raw, 0, audio_offset=0)))
    return ctx, infos, ref


def test_pal_demod_channels(decoded_pal):
    """PAL demod channels incl. demod_pilot (lddecode_core.py:288-316) within 1e-9 relative."""
    ctx, infos, ref = decoded_pal
    for slot, (raw, _) in enumerate(ref):
        for ci, ch in enumerate(['demod', 'demod_05', 'demod_sync', 'demod_burst', 'demod_pilot']):
            o = raw[0][ch]
            g = ctx.debug(slot, ci, np.float64, o.size)
            assert g.size == o.size
            scale = max(np.abs(o).max(), 1.0)
            assert np.abs(g - o).max() / scale < 1e-9, ch
        for ci, ch in enumerate(['audio_left', 'audio_right']):
            o = raw[1][ch]
            g = ctx.debug(slot, 10 + ci, np.float64, o.size)
            assert np.abs(g - o).max() < 1e-3, ch


def test_pal_field_records_and_pilot_refine(decoded_pal):
    """FieldPAL: peaks, vsyncs, VBI exact; linelocs1/2 and the pilot-refined line locations
    (refine_linelocs_pilot, lddecode_core.py:962-1021) within 1e-6 samples; the PAL
    dspicture (lineoffset 3, PAL IRE scaling, :1023-1035) within +-1 LSB; audio within +-1."""
    ctx, infos, ref = decoded_pal
    nvalid = 0
    for slot, (raw, f) in enumerate(ref):
        inf = infos[slot]
        assert inf.npeaks == len(f.peaklist)
        assert np.array_equal(ctx.debug(slot, 41, np.int32, inf.npeaks), np.array(f.peaklist))
        assert inf.nvsync == len(f.vsyncs)
        assert inf.nextfieldoffset == f.nextfieldoffset
        assert (inf.status == 0) == bool(f.valid)
        if not f.valid:
            continue
        nvalid += 1
        assert inf.istop == int(f.istop) and inf.linecount == f.linecount
        for q in range(inf.nvsync):
            assert list(inf.vsync[q]) == [int(x) for x in f.vsyncs[q]]
        assert inf.vbi_framenr == (f.vbi['framenr'] if f.vbi['framenr'] is not None else -2 ** 31)
        nl = f.linecount + 4
        for what, arr in ((20, f.linelocs1), (21, f.linelocs2), (24, f.linelocs)):
            g = ctx.debug(slot, what, np.float64, nl)
            assert np.abs(g - np.asarray(arr, dtype=np.float64)).max() < 1e-6, what
        # the pilot refine moved the lines (the comparison above is not vacuous)
        assert np.abs(np.asarray(f.linelocs) - np.asarray(f.linelocs2)).max() > 1e-3
        pic = ctx.debug(slot, 40, np.uint16, f.linecount * 1135)
        assert pic.size == f.dspicture.size
        assert np.abs(pic.astype(np.int64) - f.dspicture.astype(np.int64)).max() <= 1
        pcm, counts, nxt = ctx.field_audio([slot], [0.0])
        assert counts[0] * 2 == f.dsaudio.size
        assert np.abs(pcm[0, :2 * counts[0]].astype(np.int64) - f.dsaudio.astype(np.int64)).max() <= 1
        assert nxt[0] == f.audio_next_offset
    assert nvalid >= 3


CASES = ['ntsc_cav_u8_0p2s', 'ntsc_clv_u8_0p2s', 'ntsc_cav_r30_0p15s', 'ntsc_cav_lds_0p15s', 'pal_clv_u8_0p2s',
         'ntsc_cav_s16_0p15s', 'ntsc_cav_u8_mid_0p2s',
         # the MTF chain: a first frame re-read at MTF 0.88 (NTSC and PAL), the clamp to 0
         'ntsc_cav_u8_mtf_0p3s', 'ntsc_cav_u8_mtf0_0p3s', 'pal_cav_u8_mtf_0p3s',
         # PAL through the 10-bit loaders
         'pal_clv_lds_0p15s', 'pal_cav_r30_0p15s']
MTF_CASES = ['ntsc_cav_u8_mtf_0p3s', 'ntsc_cav_u8_mtf0_0p3s', 'pal_cav_u8_mtf_0p3s']
_ORACLE = {}


def oracle_decode(case):
    """(capture bytes, golden fixture, oracle frames, pcm, meta) of a golden case, decoded once per
    session by the oracle; the oracle's output is pinned to the fixture's SHA-256 first."""
    if case not in _ORACLE:
        import sys
        sys.path.insert(0, os.path.join(HERE, 'golden'))
        import make_golden
        from oracle.capture import FMT_BY_EXT
        from oracle.framer import decode_capture
        with open(os.path.join(HERE, 'golden', case + '.json')) as fh:
            gold = json.load(fh)
        c = make_golden.CASES[case]
        data = make_golden.build_capture(case)
        assert hashlib.sha256(data).hexdigest() == gold['capture_sha256']
        frames, pcm, meta = decode_capture(data, FMT_BY_EXT[c['fmt']], system=c['system'])
        assert len(frames) == len(gold['frames'])
        for f, a, g in zip(frames, pcm, gold['frames']):
            assert hashlib.sha256(f.tobytes()).hexdigest() == g['tbc_sha256']
            assert hashlib.sha256(a.tobytes()).hexdigest() == g['pcm_sha256']
        _ORACLE[case] = (data, gold, frames, pcm, meta)
    return _ORACLE[case]


@pytest.mark.parametrize('case', CASES)
@pytest.mark.parametrize("batch", [3, 16])
def test_end_to_end_vs_golden(case, batch):
    """Full decode (speculative batches) of every golden case -- NTSC CAV / CLV, PAL CLV, u8 /
    s16 / .r30 / .lds, a capture starting mid-field -- against the oracle's decode of the same
    capture (itself pinned to the committed fixture): metadata exact, .tbc within +-1 LSB,
    .pcm bit-exact (the fixture's SHA-256)."""
    from ldgpu.decoder import GPUDecoder
    from ldgpu.formats import NAME_TO_FMT
    data, gold, frames, pcm, meta = oracle_decode(case)
    c = gold['settings']
    dec = GPUDecoder(system=c['system'], batch=batch)
    dec.set_capture(data, NAME_TO_FMT[c['fmt']])
    got = []
    dec.decode(sink=lambda fr, au, meta: got.append((fr.copy(), au.copy(), meta)))
    assert len(got) == len(gold['frames']) >= 2
    exact = 0
    for (fr, au, m), f, a, g in zip(got, frames, pcm, gold['frames']):
        assert m == g['meta']                        # metadata / VBI / read chain: exact
        assert fr.size == f.size
        d = np.abs(fr.astype(np.int64) - f.astype(np.int64))
        assert d.max() <= 1                          # .tbc: +-1 LSB (north_star)
        exact += int((d == 0).all())
        assert au.size == g['pcm_len']
        assert hashlib.sha256(au.tobytes()).hexdigest() == g['pcm_sha256']   # .pcm bit-exact
    print('%s batch=%d: %d/%d frames bit-identical' % (case, batch, exact, len(got)))


@pytest.mark.parametrize('case', ['ntsc_clv_u8_0p2s', 'pal_clv_u8_0p2s', 'ntsc_cav_u8_mid_0p2s'])
def test_video_cut_gives_the_same_decode(case, monkeypatch):
    """The demod skips the video / burst / pilot channels of a read's blocks past its video
    cut (ldg_set_video_cut); a field kernel reaching past it returns FS_VCUT and the read is
    decoded again in full.  No cut, the default cut and a cut inside every field (every
    read redone) must give the same frames, audio and metadata bit for bit."""
    from ldgpu.decoder import GPUDecoder
    from ldgpu.formats import NAME_TO_FMT
    data, gold, frames, pcm, meta = oracle_decode(case)
    c = gold['settings']
    outs, redos = [], []
    for cut in ('0', None, '200000'):
        if cut is None:
            monkeypatch.delenv('LDG_VCUT', raising=False)
        else:
            monkeypatch.setenv('LDG_VCUT', cut)
        dec = GPUDecoder(system=c['system'], batch=8)
        dec.set_capture(data, NAME_TO_FMT[c['fmt']])
        got = []
        dec.decode(sink=lambda fr, au, m: got.append((fr.copy(), au.copy(), m)))
        outs.append(got)
        redos.append(dec.stats.get('vcut_redo', 0))
        dec.ctx.close()
    assert redos[0] == 0 and redos[2] > 0, redos
    for other in outs[1:]:
        assert len(other) == len(outs[0])
        for (f0, a0, m0), (f1, a1, m1) in zip(outs[0], other):
            assert m0 == m1
            assert np.array_equal(f0, f1)
            assert np.array_equal(a0, a1)


def test_end_to_end_pixels_vs_oracle(cav_capture):
    """Frame pixels within +-1 LSB and audio within +-1 of a fresh oracle decode."""
    mg, data = cav_capture
    from ldgpu.decoder import GPUDecoder
    from oracle.capture import FMT_U8
    from oracle.framer import decode_capture
    frames, pcm, meta = decode_capture(data, FMT_U8)
    dec = GPUDecoder(system='NTSC', batch=8)
    dec.set_capture(data, 0)
    got = []
    dec.decode(sink=lambda fr, au, m: got.append((fr.copy(), au.copy(), m)))
    assert len(got) == len(frames)
    exact = 0
    for (fr, au, m), f, a, om in zip(got, frames, pcm, meta):
        d = np.abs(fr.astype(np.int64) - f.astype(np.int64))
        assert d.max() <= 1
        exact += int((d == 0).all())
        assert np.abs(au.astype(np.int64) - a.astype(np.int64)).max() <= 1
        assert m == om
    print('bit-exact frames: %d/%d' % (exact, len(frames)))


@pytest.mark.parametrize('case', ['ntsc_cav_s16_0p15s', 'ntsc_cav_u8_mid_0p2s'])
def test_edge_captures_pixels_vs_oracle(case):
    """The s16 loader and a capture starting mid-field (first read's short next-field
    offset, demod's start-1024 quirk at the file start): pixels within +-1 LSB, audio
    within +-1 and metadata exact against a fresh oracle decode."""
    import sys
    sys.path.insert(0, os.path.join(HERE, 'golden'))
    import make_golden
    from ldgpu.decoder import GPUDecoder
    from ldgpu.formats import NAME_TO_FMT
    from oracle.capture import FMT_BY_EXT
    from oracle.framer import decode_capture
    c = make_golden.CASES[case]
    data = make_golden.build_capture(case)
    frames, pcm, meta = decode_capture(data, FMT_BY_EXT[c['fmt']], system=c['system'])
    dec = GPUDecoder(system=c['system'], batch=8)
    dec.set_capture(data, NAME_TO_FMT[c['fmt']])
    got = []
    dec.decode(sink=lambda fr, au, m: got.append((fr.copy(), au.copy(), m)))
    assert len(got) == len(frames) >= 3
    for (fr, au, m), f, a, om in zip(got, frames, pcm, meta):
        assert m == om
        assert np.abs(fr.astype(np.int64) - f.astype(np.int64)).max() <= 1
        assert np.abs(au.astype(np.int64) - a.astype(np.int64)).max() <= 1


def test_gpu_synth_capture_decodes_like_oracle():
    """The GPU-synthesised bench input decodes identically (metadata exact, +-1 LSB) on both paths."""
    from ldgpu.decoder import GPUDecoder
    from oracle.capture import FMT_U8
    from oracle.framer import decode_capture
    n = int(40e6 * 0.2)
    dec = GPUDecoder(system='NTSC', batch=8)
    dec.ctx.synth(n, fmt=0, first_frame=100, seed=5)
    dec.use_resident_capture(0, n)
    raw = dec.ctx.capture_download(0, n).tobytes()
    got = []
    dec.decode(sink=lambda fr, au, m: got.append((fr.copy(), au.copy(), m)))
    frames, pcm, meta = decode_capture(raw, FMT_U8)
    assert len(got) == len(frames) >= 3
    assert [m['vbi']['framenr'] for _, _, m in got] == list(range(101, 101 + len(got)))
    for (fr, au, m), f, a, om in zip(got, frames, pcm, meta):
        assert m == om
        assert np.abs(fr.astype(np.int64) - f.astype(np.int64)).max() <= 1
        assert np.abs(au.astype(np.int64) - a.astype(np.int64)).max() <= 1


@pytest.mark.parametrize('fmt', [2, 3])
def test_gpu_synth_10bit_formats(fmt):
    """.r30 / .lds synthesised on the GPU unpack on the GPU and decode consecutive CAV frames."""
    from ldgpu.decoder import GPUDecoder
    n = int(40e6 * 0.15)
    dec = GPUDecoder(system='NTSC', batch=8)
    dec.ctx.synth(n, fmt=fmt, first_frame=7, seed=11)
    dec.use_resident_capture(fmt, n)
    got = []
    dec.decode(sink=lambda fr, au, m: got.append(m))
    assert len(got) >= 2
    assert [m['vbi']['framenr'] for m in got] == list(range(8, 8 + len(got)))


@pytest.mark.parametrize('clv', [False, True])
def test_gpu_long_capture_decodes_every_frame(clv):
    """A 5-minute capture (12 GB u8, past the ~3000-frame point where the planner once
    pinned the whole read cache) decodes every frame the reference's EOF guard allows,
    with consecutive picture numbers / CLV timecodes, in benchmark mode (frames in HBM)."""
    from ldgpu.decoder import GPUDecoder
    n = int(40e6 * 300)
    dec = GPUDecoder(system='NTSC', batch=128)
    dec.ctx.synth(n, fmt=0, first_frame=1, clv=clv, seed=21)
    dec.use_resident_capture(0, n)
    nfr = dec.decode(sink=None)
    bpf = dec.rf.samples_per_frame * 5 // 4            # lddecode.py:42 (10-bit packing assumed)
    assert nfr == n // bpf - 1 or nfr == n // bpf, (nfr, n // bpf)
    nrs = dec.frame_numbers
    assert len(nrs) == nfr and all(b == a + 1 for a, b in zip(nrs, nrs[1:]))
    assert dec.stats['reads'] < 1.02 * dec.stats['reads_used']
