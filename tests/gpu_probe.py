"""Stage-by-stage GPU vs oracle probe (diagnostic script, run on the GPU box).

python tests/gpu_probe.py  -> prints max differences per stage for a few reads.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'ld-decode_amd'))

import numpy as np  # noqa: E402

from ldgpu import native  # noqa: E402
from ldgpu.rfparams import RFTables  # noqa: E402
from ldgpu.synth import make_capture  # noqa: E402
from oracle.capture import FMT_U8, Capture  # noqa: E402
from oracle.demod import RFDemod  # noqa: E402
from oracle.field import FieldNTSC  # noqa: E402


def main():
    t = time.time()
    data = make_capture(int(40e6 * 0.12), 'u8')
    print('synth %.1fs' % (time.time() - t), flush=True)
    rf = RFTables('NTSC')
    ctx = native.Context('NTSC', 0, max_reads=4)
    ctx.set_filters(rf.params(), rf.tables)
    buf = np.frombuffer(data, np.uint8)
    ctx.set_capture(buf, buf.size, 0, 0)
    starts = [0, 385743, 1052829]
    mtfs = [1, 1, 0.9999]
    t = time.time()
    infos = ctx.decode_reads(starts, mtfs)
    print('gpu decode_reads %.3fs' % (time.time() - t), flush=True)
    t = time.time()
    infos = ctx.decode_reads(starts, mtfs)
    print('gpu decode_reads (warm) %.3fs' % (time.time() - t), flush=True)
    orf = RFDemod(system='NTSC')
    cap = Capture(data, FMT_U8)
    for slot, (s, m) in enumerate(zip(starts, mtfs)):
        inf = infos[slot]
        print('--- read', s, 'mtf', m, 'status', inf.status, 'npeaks', inf.npeaks, 'nvsync', inf.nvsync,
              'nfo', inf.nextfieldoffset, 'istop', inf.istop, 'lc', inf.linecount, flush=True)
        t = time.time()
        raw = orf.demod(cap, s, 1000000, m)
        print('oracle demod %.1fs' % (time.time() - t), flush=True)
        for ci, ch in enumerate(['demod', 'demod_05', 'demod_sync', 'demod_burst']):
            g = ctx.debug(slot, ci, np.float64, raw[0][ch].size)
            o = raw[0][ch]
            d = np.abs(g - o)
            print('  %-12s n=%d/%d maxdiff=%.3e at %d  rel=%.3e' % (ch, g.size, o.size, d.max(), d.argmax(),
                                                                   d.max() / (np.abs(o).max() + 1e-30)), flush=True)
        for ci, ch in enumerate(['audio_left', 'audio_right']):
            g = ctx.debug(slot, 10 + ci, np.float64, raw[1][ch].size)
            o = raw[1][ch]
            d = np.abs(g - o)
            print('  %-12s n=%d/%d maxdiff=%.3e at %d' % (ch, g.size, o.size, d.max(), d.argmax()), flush=True)
        t = time.time()
        f = FieldNTSC(orf, raw, 0, audio_offset=0)
        print('oracle field %.1fs valid=%s' % (time.time() - t, f.valid), flush=True)
        print('  oracle npeaks', len(f.peaklist), 'nvsync', len(f.vsyncs), 'nfo', f.nextfieldoffset,
              'istop', getattr(f, 'istop', None), flush=True)
        pk = ctx.debug(slot, 41, np.int32, inf.npeaks)
        same = len(f.peaklist) == inf.npeaks and np.array_equal(np.array(f.peaklist), pk)
        print('  peaklist equal:', same, flush=True)
        if not f.valid or inf.status != 0:
            continue
        print('  vbi oracle', f.vbi, flush=True)
        print('  vbi gpu', inf.vbi_framenr, inf.vbi_status, inf.vbi_isclv, flush=True)
        nl = f.linecount + 4
        for what, arr in ((20, f.linelocs1), (21, f.linelocs2), (22, f.linelocs3), (23, f.linelocs4),
                          (24, f.linelocs)):
            g = ctx.debug(slot, what, np.float64, nl)
            d = np.abs(g - np.asarray(arr, dtype=np.float64))
            print('  linelocs%d maxdiff %.3e' % (what - 20, d.max()), flush=True)
        bl = ctx.debug(slot, 30, np.float32, nl)
        print('  burstlevel equal:', np.array_equal(bl, f.burstlevel), 'maxdiff', np.abs(bl - f.burstlevel).max())
        pic = ctx.debug(slot, 40, np.uint16, f.linecount * 910)
        d = np.abs(pic.astype(np.int64) - f.dspicture.astype(np.int64))
        print('  picture maxdiff', d.max(), 'n>1:', int((d > 1).sum()), 'n==1:', int((d == 1).sum()), flush=True)
        pcm, counts, nxt = ctx.field_audio([slot], [0.0])
        ga = pcm[0, :2 * counts[0]]
        da = np.abs(ga.astype(np.int64) - f.dsaudio.astype(np.int64))
        print('  audio n', counts[0], len(f.dsaudio) // 2, 'maxdiff', da.max() if da.size else None,
              'next', nxt[0], f.audio_next_offset, flush=True)


if __name__ == '__main__':
    main()
