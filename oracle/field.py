"""ORACLE (test infrastructure only): field decode / time-base correction.

Restates lddecode_core.py:431-1191 (downscale_audio, Field, FieldPAL,
FieldNTSC) and lddutils.py:83-97 (scale) / :265-303 (calczc).

numpy-1.x semantics pinned:
  * ``burstlevel`` is stored float32 (lddecode_core.py:1060) but every
    arithmetic use of an element (``/ hz_ire_scale``, ``* .6``, ``327.67*...``)
    is done in float64, as numpy-1 scalar promotion did;
  * ``np.int``/``np.float`` -> ``int``/``float``.
Exceptions the reference caught (its bare ``except:`` blocks) mark the
field invalid; ones it did not catch raise ``ReferenceCrash``.
"""
import copy

import numpy as np
from scipy import interpolate

from .demod import ReferenceCrash, inrange


def calczc(data, start_offset, target, edge='both', reverse=False, count=10):
    """lddutils.py:265-303: fractional index of the first threshold crossing."""
    s = int(start_offset)
    n = int(count + 1)
    window = data[s:s + n]
    if edge == 'both':
        edge = 'rising' if data[s] < target else 'falling'
    hits = np.where(window >= target)[0] if edge == 'rising' else np.where(window <= target)[0]
    if len(hits) == 0:
        return None
    x = s + hits[-1 if reverse else 0]
    if x == 0:
        return None
    a = data[x - 1] - target
    b = data[x] - target
    return x - 1 + (-a / (-a + b))


def scale(buf, begin, end, tgtlen):
    """lddutils.py:83-97: not-a-knot cubic spline resample of one line."""
    ib, ie = int(begin), int(end)
    span = end - begin
    dist = ie - ib
    xs = np.linspace(0, dist, num=dist + 1)
    spl = interpolate.splrep(xs, buf[ib:ib + dist + 1])
    xo = np.linspace(begin - ib, span + (begin - ib), tgtlen + 1)
    return interpolate.splev(xo, spl)[:-1]


def downscale_audio(audio, lineinfo, rf, linecount, timeoffset=0, freq=48000.0, scale_=64):
    """lddecode_core.py:431-484: 48 kHz stereo from the 625 kHz field audio."""
    sp = rf.SysParams
    frametime = (sp['line_period'] * linecount) / 1000000
    gap = 1 / freq
    ticks = np.arange(timeoffset, frametime + gap, gap, dtype=np.double)
    locs = np.zeros(len(ticks), dtype=float)
    swow = np.zeros(len(ticks), dtype=float)
    for i, t in enumerate(ticks):
        ln = ((t * 1000000) / sp['line_period']) + 1
        cur = lineinfo[int(ln)]
        try:
            nxt = lineinfo[int(ln) + 1]
        except IndexError:
            nxt = cur + rf.linelen
        pos = cur
        pos += (nxt - cur) * (ln - np.floor(ln))
        swow[i] = ((nxt - cur) / rf.linelen)
        locs[i] = pos / scale_
    out = np.zeros((2 * (len(ticks) - 1)), dtype=np.int32)
    out16 = np.zeros((2 * (len(ticks) - 1)), dtype=np.int16)
    for i in range(len(ticks) - 1):
        left = audio['audio_left'][int(locs[i])]
        right = audio['audio_right'][int(locs[i])]
        left *= swow[i]
        right *= swow[i]
        left -= sp['audio_lfreq']
        right -= sp['audio_rfreq']
        out[(i * 2) + 0] = int(np.round(left * 32767 / 150000))
        out[(i * 2) + 1] = int(np.round(right * 32767 / 150000))
    np.clip(out, -32766, 32766, out=out16)
    return out16, ticks[-1] - frametime


class Field:
    """lddecode_core.py:489-957 (system-independent sync/line analysis)."""

    def usectoinpx(self, x):
        return x * self.rf.freq

    def inpxtousec(self, x):
        return x / self.rf.freq

    # ---- sync pulses: lddecode_core.py:497-636 ------------------------------
    def get_syncpeaks(self):
        ds = self.data[0]['demod_sync']
        peaks = []
        i = self.start
        stop = len(ds) - (self.inlinelen * 2)
        while i < stop:
            loc = np.argmax(ds[i:i + (self.inlinelen // 2)])
            if ds[i + loc] > .2:
                peaks.append(i + loc)
                i += loc + int(self.rf.linelen * .4)
            else:
                i += self.rf.linelen // 2
        return peaks

    def get_hsync_median(self):
        ds = self.data[0]['demod_sync']
        levels = [ds[p] for p in self.peaklist if inrange(ds[p], 0.6, 0.8)]
        self.med_hsync = np.median(levels)
        self.std_hsync = np.std(levels)
        self.hsync_tolerance = max(np.std(levels) * 2, .01)
        return self.med_hsync, self.hsync_tolerance

    def is_regular_hsync(self, n):
        if n >= len(self.peaklist):
            return False
        ds = self.data[0]['demod_sync']
        if self.peaklist[n] > len(ds):
            return False
        lvl = ds[self.peaklist[n]]
        return inrange(lvl, self.med_hsync - self.hsync_tolerance, self.med_hsync + self.hsync_tolerance)

    def determine_field(self, n):
        if n < 11:
            return None
        vote = 0
        line0 = gap1 = None
        for i in range(n - 1, n - 20, -1):
            if self.is_regular_hsync(i) and line0 is None:
                line0 = i
                gap1 = self.peaklist[line0 + 1] - self.peaklist[line0]
                break
        if gap1 is not None and gap1 > (self.inlinelen * .75):
            vote -= 1
        linee = gap2 = None
        for i in range(n, n + 20, 1):
            if self.is_regular_hsync(i) and linee is None:
                linee = i
                gap2 = self.peaklist[linee] - self.peaklist[linee - 1]
                break
        if gap2 is not None and gap2 > (self.inlinelen * .75):
            vote += 1 if self.rf.system == 'NTSC' else -1
        if self.rf.system == 'PAL':
            vote += 1
        return line0, vote

    def determine_vsyncs(self):
        ds = self.data[0]['demod_sync']
        found = []
        if len(self.peaklist) < 200:
            return []
        med, tol = self.get_hsync_median()
        prev = 1.0
        for i, p in enumerate(self.peaklist):
            lvl = ds[p]
            if lvl > .9 and prev < med - (tol * 2):
                r = self.determine_field(i)
                if r is None:
                    raise ReferenceCrash('vsync within the first 11 peaks (determine_field -> None)')
                line0, vote = r
                if line0 is not None:
                    found.append((i, line0, vote))
            prev = lvl
        if len(found) < 2:
            return found
        va = np.array(found)
        for i in range(0, len(found)):
            if va[i][2] == 0:
                va[i][1] = -1
                print("vsync vote needed", i)
                if (i < len(found) - 1) and found[i + 1][2] != 0:
                    va[i][2] = -va[i + 1][2]
                elif (i >= 1) and found[i - 1][2] != 0:
                    va[i][2] = -va[i - 1][2]
            if va[i][1] <= 0:
                va[i][1] = va[i][0] - (6 if self.rf.system == 'PAL' else 7)
            va[i][2] = va[i][2] < 0
        return va

    # ---- line locations: lddecode_core.py:638-787 ----------------------------
    def compute_linelocs(self):
        plist = self.peaklist
        locs = {}
        lens = [self.inlinelen]
        prev_idx = prev_num = None
        for i in range(0, self.vsyncs[1][1]):
            med_len = np.median(lens[-25:])
            if self.is_regular_hsync(i):
                if prev_idx is not None:
                    gap = plist[i] - plist[prev_idx]
                    if inrange(gap / self.inlinelen, .98, 1.02):
                        lens.append(gap)
                        num = prev_num + 1
                    else:
                        num = prev_num + int(np.round((plist[i] - plist[prev_idx]) / med_len))
                else:
                    num = int(np.round((plist[i] - plist[self.vsyncs[0][1]]) / med_len))
                locs[num] = plist[i]
                prev_idx, prev_num = i, num
        filled = copy.deepcopy(locs)
        for l in range(1, self.linecount + 5):
            if l in locs:
                continue
            pv = nv = None
            for i in range(l, -10, -1):
                if i in locs:
                    pv = i
                    break
            for i in range(l, self.linecount + 1):
                if i in locs:
                    nv = i
                    break
            if pv is None:
                filled[l] = locs[nv] - (self.inlinelen * (nv - l))
            elif nv is not None:
                step = (locs[nv] - locs[pv]) / (nv - pv)
                filled[l] = locs[pv] + (step * (l - pv))
            else:
                step = locs[pv] - filled[pv - 1]
                filled[l] = locs[pv] + (step * (l - pv))
        out = [filled[l] for l in range(1, self.linecount + 5)]
        bad = [l not in locs for l in range(1, self.linecount + 5)]
        for i in range(0, 10):
            bad[i] = False
        return out, bad

    def refine_linelocs_hsync(self):
        d05 = self.data[0]['demod_05']
        fr = self.rf.freq
        ll = self.linelocs1.copy()
        for i in range(len(self.linelocs1)):
            if i < 9:
                ll[i] -= 200
            ll1 = ll[i]
            zc = calczc(d05, ll[i], self.rf.iretohz(-20), reverse=False, count=400)
            if zc is not None and not self.linebad[i]:
                ll[i] = zc
                if i >= 10:
                    w1 = d05[int(ll1 - (fr * 2)):int(ll1 + (fr * 2))]
                    wh = d05[int(zc - (fr * 1)):int(zc + (fr * 3))]
                    wb = d05[int(zc + (fr * 1)):int(zc + (fr * 3))]
                    hz = self.rf.iretohz
                    if ((np.min(wh) < hz(-60) or np.max(wh) > hz(20)) or
                            (np.min(w1) < hz(-60) or np.max(w1) > hz(100)) or
                            (np.min(wb) < hz(-10) or np.max(wb) > hz(10))):
                        self.linebad[i] = True
                    else:
                        low = np.mean(wh[0:20])
                        high = np.mean(wh[100:120])
                        zc2 = calczc(wh, 0, (low + high) / 2, reverse=False, count=len(wh))
                        zc2 += (int(zc) - (fr * 1))        # TypeError on None -> caught upstream
                        if np.abs(zc2 - zc) < (fr / 4):
                            ll[i] = zc2
                        else:
                            self.linebad[i] = True
            else:
                self.linebad[i] = True
            if i < 10:
                ll[i] += self.usectoinpx(4.72)
            if i > 10 and self.linebad[i]:
                gap = ll[i - 1] - ll[i - 2]
                ll[i] = ll[i - 1] + gap
        lo, hi = self.rf.linelen - (fr * .2), self.rf.linelen + (fr * .2)
        for i in range(9, -1, -1):
            gap = ll[i + 1] - ll[i]
            if not inrange(gap, lo, hi):
                gap = self.rf.linelen
            ll[i] = ll[i + 1] - gap
        for i in range(len(ll) - 10, len(ll)):
            gap = ll[i] - ll[i - 1]
            if not inrange(gap, lo, hi):
                gap = self.rf.linelen
            ll[i] = ll[i - 1] + gap
        return ll

    # ---- resample: lddecode_core.py:789-812 ----------------------------------
    def downscale(self, lineoffset=1, lineinfo=None, outwidth=None, wow=True, channel='demod', audio=False):
        if lineinfo is None:
            lineinfo = self.linelocs
        if outwidth is None:
            outwidth = self.outlinelen
        out = np.zeros((self.linecount * outwidth), dtype=np.double)
        for l in range(lineoffset, self.linecount + lineoffset):
            line = scale(self.data[0][channel], lineinfo[l], lineinfo[l + 1], outwidth)
            if wow:
                line *= (lineinfo[l + 1] - lineinfo[l]) / self.inlinelen
            out[(l - lineoffset) * outwidth:(l + 1 - lineoffset) * outwidth] = line
        if audio and self.rf.decode_analog_audio:
            self.dsaudio, self.audio_next_offset = downscale_audio(
                self.data[1], lineinfo, self.rf, self.linecount, self.audio_next_offset)
        return out, self.dsaudio

    # ---- Philips VBI: lddecode_core.py:814-884 --------------------------------
    def decodephillipscode(self, linenum):
        start = self.linelocs[linenum]
        data = self.data[0]['demod']
        thr = self.rf.iretohz(50)
        cur = calczc(data, int(start + self.usectoinpx(2)), thr, count=int(self.usectoinpx(12)))
        zc = []
        while cur is not None:
            zc.append((cur, data[int(cur - self.usectoinpx(0.5))] < thr))
            cur = calczc(data, cur + self.usectoinpx(1.9), thr, count=int(self.usectoinpx(0.2)))
        gaps = self.inpxtousec(np.diff([z[0] for z in zc]))
        if len(zc) == 24 and np.min(gaps) > 1.85 and np.max(gaps) < 2.15:
            bits = [z[1] for z in zc]
            # numpy-1 scalar promotion: nibbles behave as plain ints in the later <<, * and +
            return [int((np.packbits(bits[b:b + 4]) >> 4)[0]) for b in range(0, 24, 4)]
        return None

    def processphilipscode(self):
        v = {'minutes': None, 'seconds': None, 'clvframe': None, 'framenr': None,
             'statuscode': None, 'status': None, 'isclv': False}
        self.vbi = v
        for l in self.rf.SysParams['philips_codelines']:
            lc = self.linecode[l]
            if lc is None:
                continue
            if lc[0] == 15 and lc[2] == 13:
                v['minutes'] = 60 * lc[1] + lc[4] * 10 + lc[5]
                v['isclv'] = True
            elif lc[0] == 15:
                v['framenr'] = (lc[1] & 7) * 10000 + (lc[2] * 1000) + (lc[3] * 100) + (lc[4] * 10) + lc[5]
            else:
                h = (lc[0] << 20) | (lc[1] << 16) | (lc[2] << 12) | (lc[3] << 8) | (lc[4] << 4) | lc[5]
                if lc[2] == 0xE:
                    v['seconds'] = (lc[1] - 10) * 10 + lc[3]
                    v['clvframe'] = lc[4] * 10 + lc[5]
                    v['isclv'] = True
                if (h >> 12) in (0x8dc, 0x8ba):
                    v['status'] = h
                if h == 0x87ffff:
                    v['isclv'] = True

    # ---- constructor: lddecode_core.py:889-957 ---------------------------------
    def __init__(self, rf, rawdecode, start, audio_offset=0, keepraw=True):
        if rawdecode is None:
            return
        self.data = rawdecode
        self.rf = rf
        self.start = start
        self.inlinelen = rf.linelen
        self.outlinelen = rf.SysParams['outlinelen']
        self.valid = False
        self.peaklist = self.get_syncpeaks()
        self.vsyncs = self.determine_vsyncs()
        self.dspicture = None
        self.dsaudio = None
        self.audio_next_offset = audio_offset
        self.skip_reason = None
        if len(self.vsyncs) == 0:
            self.nextfieldoffset = start + (rf.linelen * 200)
            self.skip_reason = 'no_vsync'
            return
        elif len(self.vsyncs) == 1 or len(self.peaklist) < self.vsyncs[1][1] + 4:
            jumpto = self.peaklist[self.vsyncs[0][1] - 10]
            self.nextfieldoffset = start + jumpto
            self.skip_reason = 'short'
            if jumpto == 0:
                print("no/corrupt VSYNC found, jumping forward")
                self.nextfieldoffset = start + (rf.linelen * 240)
            return
        self.nextfieldoffset = self.peaklist[self.vsyncs[1][1] - 10]
        self.istop = self.vsyncs[0][2]
        self.linecount = rf.SysParams['frame_lines'] // 2
        if self.istop:
            self.linecount += 1
        try:
            self.linelocs1, self.linebad = self.compute_linelocs()
            self.linelocs2 = self.refine_linelocs_hsync()
        except Exception:
            print('unable to decode frame')
            self.valid = False
            self.skip_reason = 'linelocs'
            return
        self.linelocs = self.linelocs2
        self.isclv = False
        self.linecode = {}
        self.framenr = None
        for l in rf.SysParams['philips_codelines']:
            self.linecode[l] = self.decodephillipscode(l)
        self.processphilipscode()
        self.valid = True
        self.tbcstart = self.peaklist[self.vsyncs[1][1] - 10]


class FieldPAL(Field):
    """lddecode_core.py:961-1048."""

    def refine_linelocs_pilot(self, linelocs=None):
        ll = (self.linelocs2 if linelocs is None else linelocs).copy()
        demod, d05 = self.data[0]['demod'], self.data[0]['demod_05']
        allofs = []
        ofs = {}
        for l in range(len(ll)):
            a, b = int(ll[l] - self.usectoinpx(4.7)), int(ll[l])
            pilot = demod[a:b].copy()
            pilot -= d05[a:b]
            pilot = np.flip(pilot)
            ofs[l] = []
            adjfreq = self.rf.freq
            if l > 1:
                adjfreq /= (ll[l] - ll[l - 1]) / self.rf.linelen
            i = 0
            while i < len(pilot):
                if inrange(pilot[i], -300000, -100000):
                    zc = calczc(pilot, i, 0)
                    if zc is not None:
                        zcp = zc / (adjfreq / 3.75)
                        ofs[l].append(zcp - np.floor(zcp))
                        i = int(zc + 1)
                i += 1
            if len(ofs) >= 3:          # (sic) tests the dict, lddecode_core.py:1001
                ofs[l] = ofs[l][1:-1]
                if i >= 11:            # (sic) sample index, lddecode_core.py:1003
                    allofs += ofs[l]
            else:
                ofs[l] = []
        med = np.median(allofs)
        tgt = .5 if inrange(med, 0.25, 0.75) else 0
        for l in range(len(ll)):
            if ofs[l] != []:
                ll[l] += (tgt - np.median(ofs[l])) * (self.rf.freq / 3.75) * .25
        return ll

    def downscale(self, final=False, *args, **kwargs):
        out, aud = super().downscale(lineoffset=3, audio=final, *args, **kwargs)
        if final:
            sp = self.rf.SysParams
            red = (out - sp['ire0']) / sp['hz_ire']
            red -= sp['vsync_ire']
            k = np.double(0xd300 - 0x0100) / (100 - sp['vsync_ire'])
            self.dspicture = np.uint16(np.clip((red * k) + 256, 0, 65535) + 0.5)
            return self.dspicture, aud
        return out, aud

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        if not getattr(self, 'valid', False):
            return
        try:
            self.linelocs = self.refine_linelocs_pilot()
            self.downscale(wow=True, final=True)
        except Exception:
            print("ERROR: Unable to decode frame, skipping")
            self.valid = False
            self.skip_reason = 'tbc'


class FieldNTSC(Field):
    """lddecode_core.py:1052-1191."""

    def refine_linelocs_burst(self, linelocs2):
        hz_ire_scale = 1700000 / 140
        sburst, _ = self.downscale(outwidth=self.outlinelen, lineinfo=linelocs2,
                                   channel='demod_burst', lineoffset=0)
        ll3 = linelocs2.copy()
        level = np.zeros_like(ll3, dtype=np.float32)
        pavg = np.zeros([len(linelocs2), 2], dtype=np.double)
        W = self.outlinelen
        for l in range(self.linecount):
            ba = sburst[(W * l) + 20:W * (l + 0) + 60].copy()
            ba -= np.mean(ba)
            level[l] = np.max(np.abs(ba))
            lv = float(level[l])                       # numpy-1 promotion
            if ((lv / hz_ire_scale) > 30) or (np.std(ba) / hz_ire_scale) < 3:
                level[l] = 0
                continue
            groups = {False: [], True: []}
            bi = 0
            while bi < len(ba):
                if np.abs(ba[bi]) > float(level[l]) * .6:
                    zc = calczc(ba, bi, 0)
                    if zc is not None:
                        off = zc - ((np.floor(zc / 4) * 4) - 1)
                        if off > 3.5:
                            off -= 4
                        groups[bool(ba[bi] > 0)].append(off)
                        bi = int(zc)
                bi += 1
            if len(groups[False]) < 3 or len(groups[True]) < 3:
                continue
            for v in (False, True):
                groups[v] = np.array(groups[v][1:-1])
            if l % 2:
                pavg[l] = (2 - np.mean(groups[True]), 2 - np.mean(groups[False]))
            else:
                pavg[l] = (2 - np.mean(groups[False]), 2 - np.mean(groups[True]))
        cut = pavg[np.logical_or(pavg[:, 0] != 0, pavg[:, 1] != 0)]
        grp = 0 if np.abs(np.median(cut[:, 0])) < np.abs(np.median(cut[:, 1])) else 1
        adj = pavg[:, grp]
        level[grp::2] = -level[grp::2]
        for l in range(len(ll3)):
            if np.abs(adj[l]) > 2:
                level[l] = 0
                continue
            ll3[l] -= adj[l] * (self.rf.freq / (4 * 315 / 88)) * 1
        for l in range(2, len(ll3) - 1):
            if level[l] == 0:
                ll3[l] = (ll3[l - 1] + ll3[l + 1]) / 2
        return np.array(ll3), level

    def downscale(self, lineoffset=1, final=False, *args, **kwargs):
        out, aud = super().downscale(lineoffset=lineoffset, audio=final, *args, **kwargs)
        if final:
            sp = self.rf.SysParams
            red = (out - sp['ire0']) / sp['hz_ire']
            red -= sp['vsync_ire']
            k = np.double(0xc800 - 0x0400) / (100 - sp['vsync_ire'])
            pic = np.uint16(np.clip((red * k) + 1024, 0, 65535) + 0.5)
            if self.burstlevel is not None:
                W = self.outlinelen
                for i in range(1, self.linecount - 1):
                    hz_ire_scale = 1700000 / 140
                    pic[i * W] = 16384 if self.burstlevel[i] > 0 else 32768
                    clevel = (1 / self.colorlevel) / hz_ire_scale
                    pic[i * W + 1] = np.uint16(327.67 * clevel * abs(float(self.burstlevel[i])))
            self.dspicture = pic
            return pic, aud
        return out, aud

    def apply_offsets(self, linelocs, phaseoffset, picoffset=0):
        return np.array(linelocs) + picoffset + (phaseoffset * (self.rf.freq / (4 * 315 / 88)))

    def __init__(self, *args, **kwargs):
        self.burstlevel = None
        self.colorphase = 90 + 1.5
        self.colorlevel = 1.45
        super().__init__(*args, **kwargs)
        if not getattr(self, 'valid', False):
            print('not valid')
            return
        try:
            self.linelocs3, self.burstlevel = self.refine_linelocs_burst(self.linelocs2)
            self.linelocs4, self.burstlevel = self.refine_linelocs_burst(self.linelocs3)
            shift = self.colorphase * (np.pi / 180)
            self.linelocs = self.apply_offsets(self.linelocs4, shift - 8)
            self.downscale(wow=True, final=True)
        except Exception:
            print("ERROR: Unable to decode frame, skipping")
            self.valid = False
            self.skip_reason = 'tbc'
