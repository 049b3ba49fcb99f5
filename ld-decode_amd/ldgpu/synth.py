"""Synthetic LaserDisc RF generator (NTSC / PAL), for tests and the benchmark.

The reference ships no captures or fixtures, so the build makes
its own, from the pieces the reference source defines:

  * FM mapping ``iretohz`` = ire0 + hz_ire * IRE (lddecode_core.py:282-283,
    constants :35-36 NTSC, :66-67 PAL);
  * video pre-emphasis = the reference's ``Femp`` design "used in test signal
    generation" (lddecode_core.py:190-192): bilinear of
    zpk(-d0e-10, -d1e-10, d1/d0), applied here as the equivalent IIR;
  * analog audio FM carriers at audio_lfreq / audio_rfreq (:43-44, :72-73);
  * Philips 24-bit bi-phase VBI code geometry read by decodephillipscode
    (:814-834: first mid-cell transition after linestart + 2 us, 2 us cells,
    bit = level 0.5 us before the crossing is below 50 IRE) on the lines the
    decoder reads (linelocs indices [16,17,18] NTSC / [19,20,21] PAL);
  * NTSC 525/59.94 and PAL 625/50 line/field timing with equalizing and
    broad (serrated) vertical sync pulses on the half-line grid.

Everything is float64 and chunked, so any length streams in O(chunk) memory.
"""
import numpy as np
import scipy.signal as sps

FS = 40e6

NTSC = dict(system='NTSC', fsc=315e6 / 88, lines=525, ire0=8100000.0, hz_ire=1700000 / 140.0,
            sync_ire=-40.0, setup=7.5, burst_ire=20.0, deemp=(120 * .32, 320 * .32),
            audio_l=(1000000 * 315 / 88 / 227.5) * 146.25, audio_r=(1000000 * 315 / 88 / 227.5) * 178.75,
            code_lines=((16, 17, 18), (279, 280, 281)))
NTSC['line_us'] = 227.5 / (NTSC['fsc'] / 1e6)

PAL = dict(system='PAL', fsc=((1 / 64) * 283.75 + 25 / 1e6) * 1e6, lines=625, ire0=7100000.0, hz_ire=8000.0,
           sync_ire=-.3 * (100 / .7), setup=0.0, burst_ire=21.4, deemp=(100 * .4, 400 * .4),
           audio_l=(1000000 / 64) * 43.75, audio_r=(1000000 / 64) * 68.25,
           code_lines=((18, 19, 20), (331, 332, 333)), line_us=64.0,
           # the PAL disc's 3.75 MHz pilot on the sync tips (240 cycles per line, so
           # line-locked), which FieldPAL.refine_linelocs_pilot times the lines by
           # (lddecode_core.py:962-1021: crossings where demod - demod_05 is in
           # [-300 kHz, -100 kHz]): 25 IRE = 200 kHz peak deviation
           pilot_hz=3.75e6, pilot_ire=25.0)


def emphasis_filter(sysp):
    """Digital pre-emphasis (b, a): the reference's Femp design, lddecode_core.py:190-192."""
    d0, d1 = sysp['deemp']
    tb, ta = sps.zpk2tf([-d0 * 1e-10], [-d1 * 1e-10], d1 / d0)
    return sps.bilinear(tb, ta, 1.0 / (FS / 2))


def cav_code(picnum):
    """CAV picture number code 0xF8xxxx (decoded at lddecode_core.py:855-861)."""
    d = [int(c) for c in '%05d' % picnum]
    return (0xF << 20) | ((8 | (d[0] & 7)) << 16) | (d[1] << 12) | (d[2] << 8) | (d[3] << 4) | d[4]


def clv_minutes_code(minutes):
    """CLV programme time code 0xF?DD?? (lddecode_core.py:850-854)."""
    h, m = divmod(minutes, 60)
    return (0xF << 20) | (h << 16) | (0xDD << 8) | ((m // 10) << 4) | (m % 10)


def clv_seconds_code(seconds, frame):
    """CLV seconds / picture code 0x8?E??? (lddecode_core.py:871-876)."""
    return (0x8 << 20) | ((10 + seconds // 10) << 16) | (0xE << 12) | ((seconds % 10) << 8) | \
        ((frame // 10) << 4) | (frame % 10)


STATUS_CODE = 0x8DC123            # htop 0x8dc -> vbi['status'] (lddecode_core.py:879-881)


class FrameCodes:
    """Philips codes per frame: returns the three code words of each field."""

    def __init__(self, first_frame=1, clv=False, fps=30, skip=None):
        self.first, self.clv, self.fps = first_frame, clv, fps
        self.skip = skip            # (k0, jump): frames k >= k0 are numbered `jump` higher (a cut disc)

    def frame_number(self, k):
        if self.skip is not None and k >= self.skip[0]:
            return self.first + k + self.skip[1]
        return self.first + k

    def codes(self, k):
        n = self.frame_number(k)
        if not self.clv:
            c = cav_code(n % 80000)
            return (c, c, STATUS_CODE)
        minutes, rem = divmod(n, 60 * self.fps)
        sec, fr = divmod(rem, self.fps)
        return (clv_minutes_code(minutes), clv_seconds_code(sec, fr), 0x87FFFF)


class SynthRF:
    """Chunked generator.  ``generate(n)`` returns float64 RF; ``encode`` quantises."""

    def __init__(self, system='NTSC', first_frame=1, clv=False, seed=20181015, noise=0.02,
                 start_line=100, audio=True, bars=True, code_fields=(0, 1), frame_skip=None, dropouts=()):
        self.p = NTSC if system == 'NTSC' else PAL
        p = self.p
        self.spl = FS * p['line_us'] / 1e6          # samples per line (2542.22 / 2560)
        self.codes = FrameCodes(first_frame, clv, 30 if system == 'NTSC' else 25, skip=frame_skip)
        self.dropouts = tuple(dropouts)              # (first sample, count): RF replaced by noise
        self.seed, self.noise, self.audio = seed, noise, audio
        self.t0_lines = start_line                  # capture starts this many lines into frame 0
        self.bars = bars
        self.code_fields = tuple(code_fields)        # fields carrying the Philips codes
        self.b_emp, self.a_emp = emphasis_filter(p)
        # band-limit of the hard-edged baseband (windowed sinc, 4.4 MHz)
        self.fir = sps.firwin(63, 4.4e6 / (FS / 2))
        self.reset()

    def reset(self):
        p = self.p
        self.pos = 0
        self.fir_hist = np.full(len(self.fir) - 1, p['ire0'])
        self.zi = sps.lfilter_zi(self.b_emp, self.a_emp) * p['ire0']
        self.phase = 0.0
        self.chunk_index = 0

    # -- baseband --------------------------------------------------------------
    def _ire(self, n):
        """Hard-edged composite IRE at absolute sample indices ``n`` (int64)."""
        p = self.p
        H = p['line_us']
        L = p['lines']
        lines_abs = n / self.spl + self.t0_lines
        hl = np.floor(lines_abs * 2).astype(np.int64)      # absolute half-line index
        frame = hl // (2 * L)
        h = hl - frame * 2 * L                                 # half-line within frame
        phi = (lines_abs * 2 - hl) * (H / 2)                   # us into the half-line
        ln = h // 2                                            # 0-based frame line
        tau = (lines_abs - np.floor(lines_abs)) * H            # us into the line
        ire = np.zeros(n.shape)
        sync = p['sync_ire']
        t_us = n / FS * 1e6 + self.t0_lines * H

        if p['system'] == 'NTSC':
            vi1 = h < 18
            vi2 = (h >= 525) & (h < 543)
            hv = np.where(vi1, h, h - 525)
            in_vi = vi1 | vi2
            eq = in_vi & ((hv < 6) | (hv >= 12))
            broad = in_vi & (hv >= 6) & (hv < 12)
            blank_half = (h == 543)
            normal = ~in_vi & ~blank_half
            vbi = ((ln >= 9) & (ln < 20)) | ((ln >= 272) & (ln < 283))
        else:
            # PAL: 5 eq + 5 broad + 5 eq half-lines around each field start
            # field 1 at half-line 0 (line 1), field 2 at half-line 625 (line 313.5)
            vi1 = (h < 15) | (h >= 2 * L - 5)
            vi2 = (h >= 620) & (h < 635)
            hv = np.where(h >= 2 * L - 5, h - 2 * L, h)
            hv = np.where(vi2, h - 625, hv)
            in_vi = vi1 | vi2
            eq = in_vi & ((hv < 0) | (hv >= 5))
            broad = in_vi & (hv >= 0) & (hv < 5)
            blank_half = np.zeros(n.shape, dtype=bool)
            normal = ~in_vi
            vbi = ((ln >= 7) & (ln < 22)) | ((ln >= 319) & (ln < 335))

        ire[eq & (phi < 2.35)] = sync
        ire[broad & (phi < H / 2 - 4.7)] = sync
        nl = normal
        ire[nl & (tau < 4.7)] = sync
        if p.get('pilot_hz'):
            tip = ire == sync
            ire[tip] += p['pilot_ire'] * np.sin(2 * np.pi * p['pilot_hz'] * (t_us[tip] * 1e-6))
        # colour burst: 9 (NTSC) / 10 (PAL) cycles from 5.3 us (5.6 us PAL)
        w = 2 * np.pi * p['fsc'] * (t_us * 1e-6)
        b0 = 5.3 if p['system'] == 'NTSC' else 5.6
        bdur = (9 if p['system'] == 'NTSC' else 10) / (p['fsc'] / 1e6)
        bmask = nl & (tau >= b0) & (tau < b0 + bdur)
        if p['system'] == 'NTSC':
            ire[bmask] += p['burst_ire'] * np.sin(w[bmask] + np.pi)
        else:
            sw = np.where(ln % 2 == 0, 1.0, -1.0)
            ire[bmask] += p['burst_ire'] * np.sin(w[bmask] + np.pi + sw[bmask] * np.pi / 4)
        # active picture
        a0, a1 = 9.4, H - 1.5
        act = nl & ~vbi & (tau >= a0) & (tau < a1)
        if np.any(act):
            x = (tau[act] - a0) / (a1 - a0)
            lnf = ln[act] % (L // 2 + 1)
            lower = lnf > (L // 2) * 2 // 3
            bar = np.minimum((x * 8).astype(np.int64), 7)
            yl = np.array([77.0, 69.0, 56.0, 48.0, 36.0, 28.0, 15.0, 7.5]) if p['setup'] else \
                np.array([75.0, 67.0, 53.0, 44.0, 31.0, 22.0, 9.0, 0.0])
            camp = np.array([0.0, 31.0, 44.0, 41.0, 41.0, 44.0, 31.0, 0.0])
            cph = np.deg2rad(np.array([0.0, 167.0, 283.0, 241.0, 61.0, 103.0, 347.0, 0.0]))
            y = np.where(lower, 100.0 * x, yl[bar]) if self.bars else 100.0 * x
            c = np.where(lower | (not self.bars), 0.0, camp[bar] * np.sin(w[act] + cph[bar]))
            ire[act] = y + c
        # Philips code lines
        for fld in self.code_fields:
            for j, cl in enumerate(p['code_lines'][fld]):
                m = normal & (ln == cl)
                if not np.any(m):
                    continue
                idx = np.nonzero(m)[0]
                ks = frame[idx]
                for k in np.unique(ks):
                    sel = idx[ks == k]
                    code = self.codes.codes(int(k))[j]
                    ire[sel] = self._code_wave(tau[sel], code, ire[sel])
        return ire

    @staticmethod
    def _code_wave(tau, code, base):
        """Bi-phase 24-bit code: 2 us cells from 10 us; bit 1 = low->high mid-cell."""
        out = base.copy()
        cell = np.floor((tau - 10.0) / 2.0).astype(np.int64)
        inside = (cell >= 0) & (cell < 24)
        if not np.any(inside):
            return out
        bits = np.array([(code >> (23 - i)) & 1 for i in range(24)])
        c = cell[inside]
        second_half = ((tau[inside] - 10.0) - 2.0 * c) >= 1.0
        b = bits[c]
        high = np.where(b == 1, second_half, ~second_half)
        out[inside] = np.where(high, 100.0, 0.0)
        return out

    # -- RF ----------------------------------------------------------------------
    def generate(self, count):
        p = self.p
        n = np.arange(self.pos, self.pos + count, dtype=np.int64)
        ire = self._ire(n)
        hz = p['ire0'] + p['hz_ire'] * ire
        # band-limit (carrying FIR history) then pre-emphasis (carrying IIR state)
        ext = np.concatenate([self.fir_hist, hz])
        bl = np.convolve(ext, self.fir, mode='valid')
        self.fir_hist = ext[-(len(self.fir) - 1):]
        emph, self.zi = sps.lfilter(self.b_emp, self.a_emp, bl, zi=self.zi)
        dph = (2 * np.pi / FS) * emph
        ph = self.phase + np.cumsum(dph)
        rf = np.cos(ph)
        self.phase = float(np.mod(ph[-1], 2 * np.pi))
        if self.audio:
            t = n / FS
            for fc, fm in ((p['audio_l'], 1000.0), (p['audio_r'], 400.0)):
                frac = np.mod(n * (fc / FS), 1.0)
                rf += 0.1 * np.cos(2 * np.pi * frac + (50000.0 / fm) * np.sin(2 * np.pi * fm * t))
        if self.noise:
            rng = np.random.default_rng([self.seed, self.chunk_index])
            rf += rng.normal(0.0, self.noise, count)
        for d0, dn in self.dropouts:
            a, b = max(d0, self.pos), min(d0 + dn, self.pos + count)
            if a < b:           # a dropout: the carrier is lost, only noise remains
                rng = np.random.default_rng([self.seed, 7, a])
                rf[a - self.pos:b - self.pos] = rng.normal(0.0, 0.3, b - a)
        self.pos += count
        self.chunk_index += 1
        return rf

    @staticmethod
    def quantise(rf, fmt):
        if fmt == 'u8':
            return np.clip(np.round(128 + 100 * rf / 1.3), 0, 255).astype(np.uint8)
        if fmt == 's16':
            return np.clip(np.round(rf * 20000), -32768, 32767).astype(np.int16)
        if fmt in ('r30', 'lds', '10bit'):
            return np.clip(np.round(512 + 400 * rf / 1.3), 0, 1023).astype(np.uint16)
        raise ValueError(fmt)


def make_capture(n_samples, fmt='u8', chunk=1 << 22, **kw):
    """Generate a whole capture and return its on-disk bytes (u8 / s16 / r30 / lds)."""
    g = SynthRF(**kw)
    parts = []
    left = n_samples
    while left > 0:
        c = min(chunk, left)
        parts.append(SynthRF.quantise(g.generate(c), fmt))
        left -= c
    s = np.concatenate(parts)
    if fmt == 'u8':
        return s.tobytes()
    if fmt == 's16':
        return s.astype('<i2').tobytes()
    if fmt == 'r30':
        from .formats import pack_r30
        return pack_r30(s)
    if fmt == 'lds':
        from .formats import pack_lds
        return pack_lds(s)
    raise ValueError(fmt)
