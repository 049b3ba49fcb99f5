"""Host-side system constants and RF filter tables for the GPU decoder.

Builds, once per system, exactly the tables RFDecode builds
(lddecode_core.py:119-279; constants :30-117; lddutils.filtfft :256-257) and
packs them for ``ldg_set_filters``.  Filter *design* stays on the host
(scipy.signal, like the reference); everything per-sample runs on the GPU.
"""
from dataclasses import dataclass, field

import numpy as np
import scipy.signal as sps

BLOCKLEN = 16384
TAU = np.pi * 2


@dataclass(frozen=True)
class System:
    """SysParams_NTSC / SysParams_PAL + RFParams_* (lddecode_core.py:30-117)."""
    name: str
    fsc_mhz: float
    pilot_mhz: float
    frame_lines: int
    ire0: float
    hz_ire: float
    vsync_ire: float
    audio_lfreq: float
    audio_rfreq: float
    codelines: tuple
    topfirst: bool
    line_period: float
    fps: float
    outlinelen: int
    notch_width: float
    notch_order: int
    deemp: tuple
    bpf: tuple
    bpf_order: int
    lpf_freq: float
    lpf_order: int
    mtf_poles: tuple = field(default=())

    @property
    def clvfps(self):
        return 25 if self.name == 'PAL' else 30


def _ntsc():
    fsc = 315.0 / 88.0
    lp = 1 / (fsc / 227.5)
    return System('NTSC', fsc, fsc, 525, 8100000, 1700000 / 140.0, -40,
                  (1000000 * 315 / 88 / 227.5) * 146.25, (1000000 * 315 / 88 / 227.5) * 178.75,
                  (16, 17, 18), True, lp, 1000000 / (525 * lp), int(np.round(lp * fsc * 4)),
                  350000, 2, (120 * .32, 320 * .32), (3500000, 13200000), 3, 4200000, 5,
                  (np.pi * 12.5 / 20, np.pi * 27.5 / 20))


def _pal():
    fsc = ((1 / 64) * 283.75) + (25 / 1000000)
    return System('PAL', fsc, 3.75, 625, 7100000, 800000 / 100.0, -.3 * (100 / .7),
                  (1000000 / 64) * 43.75, (1000000 / 64) * 68.25, (19, 20, 21), False, 64, 25,
                  int(np.round(64 * fsc * 4)), 200000, 2, (100 * .4, 400 * .4), (2500000, 14500000), 3,
                  5200000, 9, (np.pi * 10 / 20, np.pi * 28 / 20))


SYSTEMS = {'NTSC': _ntsc(), 'PAL': _pal()}


def _whole(ba, n=BLOCKLEN):
    return sps.freqz(ba[0], ba[1], n, whole=1)[1]


class RFTables:
    """The filter set of one system at 40 MSPS, plus the derived scalars."""

    def __init__(self, system='NTSC', inputfreq=40):
        S = SYSTEMS[system]
        self.system = S
        self.freq = inputfreq                         # MHz, int like rf.freq
        self.freq_hz = inputfreq * 1000000
        nyq = self.freq_hz / 2
        nyq_mhz = inputfreq / 2
        self.linelen = int(np.round(self.freq_hz / (1000000.0 / S.line_period)))
        self.samples_per_frame = int(self.freq_hz / S.fps) + 1

        hil_fir = np.fft.fftshift(np.fft.ifft([0] + [1] * 128 + [0] * 128))
        hil = np.fft.fft(hil_fir, BLOCKLEN)
        poles = [.7 * np.exp(1j * a) for a in S.mtf_poles]
        mtf = _whole(sps.zpk2tf([], poles, 1.11))
        rfv = _whole(sps.butter(S.bpf_order, [S.bpf[0] / nyq, S.bpf[1] / nyq], btype='bandpass'))
        cuts = [_whole(sps.butter(S.notch_order, [(c - S.notch_width) / nyq, (c + S.notch_width) / nyq],
                                  btype='bandstop')) for c in (S.audio_lfreq, S.audio_rfreq)]
        rfv *= (cuts[0] * cuts[1])
        rfv *= hil
        lpf = _whole(sps.butter(S.lpf_order, S.lpf_freq / nyq, 'low'))
        d0, d1 = S.deemp
        tb, ta = sps.zpk2tf([-d1 * 1e-10], [-d0 * 1e-10], d0 / d1)
        deemp = _whole(sps.bilinear(tb, ta, 1.0 / nyq))
        f05_fir = sps.firwin(65, [0.5 / nyq_mhz], pass_zero=True)
        f05 = _whole((f05_fir, [1.0]))
        burst_ba = sps.butter(1, [(S.fsc_mhz - .1) / nyq_mhz, (S.fsc_mhz + .1) / nyq_mhz], btype='bandpass')
        burst = _whole(burst_ba)
        psync_ba = sps.butter(1, 0.05 / nyq_mhz, btype='low')
        pilot_ba = sps.butter(1, [3.7 / nyq_mhz, 3.8 / nyq_mhz], btype='bandpass') if S.name == 'PAL' else None
        self.tables = {
            'rfvideo': rfv, 'mtf': mtf,
            'fvideo': lpf * deemp,
            'fvideo05': lpf * deemp * f05,
            'fvideoburst': lpf * deemp * burst,
            'fpsync': _whole(psync_ba),
            'mtf_logabs': np.log(np.abs(mtf)),
            'mtf_arg': np.angle(mtf),
        }
        if S.name == 'PAL':
            self.tables['fvideopilot'] = lpf * deemp * _whole(pilot_ba)
        # the butter(1) designs behind fpsync / Fburst / Fpilot (a[0] == 1): the demod
        # runs these three channels as periodic recurrences (csrc/iir.hpp)
        iir = [psync_ba[0][0], psync_ba[0][1], psync_ba[1][1],
               *burst_ba[0], *burst_ba[1][1:]]
        iir += ([*pilot_ba[0], *pilot_ba[1][1:]] if pilot_ba is not None else [0.0] * 5)
        self.tables['iir'] = np.array(iir, np.float64)
        # the F05 taps: ldg_set_filters cross-checks fvideo05 == fvideo * DFT(taps)
        self.tables['f05_fir'] = np.asarray(f05_fir, np.float64)

        # audio (lddecode_core.py:223-279)
        fdiv1 = 32 if inputfreq >= 32 else 16
        half = BLOCKLEN // (fdiv1 * 2)
        self.freq_arf = self.freq_hz / (fdiv1 / 2)
        cfreq = (S.audio_rfreq + S.audio_lfreq) // 2
        centre = int((cfreq / self.freq_hz) * BLOCKLEN)
        a0, a1 = int(centre - half), int(centre + half)
        self.audio_lo0 = a0
        self.audio_lowfreq = cfreq - (self.freq_hz / (2 * fdiv1))

        def slice_(spec):
            return np.concatenate([spec[a0:a1], spec[BLOCKLEN - a1:BLOCKLEN - a0]])

        for key, c in (('audio_lfilt', S.audio_lfreq), ('audio_rfilt', S.audio_rfreq)):
            taps = sps.firwin(800, [(c - 150000) / nyq, (c + 150000) / nyq], pass_zero=False)
            self.tables[key] = slice_(_whole([taps, 1.0]) * hil)
        freq_aud2 = self.freq_arf / 4
        self.tables['audio_lpf2'] = _whole([sps.firwin(65, [21000 / (freq_aud2 / 2)]), [1.0]], BLOCKLEN // 4)

    def iretohz(self, ire):
        return self.system.ire0 + (self.system.hz_ire * ire)

    def params(self):
        S = self.system
        return {'freq_hz': float(self.freq_hz), 'freq': float(self.freq), 'ire0': float(S.ire0),
                'hz_ire': float(S.hz_ire), 'vsync_ire': float(S.vsync_ire),
                'sync_lo': float(self.iretohz(-55)), 'sync_hi': float(self.iretohz(-25)),
                'freq_arf': float(self.freq_arf), 'audio_lowfreq': float(self.audio_lowfreq),
                'audio_lfreq': float(S.audio_lfreq), 'audio_rfreq': float(S.audio_rfreq),
                'line_period': float(S.line_period), 'fsc_mhz': float(S.fsc_mhz),
                'linelen': self.linelen, 'outlinelen': S.outlinelen, 'frame_lines': S.frame_lines,
                'audio_lo0': self.audio_lo0, 'codelines': list(S.codelines)}
