"""ORACLE (test infrastructure only): system constants and the RF filter set.

Restates lddecode_core.py:23-117 (SysParams_* / RFParams_*) and
lddecode_core.py:119-279 (RFDecode.__init__, computevideofilters,
computeaudiofilters) plus lddutils.py:246-257 (hilbert_filter, filtfft).

numpy-2/scipy-1.15 adaptations: ``sps.zpk2tf`` is given list
arguments where the reference passed scalars (identical math:
old scipy applied ``atleast_1d`` itself).
"""
import numpy as np
import scipy.signal as sps


def _round_line(sp, mult, mhz_key):
    """calclinelen, lddecode_core.py:23-27."""
    return int(np.round(sp['line_period'] * sp[mhz_key] * mult))


def system_params(system):
    """Return fresh copies of (SysParams, RFParams) for 'NTSC' or 'PAL'.

    lddecode_core.py:30-117.  Fresh dicts per decoder because the reference
    mutates SysParams at runtime (audio_cfreq, lddecode_core.py:239).
    """
    if system == 'NTSC':
        fsc = 315.0 / 88.0
        sp = {
            'fsc_mhz': fsc, 'pilot_mhz': fsc, 'frame_lines': 525,
            'ire0': 8100000, 'hz_ire': 1700000 / 140.0, 'vsync_ire': -40,
            'analog_audio': True,
            'audio_lfreq': (1000000 * 315 / 88 / 227.5) * 146.25,
            'audio_rfreq': (1000000 * 315 / 88 / 227.5) * 178.75,
            'philips_codelines': [16, 17, 18], 'topfirst': True,
        }
        sp['line_period'] = 1 / (fsc / 227.5)
        sp['FPS'] = 1000000 / (525 * sp['line_period'])
        sp['outlinelen'] = _round_line(sp, 4, 'fsc_mhz')
        rp = {
            'audio_notchwidth': 350000, 'audio_notchorder': 2,
            'video_deemp': (120 * .32, 320 * .32),
            'video_bpf': [3500000, 13200000], 'video_bpf_order': 3,
            'video_lpf_freq': 4200000, 'video_lpf_order': 5,
        }
    elif system == 'PAL':
        sp = {
            'FPS': 25, 'fsc_mhz': ((1 / 64) * 283.75) + (25 / 1000000),
            'pilot_mhz': 3.75, 'frame_lines': 625, 'line_period': 64,
            'ire0': 7100000, 'hz_ire': 800000 / 100.0,
            'analog_audio': True,
            'audio_lfreq': (1000000 / 64) * 43.75,
            'audio_rfreq': (1000000 / 64) * 68.25,
            'philips_codelines': [19, 20, 21], 'topfirst': False,
        }
        sp['outlinelen'] = _round_line(sp, 4, 'fsc_mhz')
        sp['outlinelen_pilot'] = _round_line(sp, 4, 'pilot_mhz')
        sp['vsync_ire'] = -.3 * (100 / .7)
        rp = {
            'audio_notchwidth': 200000, 'audio_notchorder': 2,
            'video_deemp': (100 * .4, 400 * .4),
            'video_bpf': (2500000, 14500000), 'video_bpf_order': 3,
            'video_lpf_freq': 5200000, 'video_lpf_order': 9,
        }
    else:
        raise ValueError(system)
    return sp, rp


# lddutils.py:246-249: 257-tap one-sided (complex) "hilbert" FIR.
HILBERT_TERMS = 128
HILBERT_FIR = np.fft.fftshift(np.fft.ifft([0] + [1] * HILBERT_TERMS + [0] * HILBERT_TERMS))


def freq_response(ba, n):
    """filtfft, lddutils.py:256-257: whole-circle freqz sampled at n points."""
    return sps.freqz(ba[0], ba[1], n, whole=1)[1]


def _polar(r, theta):
    return r * np.exp(1j * theta)


class FilterSet:
    """The RFDecode filter tables (lddecode_core.py:119-279).

    Attributes mirror the reference: ``blocklen``, ``blockcut``,
    ``blockcut_end``, ``freq`` (MHz), ``freq_hz``, ``linelen``, ``SysParams``,
    ``DecoderParams`` and the ``Filters`` dict.
    """

    def __init__(self, inputfreq=40, system='NTSC', blocklen=16384, decode_analog_audio=True):
        self.blocklen = blocklen
        self.blockcut = 1024
        self.system = system
        self.freq = inputfreq
        self.freq_half = inputfreq / 2
        self.freq_hz = inputfreq * 1000000
        self.freq_hz_half = inputfreq * 1000000 / 2
        self.SysParams, self.DecoderParams = system_params(system)
        self.linelen = int(np.round(self.freq_hz / (1000000.0 / self.SysParams['line_period'])))
        self.decode_analog_audio = decode_analog_audio
        self.Filters = {}
        self._video_filters()
        if decode_analog_audio:
            self._audio_filters()
        self.blockcut_end = self.Filters['F05_offset']

    # lddecode_core.py:152-214
    def _video_filters(self):
        sp, dp, n = self.SysParams, self.DecoderParams, self.blocklen
        nyq_hz, nyq_mhz = self.freq_hz_half, self.freq_half
        f = self.Filters
        if self.system == 'NTSC':
            poles = [_polar(.7, np.pi * 12.5 / 20), _polar(.7, np.pi * 27.5 / 20)]
        else:
            poles = [_polar(.7, np.pi * 10 / 20), _polar(.7, np.pi * 28 / 20)]
        f['MTF'] = freq_response(sps.zpk2tf([], poles, 1.11), n)
        f['hilbert'] = np.fft.fft(HILBERT_FIR, n)

        bpf = sps.butter(dp['video_bpf_order'],
                         [dp['video_bpf'][0] / nyq_hz, dp['video_bpf'][1] / nyq_hz], btype='bandpass')
        f['RFVideo'] = freq_response(bpf, n)
        if sp['analog_audio']:
            w = dp['audio_notchwidth']
            for key, carrier in (('Fcutl', sp['audio_lfreq']), ('Fcutr', sp['audio_rfreq'])):
                notch = sps.butter(dp['audio_notchorder'],
                                   [(carrier - w) / nyq_hz, (carrier + w) / nyq_hz], btype='bandstop')
                f[key] = freq_response(notch, n)
            f['RFVideo'] *= (f['Fcutl'] * f['Fcutr'])
        f['RFVideo'] *= f['hilbert']

        lpf = sps.butter(dp['video_lpf_order'], dp['video_lpf_freq'] / nyq_hz, 'low')
        f['Fvideo_lpf'] = freq_response(lpf, n)

        d0, d1 = dp['video_deemp']
        tb, ta = sps.zpk2tf([-d1 * (10 ** -10)], [-d0 * (10 ** -10)], d0 / d1)
        f['Fdeemp'] = freq_response(sps.bilinear(tb, ta, 1.0 / nyq_hz), n)
        tb, ta = sps.zpk2tf([-d0 * (10 ** -10)], [-d1 * (10 ** -10)], d1 / d0)
        f['Femp'] = freq_response(sps.bilinear(tb, ta, 1.0 / nyq_hz), n)
        f['FVideo'] = f['Fvideo_lpf'] * f['Fdeemp']

        f05 = sps.firwin(65, [0.5 / nyq_mhz], pass_zero=True)
        f['F05_offset'] = 32
        f['F05'] = freq_response((f05, [1.0]), n)
        f['FVideo05'] = f['Fvideo_lpf'] * f['Fdeemp'] * f['F05']

        fsc = sp['fsc_mhz']
        burst = sps.butter(1, [(fsc - .1) / nyq_mhz, (fsc + .1) / nyq_mhz], btype='bandpass')
        f['Fburst'] = freq_response(burst, n)
        f['FVideoBurst'] = f['Fvideo_lpf'] * f['Fdeemp'] * f['Fburst']
        if self.system == 'PAL':
            pilot = sps.butter(1, [3.7 / nyq_mhz, 3.8 / nyq_mhz], btype='bandpass')
            f['Fpilot'] = freq_response(pilot, n)
            f['FVideoPilot'] = f['Fvideo_lpf'] * f['Fdeemp'] * f['Fpilot']
        f['FPsync'] = freq_response(sps.butter(1, 0.05 / nyq_mhz, btype='low'), n)

    # lddecode_core.py:217-279
    def _audio_filters(self):
        f, sp, n = self.Filters, self.SysParams, self.blocklen
        fdiv1 = 32 if self.freq >= 32 else 16
        half = n // (fdiv1 * 2)
        f['freq_arf'] = self.freq_hz / (fdiv1 / 2)
        f['audio_fdiv1'] = fdiv1
        sp['audio_cfreq'] = (sp['audio_rfreq'] + sp['audio_lfreq']) // 2
        centre = int((sp['audio_cfreq'] / self.freq_hz) * n)
        lo, hi = int(centre - half), int(centre + half)
        f['audio_fdslice_lo'] = slice(lo, hi)
        f['audio_fdslice_hi'] = slice(n - hi, n - lo)
        f['audio_lowfreq'] = sp['audio_cfreq'] - (self.freq_hz / (2 * fdiv1))

        apass = 150000
        for key, carrier in (('audio_lfilt', sp['audio_lfreq']), ('audio_rfilt', sp['audio_rfreq'])):
            taps = sps.firwin(800, [(carrier - apass) / self.freq_hz_half,
                                    (carrier + apass) / self.freq_hz_half], pass_zero=False)
            f[key] = self.audio_fdslice(freq_response([taps, 1.0], n) * f['hilbert'])

        fdiv2 = 4
        f['audio_fdiv2'] = fdiv2
        f['audio_fdiv'] = fdiv1 * fdiv2
        f['freq_aud2'] = f['freq_arf'] / fdiv2
        f['audio_fdslice2_lo'] = slice(0, n // (fdiv2 * 2))
        f['audio_fdslice2_hi'] = slice(n - n // (fdiv2 * 2), n)
        f['audio_lpf2'] = freq_response([sps.firwin(65, [21000 / (f['freq_aud2'] / 2)]), [1.0]], n // fdiv2)
        d75 = 1000000 / (2 * np.pi * 75)
        db, da = sps.butter(1, [d75 / (f['freq_aud2'] / 2)], btype='lowpass')
        f['audio_deemp2'] = freq_response([db, da], n // fdiv2)   # computed, never applied (:343)

    def audio_fdslice(self, spec):
        return np.concatenate([spec[self.Filters['audio_fdslice_lo']], spec[self.Filters['audio_fdslice_hi']]])

    def audio_fdslice2(self, spec):
        return np.concatenate([spec[self.Filters['audio_fdslice2_lo']], spec[self.Filters['audio_fdslice2_hi']]])

    def iretohz(self, ire):
        return self.SysParams['ire0'] + (self.SysParams['hz_ire'] * ire)

    def hztoire(self, hz):
        return (hz - self.SysParams['ire0']) / self.SysParams['hz_ire']
