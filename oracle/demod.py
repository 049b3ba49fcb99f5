"""ORACLE (test infrastructure only): RF demodulation.

Restates RFDecode.demodblock / runfilter_audio_phase2 / audio_phase2 / demod
(lddecode_core.py:288-427) and lddutils.unwrap_hilbert / inrange
(lddutils.py:259-260, 320-334) with plain numpy, operation for operation.
Channel records are dicts of float64 arrays keyed like the reference's
rec-arrays ('demod', 'demod_05', 'demod_sync', 'demod_burst'[, 'demod_pilot'];
'audio_left', 'audio_right').
"""
import numpy as np

from .params import FilterSet

TAU = np.pi * 2


class ReferenceCrash(Exception):
    """The reference would have raised an uncaught exception here."""


def inrange(a, lo, hi):
    return (a >= lo) & (a <= hi)


def unwrap_hilbert(analytic, freq_hz):
    """lddutils.py:320-334 -- FM demodulation of an analytic signal (Hz)."""
    ang = np.angle(analytic)
    d = np.pad(np.diff(ang), (1, 0), mode='constant')
    if d[0] < -np.pi:
        d[0] += TAU
    u = np.unwrap(d)
    while np.min(u) < 0:
        u[u < 0] += TAU
    while np.max(u) > TAU:
        u[u > TAU] -= TAU
    return u * (freq_hz / TAU)


class RFDemod(FilterSet):
    """Oracle RFDecode: filter set + block demodulator + overlap-save driver."""

    def demodblock(self, data, mtf_level=0):
        """lddecode_core.py:288-330."""
        F = self.Filters
        spec = np.fft.fft(data[:self.blocklen])
        filt = spec * F['RFVideo']
        if mtf_level != 0:
            filt *= F['MTF'] ** mtf_level
        demod = unwrap_hilbert(np.fft.ifft(filt), self.freq_hz)
        dspec = np.fft.fft(demod)
        video = {}
        video['demod'] = np.fft.ifft(dspec * F['FVideo']).real
        v05 = np.fft.ifft(dspec * F['FVideo05']).real
        video['demod_05'] = np.roll(v05, -F['F05_offset'])
        video['demod_burst'] = np.fft.ifft(dspec * F['FVideoBurst']).real
        sync_in = inrange(video['demod_05'], self.iretohz(-55), self.iretohz(-25))
        video['demod_sync'] = np.fft.ifft(np.fft.fft(sync_in) * F['FPsync']).real
        if self.system == 'PAL':
            video['demod_pilot'] = np.fft.ifft(dspec * F['FVideoPilot']).real
        if not self.decode_analog_audio:
            return video, None
        sliced = self.audio_fdslice(spec)
        audio = {}
        for ch, key in (('audio_left', 'audio_lfilt'), ('audio_right', 'audio_rfilt')):
            a = np.fft.ifft(sliced * F[key])
            audio[ch] = unwrap_hilbert(a, F['freq_arf']) + F['audio_lowfreq']
        return video, audio

    def video_channels(self):
        base = ['demod', 'demod_05', 'demod_sync', 'demod_burst']
        return base + (['demod_pilot'] if self.system == 'PAL' else [])

    def _phase2_block(self, faudio, start):
        """runfilter_audio_phase2, lddecode_core.py:335-346."""
        F = self.Filters
        out = {}
        for ch in ('audio_left', 'audio_right'):
            seg = faudio[ch][start:start + self.blocklen].copy()
            spec = self.audio_fdslice2(np.fft.fft(seg)) * F['audio_lpf2']
            out[ch] = np.fft.ifft(spec).real / F['audio_fdiv2']
        return out

    def audio_phase2(self, faudio):
        """lddecode_core.py:348-371 (second audio decimation over one field read)."""
        F = self.Filters
        n_in = faudio['audio_left'].shape[0]
        n_out = n_in // F['audio_fdiv2']
        res = {ch: np.zeros(n_out) for ch in ('audio_left', 'audio_right')}
        tmp = self._phase2_block(faudio, 0)
        first = tmp['audio_left'].shape[0]
        for ch in res:
            res[ch][:first] = tmp[ch]
        skip = 64
        jump = self.blocklen - skip * F['audio_fdiv2']
        pos = first
        for s in range(jump, n_in - jump, jump):
            tmp = self._phase2_block(faudio, s)
            m = tmp['audio_left'].shape[0] - skip
            for ch in res:
                dst = res[ch][pos:pos + m]
                if dst.shape[0] != m:
                    raise ReferenceCrash('audio_phase2 broadcast')
                res[ch][pos:pos + m] = tmp[ch][skip:]
            pos += m
        tmp = self._phase2_block(faudio, n_in - self.blocklen - 1)
        m = tmp['audio_left'].shape[0] - skip
        for ch in res:
            res[ch][n_out - m:] = tmp[ch][skip:]
        return res

    def block_starts(self, start, length):
        """The overlap-save grid of one demod() call (lddecode_core.py:374-385)."""
        end = int(start + length) + 1
        start = int(start - self.blockcut) if start > self.blockcut else 0
        step = self.blocklen - self.blockcut - self.blockcut_end
        return start, end, list(range(start, end, step))

    def demod(self, capture, start, length, mtf_level=0):
        """lddecode_core.py:373-427.  Returns (video, audio) or None on loader failure."""
        start0, end, starts = self.block_starts(start, length)
        step = self.blocklen - self.blockcut - self.blockcut_end
        n_out = end - start0 + 1
        video = audio = None
        tv = ta = None
        for i in starts:
            try:
                raw = capture.load(i, self.blocklen)
            except Exception:
                return None
            if raw is None:
                return None
            if raw.shape[0] < self.blocklen:
                # the reference's demodblock would multiply mismatched shapes
                raise ReferenceCrash('short block read at sample %d' % i)
            tv, ta = self.demodblock(raw, mtf_level=mtf_level)
            if video is None:
                video = {k: np.zeros(n_out) for k in tv}
            off = i - start0
            if off + (self.blocklen - self.blockcut) > n_out:
                copylen = n_out - off
            else:
                copylen = step
            for k in tv:
                video[k][off:off + copylen] = tv[k][self.blockcut:self.blockcut + copylen]
            if ta is not None:
                ds = tv['demod'].shape[0] // ta['audio_left'].shape[0]
                if audio is None:
                    audio = {k: np.zeros(((end - start0) // ds) + 1) for k in ta}
                for k in ta:
                    a0, a1 = off // ds, (off + copylen) // ds
                    audio[k][a0:a1] = ta[k][self.blockcut // ds:(self.blockcut + copylen) // ds]
        if ta is not None:
            return video, self.audio_phase2(audio)
        return video, None
