"""ORACLE (test infrastructure only): frame assembly and the CLI decode loop.

Restates Framer (lddecode_core.py:1193-1334), findframe (:1338-1378) and the
main loop of lddecode.py:39-107 over an in-memory ``Capture``.
``decode_capture`` returns the .tbc frames, .pcm audio and a per-frame
metadata record list (the build-defined JSON schema).
"""
import copy

import numpy as np

from .capture import FMT_LDS, FMT_R30, FMT_S16, FMT_U8, Capture
from .demod import RFDemod
from .field import Field, FieldNTSC, FieldPAL


class TrackedCapture(Capture):
    """Capture that remembers the byte offset after its last load (``fd.tell()``)."""

    def __init__(self, data, fmt):
        super().__init__(data, fmt)
        self.pos = 0

    def load(self, sample, readlen):
        sample, readlen = int(sample), int(readlen)
        if self.fmt == FMT_U8:
            start, need = sample, readlen
        elif self.fmt == FMT_S16:
            start, need = sample * 2, readlen * 2
        elif self.fmt == FMT_R30:
            start, need = (sample // 3) * 4, int(np.ceil(readlen * 3 / 4) * 4) + 4
        else:
            start, need = (sample // 4) * 5, int(np.ceil(readlen * 5 // 4)) + 5
        start = max(start, 0)
        self.pos = start + max(0, min(need, self.nbytes - start))
        return super().load(sample, readlen)


class Framer:
    """lddecode_core.py:1193-1334."""

    def __init__(self, rf, full_decode=True, log=print):
        self.rf = rf
        self.full_decode = full_decode
        self.log = log
        if rf.system == 'PAL':
            self.FieldClass, self.readlen, self.outlines, self.clvfps = FieldPAL, 1000000, 625, 25
        else:
            self.FieldClass, self.readlen, self.outlines, self.clvfps = FieldNTSC, 1000000, 525, 30
        if not full_decode:
            self.FieldClass = Field
        self.outwidth = rf.SysParams['outlinelen']
        self.audio_offset = 0
        self.mtf_level = 1
        self.field_log = []       # (readsample, nextsample, valid, istop, mtf) per Field built

    def readfield(self, capture, sample, fieldcount=0):
        """lddecode_core.py:1194-1223."""
        readsample = sample
        while True:
            raw = self.rf.demod(capture, readsample, self.readlen, self.mtf_level)
            if raw is None:
                return None, None, None
            f = self.FieldClass(self.rf, raw, 0, audio_offset=self.audio_offset)
            nextsample = readsample + f.nextfieldoffset
            if not f.valid:
                if len(f.peaklist) < 100:
                    nextsample = readsample + (self.rf.freq_hz * 10)
                elif len(f.vsyncs) == 0:
                    nextsample = readsample + (self.rf.freq_hz * 1)
            f.readsample, f.nextsample, f.mtf_level = readsample, nextsample, self.mtf_level
            self.field_log.append(f)
            if not f.valid:
                readsample = nextsample
            else:
                return f, readsample, nextsample

    def mergevbi(self, fields):
        """lddecode_core.py:1225-1236."""
        merged = copy.copy(fields[0].vbi)
        for k in merged.keys():
            if fields[1].vbi[k] is not None:
                merged[k] = fields[1].vbi[k]
        if merged['seconds'] is not None:
            merged['framenr'] = merged['minutes'] * 60 * self.clvfps
            merged['framenr'] += merged['seconds'] * self.clvfps
            merged['framenr'] += merged['clvframe']
        return merged

    def formatoutput(self, fields):
        """lddecode_core.py:1238-1252: interleave two fields into one frame."""
        W = self.outwidth
        lc = (min(fields[0].linecount, fields[1].linecount) * 2) - 0
        frame = np.zeros((W * self.outlines), dtype=np.uint16)
        src_w = fields[0].outlinelen
        for i in range(0, lc, 2):
            row = i // 2
            frame[i * W:(i + 1) * W] = fields[0].dspicture[row * src_w:row * src_w + W]
            frame[(i + 1) * W:(i + 2) * W] = fields[1].dspicture[row * src_w:row * src_w + W]
        longer = np.argmax([fields[0].linecount, fields[1].linecount])
        row = lc // 2
        frame[lc * W:(lc + 1) * W] = fields[longer].dspicture[row * src_w:row * src_w + W]
        return frame

    def readframe(self, capture, sample, firstframe=False, CAV=False):
        """lddecode_core.py:1254-1311 (including the MTF re-read recursion)."""
        fieldcount = 0
        fields = [None, None]
        audio = []
        f = None
        while fieldcount < 2:
            f, readsample, nextsample = self.readfield(capture, sample, fieldcount)
            if f is not None:
                self.log(sample, nextsample, f is not None, f.istop)
            else:
                self.log(sample, nextsample, f is not None)
            if f is not None:
                if f.istop:
                    fields[0] = f
                else:
                    fields[1] = f
                if ((not CAV and (f.istop == self.rf.SysParams['topfirst'])) or
                        (CAV and (f.vbi['framenr'] or f.vbi['minutes']))):
                    fieldcount = 1
                    self.firstsample = f.tbcstart + readsample
                elif fieldcount == 1:
                    fieldcount = 2
                if (fieldcount or not firstframe) and f.dsaudio is not None:
                    audio.append(f.dsaudio)
            elif readsample is None:
                return None, None, None, None
            sample = nextsample
        if len(audio):
            conaudio = np.concatenate(audio)
            self.audio_offset = f.audio_next_offset
        else:
            conaudio = None
        combined = self.formatoutput(fields) if self.full_decode else None
        self.vbi = self.mergevbi(fields)
        if not f.vbi['isclv'] and f.vbi['framenr'] is not None:
            newmtf = 1 - (f.vbi['framenr'] / 10000)
            if newmtf < 0:
                newmtf = 0
            oldmtf = self.mtf_level
            self.mtf_level = newmtf
            if np.abs(newmtf - oldmtf) > .1:
                return self.readframe(capture, sample, firstframe, CAV)
        return combined, conaudio, sample, fields


def findframe(capture, rf, target, nextsample=0, log=print):
    """lddecode_core.py:1338-1378: seek to a VBI frame number."""
    framer = Framer(rf, full_decode=False, log=log)
    spf = int(rf.freq_hz / rf.SysParams['FPS'])
    framer.vbi = {'framenr': None}
    iscav = False
    retry = 5
    rv = None
    tolerance = 0
    while framer.vbi['framenr'] is None and retry:
        rv = framer.readframe(capture, nextsample, CAV=False)
        log(rv, framer.vbi)
        if framer.vbi['isclv']:
            tolerance = 1
        else:
            tolerance = 0
            iscav = True
        nextsample = rv[2] + (rf.freq_hz * 10)
        retry -= 1
    if retry == 0 and framer.vbi['framenr'] is None:
        log("SEEK ERROR: Unable to find a usable frame")
        return None
    retry = 5
    while np.abs(target - framer.vbi['framenr']) > tolerance and retry:
        offset = (spf * (target - 1 - framer.vbi['framenr']))
        nextsample = rv[2] + offset
        rv = framer.readframe(capture, nextsample, CAV=iscav)
        log(framer.vbi)
        retry -= 1
    if np.abs(target - framer.vbi['framenr']) > tolerance:
        log("SEEK WARNING: seeked to frame {0} instead of {1}".format(framer.vbi['framenr'], target))
    return nextsample


def field_record(f):
    """Per-field metadata (build-defined JSON schema; every member is reference-computed)."""
    rec = {'readsample': int(f.readsample), 'nextsample': int(f.nextsample), 'valid': bool(f.valid),
           'mtf_level': float(f.mtf_level)}
    if f.valid:
        rec.update({'istop': bool(f.istop), 'linecount': int(f.linecount),
                    'nextfieldoffset': int(f.nextfieldoffset),
                    'vbi': {k: (None if v is None else (bool(v) if isinstance(v, (bool, np.bool_)) else int(v)))
                            for k, v in f.vbi.items()},
                    'linecode': {str(k): (None if v is None else [int(x) for x in v])
                                 for k, v in f.linecode.items()}})
    return rec


def decode_capture(data, fmt, system='NTSC', start=0, length=None, seek=-1, log=None):
    """The lddecode.py:39-107 decode loop (no cut mode).

    Returns (tbc_frames list[np.uint16 array], pcm list[np.int16 array], meta list[dict]).
    """
    log = log or (lambda *a, **k: None)
    rf = RFDemod(system=system)
    spf = int(rf.freq_hz / rf.SysParams['FPS']) + 1
    bpf = spf * 5 // 4                        # (sic) 10-bit packing assumed, lddecode.py:42
    cap = TrackedCapture(data, fmt)
    size = cap.nbytes
    if (size // bpf - start) < 2:
        raise ValueError('start frame is past end of file')
    num_frames = length if length is not None else size // bpf - start
    if seek >= 0:
        nextsample = findframe(cap, rf, seek, start * spf, log=log)
    else:
        nextsample = start * spf
    framer = Framer(rf, log=log)
    frames, pcm, meta = [], [], []
    for fi in range(0, num_frames):
        if cap.pos + bpf * 1.05 <= size:
            nlog = len(framer.field_log)
            combined, audio, nextsample, fields = framer.readframe(cap, nextsample, fi == 0)
            log('frame ', framer.vbi['framenr'])
            frames.append(combined)
            pcm.append(audio)
            meta.append({'frame': fi, 'vbi': {k: (None if v is None else
                                                  (bool(v) if isinstance(v, (bool, np.bool_)) else int(v)))
                                              for k, v in framer.vbi.items()},
                         'nextsample': int(nextsample),
                         'fields': [field_record(x) for x in framer.field_log[nlog:]]})
        else:
            break
    return frames, pcm, meta
