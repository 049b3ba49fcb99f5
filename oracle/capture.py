"""ORACLE (test infrastructure only): RF capture loaders.

Restates the loader plugin API of lddutils.py:117-229:
``loader(infile, sample, readlen) -> ndarray | None`` for unpacked u8/s16
(:131-147), ``.r30`` three-10-bit-in-uint32 (:150-173) and ``.lds`` four
10-bit samples in 5 bytes (:195-229).  The capture is held in memory
(``bytes`` / numpy buffer) instead of a seekable file; short reads at EOF
behave like the reference's ``read()`` returning fewer bytes.
"""
import numpy as np

FMT_U8, FMT_S16, FMT_R30, FMT_LDS = 0, 1, 2, 3
FMT_BY_EXT = {'u8': FMT_U8, 'raw': FMT_U8, 'r8': FMT_U8, 'r16': FMT_S16, 's16': FMT_S16,
              'r30': FMT_R30, 'lds': FMT_LDS}


class LoaderShapeError(Exception):
    """The reference loader raised (numpy broadcast error on a short read)."""


class Capture:
    """An RF capture in one of the four on-disk formats."""

    def __init__(self, data, fmt):
        self.buf = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) \
            else data.view(np.uint8).reshape(-1)
        self.fmt = fmt

    @property
    def nbytes(self):
        return self.buf.size

    def _read_bytes(self, pos, n):
        pos = max(0, int(pos))
        return self.buf[pos:pos + int(n)]

    def load(self, sample, readlen):
        """One loader call, with the reference's exact semantics."""
        sample, readlen = int(sample), int(readlen)
        if self.fmt == FMT_U8:        # lddutils.py:131-144
            return self._read_bytes(sample, readlen).copy()
        if self.fmt == FMT_S16:       # lddutils.py:131-147
            raw = self._read_bytes(sample * 2, readlen * 2)
            raw = raw[:(raw.size // 2) * 2]
            return raw.view('<i2').copy()
        if self.fmt == FMT_R30:       # lddutils.py:150-173
            start, offset = (sample // 3) * 4, sample % 3
            needed = int(np.ceil(readlen * 3 / 4) * 4) + 4
            raw = self._read_bytes(start, needed).copy()
            words = raw[:(raw.size // 4) * 4].view('<u4')
            out = np.zeros(words.size * 3, dtype=np.int16)
            out[0::3] = words & 0x3ff
            out[1::3] = (words >> 10) & 0x3ff
            out[2::3] = (words >> 20) & 0x3ff
            return out[offset:offset + readlen]
        if self.fmt == FMT_LDS:       # lddutils.py:195-229
            start, offset = (sample // 4) * 5, sample % 4
            needed = int(np.ceil(readlen * 5 // 4)) + 5
            b = self._read_bytes(start, needed).astype(np.uint16)
            out = np.zeros(readlen + 4, dtype=np.uint16)
            lanes = [b[0::5], b[1::5], b[2::5], b[3::5], b[4::5]]
            # each output lane k is built from byte lanes k and k+1 (broadcast must match)
            for k in range(4):
                if not (out[k::4].size == lanes[k].size == lanes[k + 1].size):
                    raise LoaderShapeError('short .lds read')
            out[0::4] = (lanes[0] << 2) | ((lanes[1] >> 6) & 0x03)
            out[1::4] = ((lanes[1] & 0x3f) << 4) | ((lanes[2] >> 4) & 0x0f)
            out[2::4] = ((lanes[2] & 0x0f) << 6) | ((lanes[3] >> 2) & 0x3f)
            out[3::4] = ((lanes[3] & 0x03) << 8) | lanes[4]
            return out[offset:offset + readlen]
        raise ValueError(self.fmt)

    def num_samples(self):
        n = self.nbytes
        return {FMT_U8: n, FMT_S16: n // 2, FMT_R30: (n // 4) * 3, FMT_LDS: (n // 5) * 4}[self.fmt]


def pack_r30(samples10):
    """Pack unsigned 10-bit samples three per little-endian uint32 (ddpack.c:18-23 layout)."""
    s = np.asarray(samples10, dtype=np.uint32)
    n = (s.size // 3) * 3
    s = s[:n].reshape(-1, 3)
    words = (s[:, 0] & 0x3ff) | ((s[:, 1] & 0x3ff) << 10) | ((s[:, 2] & 0x3ff) << 20)
    return words.astype('<u4').tobytes()


def pack_lds(samples10):
    """Pack 10-bit samples four per five bytes (inverse of lddutils.py:213-227)."""
    s = np.asarray(samples10, dtype=np.uint16)
    n = (s.size // 4) * 4
    s = s[:n].reshape(-1, 4).astype(np.uint16)
    out = np.empty((s.shape[0], 5), dtype=np.uint8)
    out[:, 0] = s[:, 0] >> 2
    out[:, 1] = ((s[:, 0] & 0x3) << 6) | (s[:, 1] >> 4)
    out[:, 2] = ((s[:, 1] & 0xf) << 4) | (s[:, 2] >> 6)
    out[:, 3] = ((s[:, 2] & 0x3f) << 2) | (s[:, 3] >> 8)
    out[:, 4] = s[:, 3] & 0xff
    return out.tobytes()
