"""RF capture container formats (the loader plugin API's four formats).

Byte layouts follow lddutils.py:131-229 (readers) and ddpack.c:11-29 (.r30
writer).  These are host-side helpers for writing test/bench captures and for
the CLI's cut mode; the decode path unpacks on the GPU inside the demod kernel
(csrc/demod.hip load_sample).
"""
import numpy as np

FMT_U8, FMT_S16, FMT_R30, FMT_LDS = 0, 1, 2, 3
EXT_TO_FMT = {'u8': FMT_U8, 'raw': FMT_U8, 'r8': FMT_U8, 'r16': FMT_S16, 's16': FMT_S16,
              'r30': FMT_R30, 'lds': FMT_LDS}
NAME_TO_FMT = {'u8': FMT_U8, 's16': FMT_S16, 'r30': FMT_R30, 'lds': FMT_LDS}


def fmt_from_path(path):
    """Loader selection by extension (lddecode.py:53-58, plus the u8 mapping of SURVEY F3)."""
    return EXT_TO_FMT.get(path.rsplit('.', 1)[-1].lower(), FMT_U8)


def bytes_for_samples(fmt, n):
    """Bytes holding samples [0, n) of a capture (whole packing groups)."""
    if fmt == FMT_U8:
        return n
    if fmt == FMT_S16:
        return 2 * n
    if fmt == FMT_R30:
        return ((n + 2) // 3) * 4
    return ((n + 3) // 4) * 5


def samples_in_bytes(fmt, nbytes):
    return {FMT_U8: nbytes, FMT_S16: nbytes // 2, FMT_R30: (nbytes // 4) * 3,
            FMT_LDS: (nbytes // 5) * 4}[fmt]


def pack_r30(samples10):
    """Three unsigned 10-bit samples per little-endian uint32, low bits first."""
    s = np.asarray(samples10, dtype=np.uint32)
    s = s[:(s.size // 3) * 3].reshape(-1, 3)
    w = (s[:, 0] & 0x3ff) | ((s[:, 1] & 0x3ff) << 10) | ((s[:, 2] & 0x3ff) << 20)
    return w.astype('<u4').tobytes()


def pack_lds(samples10):
    """Four 10-bit samples in five bytes, MSB-first bit stream."""
    s = np.asarray(samples10, dtype=np.uint16)
    s = s[:(s.size // 4) * 4].reshape(-1, 4)
    o = np.empty((s.shape[0], 5), dtype=np.uint8)
    o[:, 0] = s[:, 0] >> 2
    o[:, 1] = ((s[:, 0] & 0x3) << 6) | (s[:, 1] >> 4)
    o[:, 2] = ((s[:, 1] & 0xf) << 4) | (s[:, 2] >> 6)
    o[:, 3] = ((s[:, 2] & 0x3f) << 2) | (s[:, 3] >> 8)
    o[:, 4] = s[:, 3] & 0xff
    return o.tobytes()


def read_samples(buf, fmt, sample, count):
    """The loader plugin's ``loader(infile, sample, count)`` as int16 for a window
    inside the capture (lddutils.py:131-229; the CLI cut mode, lddecode.py:73-78).
    buf: the capture's bytes (ndarray of uint8, e.g. a np.memmap)."""
    sample, count = int(sample), int(count)
    if fmt == FMT_U8:
        return np.asarray(buf[sample:sample + count], dtype=np.int16)
    if fmt == FMT_S16:
        return np.frombuffer(bytes(buf[2 * sample:2 * (sample + count)]), dtype='<i2').copy()
    if fmt == FMT_R30:
        w0, off = sample // 3, sample % 3
        nw = (off + count + 2) // 3
        words = np.frombuffer(bytes(buf[4 * w0:4 * (w0 + nw)]), dtype='<u4')
        out = np.empty(words.size * 3, dtype=np.int16)
        out[0::3] = words & 0x3ff
        out[1::3] = (words >> 10) & 0x3ff
        out[2::3] = (words >> 20) & 0x3ff
        return out[off:off + count]
    g0, off = sample // 4, sample % 4
    ng = (off + count + 3) // 4
    b = np.frombuffer(bytes(buf[5 * g0:5 * (g0 + ng)]), dtype=np.uint8).astype(np.uint16).reshape(-1, 5)
    out = np.empty((b.shape[0], 4), dtype=np.int16)
    out[:, 0] = (b[:, 0] << 2) | (b[:, 1] >> 6)
    out[:, 1] = ((b[:, 1] & 0x3f) << 4) | (b[:, 2] >> 4)
    out[:, 2] = ((b[:, 2] & 0x0f) << 6) | (b[:, 3] >> 2)
    out[:, 3] = ((b[:, 3] & 0x03) << 8) | b[:, 4]
    return out.reshape(-1)[off:off + count]
