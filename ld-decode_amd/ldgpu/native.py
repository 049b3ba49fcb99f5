"""ctypes binding of libldgpu.so (include/ldgpu.h).

The library is built in-tree (``ld-decode_amd/ldgpu/libldgpu.so``) by
``__graft_entry__.build()``.  There is no CPU fallback: if the library or a
GPU is missing, ``load()`` / ``Context`` raise.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, 'libldgpu.so')

LDG_OK = 0
FS_VALID, FS_NO_VSYNC, FS_SHORT, FS_LINELOCS, FS_TBC, FS_EOF, FS_CRASH, FS_PENDING, FS_MIGRATED, FS_VCUT = range(10)
VBI_NONE = -2147483648
READ_FULL, READ_PROBE = 1, 2            # ldg_decode_reads_async2 per-read flags (include/ldgpu.h)
LOG_NO_VSYNC = 1 << 16            # ldg_field_info.log_flags (include/ldgpu.h)
MAX_VSYNCS = 16

EXPORTS = ['ldg_create', 'ldg_destroy', 'ldg_last_error', 'ldg_set_filters', 'ldg_set_capture',
           'ldg_decode_reads', 'ldg_field_audio', 'ldg_assemble_frames', 'ldg_debug_read',
           'ldg_comb_ntsc', 'ldg_comb_reset', 'ldg_version', 'ldg_device_count', 'ldg_profile_enable',
           'ldg_profile_read', 'ldg_synth_capture', 'ldg_capture_download', 'ldg_comb_ntsc_async', 'ldg_sync', 'ldg_demod_isolated', 'ldg_demod_isolated_ex', 'ldg_comb_set_opts', 'ldg_output_async', 'ldg_output_wait',
           'ldg_host_alloc', 'ldg_host_free',
           'ldg_archive_fields', 'ldg_archive_audio', 'ldg_decode_reads_async', 'ldg_decode_reads_async2',
           'ldg_set_video_cut', 'ldg_decode_reads_wait',
           'ldg_field_audio_async', 'ldg_field_audio_collect', 'ldg_comb_ntsc3d', 'ldg_cx_create', 'ldg_cx_destroy', 'ldg_cx_process', 'ldg_comb_pal', 'ldg_comb_set_state', 'ldg_profile_spans', 'ldg_profile_spans_union', 'ldg_profile_span_table',
           'ldg_audio_offsets', 'ldg_comb_async', 'ldg_debug_rf_table',
           'ldg_stream_open', 'ldg_stream_release', 'ldg_stream_seek', 'ldg_stream_window', 'ldg_stream_stats',
           'ldg_stream_close', 'ldg_device_memory']
STREAM_STATS = ('bytes_read', 'read_s', 'chunks', 'launch_waits', 'launch_wait_s', 'space_wait_s', 'seeks',
                'ring_bytes', 'chunk_bytes', 'stage_wait_s')     # ldg_stream_stats, in order


class FieldInfo(C.Structure):
    _fields_ = [('status', C.c_int32), ('npeaks', C.c_int32), ('nvsync', C.c_int32), ('istop', C.c_int32),
                ('linecount', C.c_int32), ('nlines', C.c_int32), ('n_out', C.c_int64),
                ('nextfieldoffset', C.c_int64), ('tbcstart', C.c_int64), ('med_hsync', C.c_double),
                ('hsync_tol', C.c_double), ('vsync', (C.c_int32 * 3) * MAX_VSYNCS),
                ('linecode', (C.c_int32 * 6) * 3), ('linecode_ok', C.c_int32 * 3),
                ('vbi_minutes', C.c_int32), ('vbi_seconds', C.c_int32), ('vbi_clvframe', C.c_int32),
                ('vbi_framenr', C.c_int32), ('vbi_status', C.c_int32), ('vbi_isclv', C.c_int32),
                ('burst_group', C.c_int32), ('log_flags', C.c_int32), ('pad_', C.c_int32),
                ('readsample', C.c_int64)]


class Config(C.Structure):
    _fields_ = [('system', C.c_int32), ('device', C.c_int32), ('max_reads', C.c_int32),
                ('max_frames', C.c_int32)]


class Params(C.Structure):
    _fields_ = [('freq_hz', C.c_double), ('freq', C.c_double), ('ire0', C.c_double), ('hz_ire', C.c_double),
                ('vsync_ire', C.c_double), ('sync_lo', C.c_double), ('sync_hi', C.c_double),
                ('freq_arf', C.c_double), ('audio_lowfreq', C.c_double), ('audio_lfreq', C.c_double),
                ('audio_rfreq', C.c_double), ('line_period', C.c_double), ('fsc_mhz', C.c_double),
                ('linelen', C.c_int32), ('outlinelen', C.c_int32), ('frame_lines', C.c_int32),
                ('audio_lo0', C.c_int32), ('codelines', C.c_int32 * 3), ('pad_', C.c_int32)]


class KernelStat(C.Structure):
    _fields_ = [('name', C.c_char * 48), ('launches', C.c_int64), ('total_ms', C.c_double)]


class SynthParams(C.Structure):
    _fields_ = [('fmt', C.c_int32), ('pad_', C.c_int32), ('nsamples', C.c_int64), ('seed', C.c_uint64),
                ('noise', C.c_double), ('start_line', C.c_double)]


_DP = C.POINTER(C.c_double)


class CombOpts(C.Structure):
    """ldg_comb_opts (include/ldgpu.h): comb-ntsc's command-line options."""
    _fields_ = [('black_ire', C.c_double), ('brightness', C.c_double), ('nr_y', C.c_double), ('nr_c', C.c_double),
                ('bw', C.c_int32), ('adaptive2d', C.c_int32), ('colorlpf', C.c_int32), ('colorlpf_hq', C.c_int32),
                ('linesout', C.c_int32), ('debug_line', C.c_int32), ('wide', C.c_int32),
                ('opticalflow', C.c_int32)]


COMB_DEFAULTS = dict(black_ire=7.5, brightness=236.0, nr_y=1.0, nr_c=0.0, bw=False, adaptive2d=True, colorlpf=True,
                     colorlpf_hq=True, linesout=480, debug_line=-1000, wide=False, opticalflow=False)


class Filters(C.Structure):
    _fields_ = [(k, _DP) for k in ('rfvideo', 'mtf', 'fvideo', 'fvideo05', 'fvideoburst', 'fvideopilot', 'fpsync',
                                   'audio_lfilt', 'audio_rfilt', 'audio_lpf2', 'mtf_logabs', 'mtf_arg', 'iir',
                                   'f05_fir')]


_lib = None


def lib_source_hash():
    """The source hash (build.py source_hash) of the loaded libldgpu.so: its build stamp, or
    None when the library carries none (a variant build loaded through LDGPU_LIB)."""
    lib = load()
    stamp = lib._name + '.sha256'
    return open(stamp).read().strip() if os.path.exists(stamp) else None


def load(path=None):
    """Load libldgpu.so and declare its signatures (no device access).
    LDGPU_LIB names another build of the same library (profiling variants)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get('LDGPU_LIB') or LIB_PATH
    if not os.path.exists(path):
        raise RuntimeError('libldgpu.so not built (%s); run __graft_entry__.build()' % path)
    lib = C.CDLL(path)
    vp = C.c_void_p
    lib.ldg_create.argtypes = [C.POINTER(Config), C.POINTER(vp)]
    lib.ldg_destroy.argtypes = [vp]
    lib.ldg_last_error.argtypes = [vp]
    lib.ldg_last_error.restype = C.c_char_p
    lib.ldg_set_filters.argtypes = [vp, C.POINTER(Params), C.POINTER(Filters)]
    lib.ldg_set_capture.argtypes = [vp, vp, C.c_int64, C.c_int, C.c_int64, C.c_int]
    lib.ldg_decode_reads.argtypes = [vp, C.c_int, C.POINTER(C.c_int64), C.POINTER(C.c_double),
                                     C.POINTER(C.c_int32), C.POINTER(FieldInfo)]
    lib.ldg_field_audio.argtypes = [vp, C.c_int, C.POINTER(C.c_int32), C.POINTER(C.c_double),
                                    C.POINTER(C.c_int16), C.c_int64, C.POINTER(C.c_int32), C.POINTER(C.c_double)]
    lib.ldg_field_audio_async.argtypes = [vp, C.c_int, vp, vp]
    lib.ldg_field_audio_collect.argtypes = [vp, vp, C.c_int64, vp, vp]
    lib.ldg_assemble_frames.argtypes = [vp, C.c_int, C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                        C.POINTER(C.c_uint16), C.c_int]
    lib.ldg_debug_read.argtypes = [vp, C.c_int, C.c_int, vp, C.c_int64]
    lib.ldg_debug_read.restype = C.c_int64
    lib.ldg_debug_rf_table.argtypes = [vp, C.c_double, vp]
    lib.ldg_comb_ntsc.argtypes = [vp, C.c_int, vp, vp, C.c_int]
    lib.ldg_comb_reset.argtypes = [vp]
    lib.ldg_comb_set_opts.argtypes = [vp, C.POINTER(CombOpts)]
    lib.ldg_output_async.argtypes = [vp, C.c_int, vp, vp, vp, vp]
    lib.ldg_output_wait.argtypes = [vp]
    lib.ldg_host_alloc.argtypes = [C.c_int64, C.POINTER(vp)]
    lib.ldg_host_free.argtypes = [vp]
    lib.ldg_comb_ntsc_async.argtypes = [vp, C.c_int]
    lib.ldg_comb_async.argtypes = [vp, C.c_int]
    lib.ldg_comb_ntsc3d.argtypes = [vp, C.c_int, vp, vp, C.POINTER(C.c_int), C.c_double, C.c_double]
    lib.ldg_decode_reads_async.argtypes = [vp, C.c_int, vp, vp, vp]
    lib.ldg_decode_reads_async2.argtypes = [vp, C.c_int, vp, vp, vp, vp]
    lib.ldg_set_video_cut.argtypes = [vp, C.c_int64]
    lib.ldg_decode_reads_wait.argtypes = [vp, vp]
    lib.ldg_archive_fields.argtypes = [vp, C.c_int, vp, C.c_int64]
    lib.ldg_archive_audio.argtypes = [vp, C.c_int, vp, vp, vp, C.c_int64, vp, vp]
    lib.ldg_sync.argtypes = [vp]
    lib.ldg_demod_isolated.argtypes = [vp, C.c_int, vp, C.c_int, C.POINTER(C.c_double)]
    lib.ldg_demod_isolated_ex.argtypes = [vp, C.c_int, vp, C.c_int, C.c_int, C.POINTER(C.c_double)]
    lib.ldg_profile_enable.argtypes = [vp, C.c_int]
    lib.ldg_profile_read.argtypes = [vp, C.POINTER(KernelStat), C.c_int]
    lib.ldg_profile_spans.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_int64)]
    lib.ldg_profile_spans_union.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_int64)]
    lib.ldg_profile_span_table.argtypes = [vp, vp, C.c_int]
    lib.ldg_synth_capture.argtypes = [vp, C.POINTER(SynthParams), C.POINTER(C.c_double), C.POINTER(C.c_double),
                                      C.POINTER(C.c_uint32), C.c_int64]
    lib.ldg_capture_download.argtypes = [vp, vp, C.c_int64, C.c_int64]
    lib.ldg_capture_download.restype = C.c_int64
    lib.ldg_comb_pal.argtypes = [vp, C.c_int, vp, vp]
    lib.ldg_comb_set_state.argtypes = [vp, C.c_double]
    lib.ldg_cx_create.argtypes = [C.POINTER(vp)]
    lib.ldg_cx_destroy.argtypes = [vp]
    lib.ldg_cx_process.argtypes = [vp, C.c_int64, vp, vp]
    lib.ldg_audio_offsets.argtypes = [C.c_double, C.c_int64, vp, C.c_double, vp]
    lib.ldg_stream_open.argtypes = [vp, C.c_char_p, C.c_int, C.c_int64, C.c_int64]
    lib.ldg_stream_release.argtypes = [vp, C.c_int64]
    lib.ldg_stream_seek.argtypes = [vp, C.c_int64]
    lib.ldg_stream_window.argtypes = [vp, vp]
    lib.ldg_stream_stats.argtypes = [vp, vp, C.c_int]
    lib.ldg_stream_close.argtypes = [vp]
    lib.ldg_device_memory.argtypes = [C.c_int, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    lib.ldg_version.restype = C.c_char_p
    lib.ldg_device_count.restype = C.c_int
    _lib = lib
    return lib


def device_memory(device=0):
    """(free, total) bytes of device memory (ldg_device_memory)."""
    f, t = C.c_int64(), C.c_int64()
    rc = load().ldg_device_memory(int(device), C.byref(f), C.byref(t))
    if rc != LDG_OK:
        raise LDGError('ldg_device_memory failed (%d)' % rc)
    return f.value, t.value


def _ptr(a, t=C.c_double):
    return a.ctypes.data_as(C.POINTER(t))


class LDGError(RuntimeError):
    pass


class PinnedBuffer:
    """Page-locked host memory (ldg_host_alloc) viewed as a numpy uint16 array; grows on
    demand.  A grown buffer keeps its old allocation alive (retired) until
    release_retired(): a view handed to a sink before the growth stays valid until the
    owner says the views are dead (GPUDecoder.decode: at its end)."""

    def __init__(self):
        self.lib = load()
        self.ptr, self.nbytes, self.arr = None, 0, None
        self.retired = []

    def view(self, count):
        nbytes = max(2 * count, 2)
        if nbytes > self.nbytes:
            if self.ptr is not None:
                self.retired.append(self.ptr)
            self.ptr, self.nbytes, self.arr = None, 0, None
            p = C.c_void_p()
            if self.lib.ldg_host_alloc(nbytes, C.byref(p)) != LDG_OK:
                raise LDGError('ldg_host_alloc(%d) failed' % nbytes)
            self.ptr, self.nbytes = p, nbytes
            self.arr = np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint16)), shape=(nbytes // 2,))
        return self.arr[:count]

    def release_retired(self):
        for p in self.retired:
            self.lib.ldg_host_free(p)
        self.retired = []

    def free(self):
        self.release_retired()
        if self.ptr is not None:
            self.lib.ldg_host_free(self.ptr)
            self.ptr, self.nbytes, self.arr = None, 0, None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Context:
    """One libldgpu context (one GPU).  Owns device memory for ``max_reads`` field reads."""

    def __init__(self, system='NTSC', device=0, max_reads=32, max_frames=None):
        self.lib = load()
        if self.lib.ldg_device_count() <= 0:
            raise LDGError('no HIP device visible: the ldgpu decode path needs an MI355X (no CPU fallback)')
        cfg = Config(1 if system == 'PAL' else 0, device, max_reads, max_frames or max_reads)
        h = C.c_void_p()
        rc = self.lib.ldg_create(C.byref(cfg), C.byref(h))
        if rc != LDG_OK:
            raise LDGError('ldg_create failed (%d)' % rc)
        self.h = h
        self.system = system
        self.max_reads = max_reads
        self.max_frames = max_frames or max_reads
        self._keep = []
        self._pending = []          # read counts of the outstanding ldg_decode_reads_async calls

    def _check(self, rc, what):
        if rc != LDG_OK:
            raise LDGError('%s failed (%d): %s' % (what, rc, self.lib.ldg_last_error(self.h).decode()))

    def close(self):
        if self.h:
            self.lib.ldg_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_filters(self, params, tables):
        """params: dict of ldg_params fields; tables: dict name -> complex128/float64 array."""
        p = Params()
        for k, _ in Params._fields_:
            if k == 'codelines':
                for i, v in enumerate(params['codelines']):
                    p.codelines[i] = int(v)
            elif k != 'pad_':
                setattr(p, k, params[k])
        keep = {}
        f = Filters()
        for k, _ in Filters._fields_:
            a = tables.get(k)
            if a is None:
                setattr(f, k, C.POINTER(C.c_double)())
                continue
            if np.iscomplexobj(a):
                a = np.ascontiguousarray(a, dtype=np.complex128).view(np.float64)
            else:
                a = np.ascontiguousarray(a, dtype=np.float64)
            keep[k] = a
            setattr(f, k, _ptr(a))
        self._check(self.lib.ldg_set_filters(self.h, C.byref(p), C.byref(f)), 'ldg_set_filters')
        self.params = params

    def set_capture(self, raw, nsamples, fmt, first_sample=0, device_ptr=None):
        if device_ptr is not None:
            rc = self.lib.ldg_set_capture(self.h, C.c_void_p(device_ptr), nsamples, fmt, first_sample, 1)
        else:
            buf = np.frombuffer(raw, dtype=np.uint8) if not isinstance(raw, np.ndarray) else raw.view(np.uint8)
            buf = np.ascontiguousarray(buf)
            rc = self.lib.ldg_set_capture(self.h, buf.ctypes.data_as(C.c_void_p), nsamples, fmt, first_sample, 0)
        self._check(rc, 'ldg_set_capture')

    # ---- streamed capture (ldg_stream_*) -------------------------------------------
    def stream_open(self, path, fmt, ring_bytes, first_sample=0):
        """Stream the capture file at `path` through an HBM ring of ring_bytes (see
        include/ldgpu.h); replaces any resident capture."""
        self._check(self.lib.ldg_stream_open(self.h, os.fsencode(path), int(fmt), int(ring_bytes), int(first_sample)),
                    'ldg_stream_open')

    def stream_release(self, below_sample):
        self._check(self.lib.ldg_stream_release(self.h, int(below_sample)), 'ldg_stream_release')

    def stream_seek(self, first_sample):
        self._check(self.lib.ldg_stream_seek(self.h, int(first_sample)), 'ldg_stream_seek')

    def stream_window(self):
        """(lowest readable sample, highest block end a launch may reach, samples read so far,
        total samples)"""
        out = np.zeros(4, dtype=np.int64)
        self._check(self.lib.ldg_stream_window(self.h, out.ctypes.data), 'ldg_stream_window')
        return tuple(int(x) for x in out)

    def stream_stats(self):
        out = np.zeros(len(STREAM_STATS), dtype=np.float64)
        n = self.lib.ldg_stream_stats(self.h, out.ctypes.data, out.size)
        if n < 0:
            self._check(n, 'ldg_stream_stats')
        return dict(zip(STREAM_STATS[:n], (float(x) for x in out[:n])))

    def stream_close(self):
        self._check(self.lib.ldg_stream_close(self.h), 'ldg_stream_close')

    def decode_reads(self, starts, mtfs, slots=None):
        n = len(starts)
        s = np.ascontiguousarray(starts, dtype=np.int64)
        m = np.ascontiguousarray(mtfs, dtype=np.float64)
        sl = np.ascontiguousarray(slots if slots is not None else np.arange(n), dtype=np.int32)
        info = (FieldInfo * n)()
        self._check(self.lib.ldg_decode_reads(self.h, n, _ptr(s, C.c_int64), _ptr(m), _ptr(sl, C.c_int32), info),
                    'ldg_decode_reads')
        out = list(info)
        for _ in range(3):
            # a read whose odd-half park another demod workgroup overwrote (FS_MIGRATED) is void: decode it again
            redo = [i for i, x in enumerate(out) if x.status == FS_MIGRATED]
            if not redo:
                break
            again = self.decode_reads(s[redo], m[redo], sl[redo])
            for i, x in zip(redo, again):
                out[i] = x
        return out

    def decode_reads_async(self, starts, mtfs, slots, full=None):
        """Launch a decode (ldg_decode_reads_async2, up to 8 outstanding); decode_reads_wait()
        returns the records of the oldest outstanding one.  full: per read flags, READ_FULL
        (or True) exempts it from the video cut (set_video_cut; reads that came back FS_VCUT),
        READ_PROBE moves a predicted start to the sync peak a probe finds (the record's
        readsample is the start decoded).  Returns the flags as the library left them
        (READ_PROBE set exactly for the reads probed), or None."""
        s, m, sl = (np.ascontiguousarray(starts, dtype=np.int64), np.ascontiguousarray(mtfs, dtype=np.float64),
                    np.ascontiguousarray(slots, dtype=np.int32))
        f = None if full is None else np.ascontiguousarray(full, dtype=np.uint8)
        self._check(self.lib.ldg_decode_reads_async2(self.h, s.size, s.ctypes.data, m.ctypes.data, sl.ctypes.data,
                                                     None if f is None else f.ctypes.data),
                    'ldg_decode_reads_async2')
        self._pending.append(s.size)
        return f

    def set_video_cut(self, out_samples):
        """The demod skips the video / burst / pilot channels of blocks whose outputs start at
        or past out_samples (0: no cut); a field that needs them comes back FS_VCUT."""
        self._check(self.lib.ldg_set_video_cut(self.h, int(out_samples)), 'ldg_set_video_cut')

    def decode_reads_wait(self):
        n = self._pending[0]
        info = (FieldInfo * n)()
        self._check(self.lib.ldg_decode_reads_wait(self.h, info), 'ldg_decode_reads_wait')
        self._pending.pop(0)
        return list(info)

    def field_audio(self, slots, offsets):
        n = len(slots)
        stride = 2048
        pcm = np.zeros((max(n, 1), stride), dtype=np.int16)
        counts = np.zeros(max(n, 1), dtype=np.int32)
        nxt = np.zeros(max(n, 1), dtype=np.float64)
        sl = np.ascontiguousarray(slots, dtype=np.int32)
        of = np.ascontiguousarray(offsets, dtype=np.float64)
        self._check(self.lib.ldg_field_audio(self.h, n, _ptr(sl, C.c_int32), _ptr(of), _ptr(pcm, C.c_int16), stride,
                                             _ptr(counts, C.c_int32), _ptr(nxt)), 'ldg_field_audio')
        return pcm[:n], counts[:n], nxt[:n]

    def field_audio_async(self, slots, offsets):
        """Launch ldg_field_audio_async; field_audio_collect() returns what field_audio would."""
        sl = np.ascontiguousarray(slots, dtype=np.int32)
        of = np.ascontiguousarray(offsets, dtype=np.float64)
        self._check(self.lib.ldg_field_audio_async(self.h, sl.size, sl.ctypes.data, of.ctypes.data),
                    'ldg_field_audio_async')
        self._audio_n = sl.size

    def field_audio_collect(self):
        n = self._audio_n
        stride = 2048
        pcm = np.zeros((max(n, 1), stride), dtype=np.int16)
        counts = np.zeros(max(n, 1), dtype=np.int32)
        nxt = np.zeros(max(n, 1), dtype=np.float64)
        self._check(self.lib.ldg_field_audio_collect(self.h, pcm.ctypes.data, stride, counts.ctypes.data,
                                                     nxt.ctypes.data), 'ldg_field_audio_collect')
        return pcm[:n], counts[:n], nxt[:n]

    def archive_fields(self, slots, first):
        sl = np.ascontiguousarray(slots, dtype=np.int32)
        self._check(self.lib.ldg_archive_fields(self.h, sl.size, sl.ctypes.data, int(first)), 'ldg_archive_fields')

    def archive_audio(self, entries, offsets, packed=False):
        """ldg_field_audio over archive entries -> (pcm[n, 2048], counts, next offsets); packed:
        pcm is one flat array, the fields' 2 * counts samples one after another."""
        n = len(entries)
        stride = 0 if packed else 2048
        pcm = np.empty(max(n, 1) * 2048, dtype=np.int16) if packed else np.zeros((max(n, 1), stride), dtype=np.int16)
        counts = np.zeros(max(n, 1), dtype=np.int32)
        nxt = np.zeros(max(n, 1), dtype=np.float64)
        e = np.ascontiguousarray(entries, dtype=np.int64)
        o = np.ascontiguousarray(offsets, dtype=np.float64)
        self._check(self.lib.ldg_archive_audio(self.h, n, e.ctypes.data, o.ctypes.data, pcm.ctypes.data, stride,
                                               counts.ctypes.data, nxt.ctypes.data), 'ldg_archive_audio')
        if packed:
            return pcm[:int(2 * np.maximum(counts[:n], 0).sum())], counts[:n], nxt[:n]
        return pcm[:n], counts[:n], nxt[:n]

    def assemble_frames_device(self, tops, bottoms):
        """Assemble frames into the context's device frame buffer (no host copy)."""
        n = len(tops)
        t = np.ascontiguousarray(tops, dtype=np.int32)
        b = np.ascontiguousarray(bottoms, dtype=np.int32)
        self._check(self.lib.ldg_assemble_frames(self.h, n, _ptr(t, C.c_int32), _ptr(b, C.c_int32),
                                                 C.POINTER(C.c_uint16)(), 1), 'ldg_assemble_frames')

    def assemble_frames(self, tops, bottoms, W, H):
        n = len(tops)
        out = np.zeros((max(n, 1), H * W), dtype=np.uint16)
        t = np.ascontiguousarray(tops, dtype=np.int32)
        b = np.ascontiguousarray(bottoms, dtype=np.int32)
        self._check(self.lib.ldg_assemble_frames(self.h, n, _ptr(t, C.c_int32), _ptr(b, C.c_int32),
                                                 _ptr(out, C.c_uint16), 0), 'ldg_assemble_frames')
        return out[:n]

    def debug(self, slot, what, dtype, count):
        a = np.zeros(count, dtype=dtype)
        rc = self.lib.ldg_debug_read(self.h, slot, what, a.ctypes.data_as(C.c_void_p), a.nbytes)
        if rc < 0:
            raise LDGError('ldg_debug_read(%d,%d) -> %d' % (slot, what, rc))
        return a[:rc // a.itemsize]

    def rf_table(self, mtf):
        """The demod's RF filter RFVideo * MTF**mtf (complex128[16384], natural bin order)."""
        a = np.zeros(2 * 16384, dtype=np.float64)
        rc = self.lib.ldg_debug_rf_table(self.h, float(mtf), a.ctypes.data_as(C.c_void_p))
        if rc != LDG_OK:
            raise LDGError('ldg_debug_rf_table(%r) -> %d' % (mtf, rc))
        return a.view(np.complex128)

    def comb_ntsc(self, frames):
        """2D NTSC comb (comb-ntsc.cxx dim=2): n x (525, 910) uint16 frames -> n x (480, 744, 3) rgb48
        (comb_lines x comb_width with -v / -W).  State (burst-level EMA, -W's Y-NR history)
        carries across calls like one reference comb process."""
        f = np.ascontiguousarray(frames, dtype=np.uint16).reshape(-1, 525 * 910)
        out = np.zeros((f.shape[0], self.comb_lines, self.comb_width, 3), dtype=np.uint16)
        self._check(self.lib.ldg_comb_ntsc(self.h, f.shape[0], f.ctypes.data_as(C.c_void_p),
                                           out.ctypes.data_as(C.c_void_p), 0), 'ldg_comb_ntsc')
        return out

    def comb_ntsc3d(self, frames, core_ire=-1.0, range_ire=-1.0):
        """3D NTSC comb, comb-ntsc -d 3 -F (or, after comb_set_opts(opticalflow=True), -d 3 with
        the build-defined optical flow): n x (525, 910) uint16 frames in, the rgb48 frames that
        now have both neighbours out (none for a process's first two frames)."""
        f = np.ascontiguousarray(frames, dtype=np.uint16).reshape(-1, 525 * 910)
        out = np.zeros((f.shape[0], self.comb_lines, self.comb_width, 3), dtype=np.uint16)
        n_out = C.c_int(0)
        self._check(self.lib.ldg_comb_ntsc3d(self.h, f.shape[0], f.ctypes.data_as(C.c_void_p),
                                             out.ctypes.data_as(C.c_void_p), C.byref(n_out), core_ire, range_ire),
                    'ldg_comb_ntsc3d')
        return out[:n_out.value]

    def comb_pal(self, frames):
        """PAL Y/C decoder (build-defined, see include/ldgpu.h): n x (625, 1135) uint16 frames ->
        n x (576, 1057, 3) rgb48."""
        f = np.ascontiguousarray(frames, dtype=np.uint16).reshape(-1, 625 * 1135)
        out = np.zeros((f.shape[0], 576, 1057, 3), dtype=np.uint16)
        self._check(self.lib.ldg_comb_pal(self.h, f.shape[0], f.ctypes.data_as(C.c_void_p),
                                          out.ctypes.data_as(C.c_void_p)), 'ldg_comb_pal')
        return out

    def comb_ntsc_device(self, n):
        """Comb the first n frames of the context's device frame buffer (ldg_assemble_frames
        with out=NULL) into the context's device rgb buffer (benchmark mode)."""
        self._check(self.lib.ldg_comb_ntsc(self.h, n, None, None, 1), 'ldg_comb_ntsc')

    def comb_ntsc_async(self, n):
        """ldg_comb_ntsc_async: comb the context's first n device frames on the comb stream."""
        self._check(self.lib.ldg_comb_ntsc_async(self.h, n), 'ldg_comb_ntsc_async')

    def comb_async(self, n):
        """ldg_comb_async: the context's system's comb (NTSC 2D, or the PAL Y/C decoder) over
        its first n device frames, on the comb stream."""
        self._check(self.lib.ldg_comb_async(self.h, n), 'ldg_comb_async')

    def demod_isolated(self, slots, iters, variant=0):
        """Mean HIP-event ms of one demod-only launch over these live slots: variant 0
        ldg_k_demod_iso (every block in full), 1 ldg_k_demod_iso_cut (the shipped body)."""
        sl = np.ascontiguousarray(slots, dtype=np.int32)
        ms = C.c_double()
        self._check(self.lib.ldg_demod_isolated_ex(self.h, sl.size, sl.ctypes.data, iters, variant, C.byref(ms)),
                    'ldg_demod_isolated_ex')
        return ms.value

    def output_async(self, tops, bottoms, tbc, rgb=None):
        """ldg_output_async: frames (and the 2D comb's rgb48 when rgb is given) into the host
        arrays `tbc` / `rgb` (pinned: PinnedBuffer views) on the output stream; returns at once,
        output_wait() waits for the copies."""
        n = len(tops)
        t = np.ascontiguousarray(tops, dtype=np.int32)
        b = np.ascontiguousarray(bottoms, dtype=np.int32)
        self._out_keep = (t, b)
        self._check(self.lib.ldg_output_async(self.h, n, t.ctypes.data, b.ctypes.data, tbc.ctypes.data,
                                              rgb.ctypes.data if rgb is not None else None), 'ldg_output_async')

    def output_wait(self):
        self._check(self.lib.ldg_output_wait(self.h), 'ldg_output_wait')

    def sync(self):
        self._check(self.lib.ldg_sync(self.h), 'ldg_sync')

    def comb_set_state(self, aburstlev):
        self._check(self.lib.ldg_comb_set_state(self.h, float(aburstlev)), 'ldg_comb_set_state')

    comb_lines = 480                 # rows per rgb48 frame (comb-ntsc -v: 525)
    comb_width = 744                 # pixels per rgb48 row (comb-ntsc -W: 910)

    def comb_set_opts(self, **opts):
        """comb-ntsc's options (ldg_comb_set_opts; keys of COMB_DEFAULTS, values as on the
        reference's command line); no arguments restores the defaults."""
        o = dict(COMB_DEFAULTS)
        for k, v in opts.items():
            if k not in o:
                raise TypeError('unknown comb option %s' % k)
            o[k] = v
        c = CombOpts(**{k: (int(v) if isinstance(v, bool) else v) for k, v in o.items()})
        self._check(self.lib.ldg_comb_set_opts(self.h, C.byref(c)), 'ldg_comb_set_opts')
        self.comb_lines = int(o['linesout'])
        self.comb_width = 910 if o['wide'] else 744

    def comb_reset(self):
        self._check(self.lib.ldg_comb_reset(self.h), 'ldg_comb_reset')

    # ---- profiling / tooling -------------------------------------------------------
    def profile(self, on=True):
        """on: True (every kernel), 'demod' (the demod only), False."""
        mode = 2 if on == 'demod' else (1 if on else 0)
        self._check(self.lib.ldg_profile_enable(self.h, mode), 'ldg_profile_enable')

    def profile_spans(self):
        """(count, total ms) of the demod launches' execution spans since profile(on)."""
        t, n = C.c_double(0), C.c_int64(0)
        self._check(self.lib.ldg_profile_spans(self.h, C.byref(t), C.byref(n)), 'ldg_profile_spans')
        return int(n.value), float(t.value)

    def profile_spans_union(self):
        """(count, ms) of demod launches and the time at least one of them was executing."""
        t, n = C.c_double(0), C.c_int64(0)
        self._check(self.lib.ldg_profile_spans_union(self.h, C.byref(t), C.byref(n)), 'ldg_profile_spans_union')
        return int(n.value), float(t.value)

    def profile_span_table(self):
        """float64[n, 4]: every profiled demod launch in issue order -- execution start, end
        and host issue time, ms on the device clock from the first start, and the issue time
        in ms of the host's monotonic clock (time.perf_counter() * 1e3; ldg_profile_span_table)."""
        out = np.zeros((8192, 4), dtype=np.float64)
        n = self.lib.ldg_profile_span_table(self.h, out.ctypes.data, out.shape[0])
        if n < 0:
            self._check(n, 'ldg_profile_span_table')
        return out[:n]

    def profile_stats(self):
        arr = (KernelStat * 64)()
        n = self.lib.ldg_profile_read(self.h, arr, 64)
        return {arr[i].name.decode(): (int(arr[i].launches), float(arr[i].total_ms)) for i in range(min(n, 64))}

    def synth(self, nsamples, fmt=0, first_frame=1, clv=False, seed=20181015, noise=0.02, start_line=100,
              start_sample=0):
        """Generate a synthetic NTSC capture straight into this context's HBM capture buffer.
        start_sample: generate samples [start_sample, start_sample + nsamples) of the capture
        (a shard's window; line timing and frame codes follow the whole capture's)."""
        import scipy.signal as sps
        from .synth import NTSC, FrameCodes, emphasis_filter, FS
        fir = np.ascontiguousarray(sps.firwin(63, 4.4e6 / (FS / 2)), dtype=np.float64)
        b, a = emphasis_filter(NTSC)
        emph = np.array([b[0], b[1], a[1]], dtype=np.float64)
        spl = FS * NTSC['line_us'] / 1e6
        start_line = start_line + start_sample / spl
        nframes = int((nsamples / spl + start_line) // 525) + 2
        fc = FrameCodes(first_frame, clv, 30)
        codes = np.array([fc.codes(k) for k in range(nframes)], dtype=np.uint32).reshape(-1)
        p = SynthParams(fmt, 0, nsamples, seed, noise, start_line)
        self._check(self.lib.ldg_synth_capture(self.h, C.byref(p), _ptr(fir), _ptr(emph), _ptr(codes, C.c_uint32),
                                               nframes), 'ldg_synth_capture')

    def capture_copy_to_device(self, dst_ptr, offset, nbytes):
        """Copy resident capture bytes into a device buffer (e.g. a torch CUDA tensor)."""
        n = self.lib.ldg_capture_download(self.h, C.c_void_p(dst_ptr), offset, nbytes)
        if n != nbytes:
            raise LDGError('ldg_capture_download -> %d' % n)

    def capture_download(self, offset, nbytes):
        a = np.zeros(nbytes, dtype=np.uint8)
        n = self.lib.ldg_capture_download(self.h, a.ctypes.data_as(C.c_void_p), offset, nbytes)
        if n < 0:
            raise LDGError('ldg_capture_download -> %d' % n)
        return a[:n]


def audio_offsets(o0, linecounts, line_period):
    """ldg_audio_offsets: [o0, o1, ..., on] of downscale_audio's 48 kHz offset chain over
    the fields' line counts (host code in the library, no device needed)."""
    lc = np.ascontiguousarray(linecounts, dtype=np.float64)
    out = np.zeros(lc.size + 1, dtype=np.float64)
    rc = load().ldg_audio_offsets(float(o0), lc.size, lc.ctypes.data, float(line_period), out.ctypes.data)
    if rc != 0:
        raise IndexError('downscale_audio: empty tick range (the reference raises here)')
    return out.tolist()


class CXExpander:
    """cx-expander (cx-expander.cxx:34-92) through ldg_cx_process: host code, no device needed.
    State carries across process() calls like one cx process."""

    def __init__(self):
        self.lib = load()
        h = C.c_void_p()
        if self.lib.ldg_cx_create(C.byref(h)) != LDG_OK:
            raise LDGError('ldg_cx_create failed')
        self.h = h

    def process(self, stereo_u16):
        """(n, 2) or flat interleaved uint16 -> (n, 2) uint16."""
        a = np.ascontiguousarray(stereo_u16, dtype=np.uint16).reshape(-1, 2)
        out = np.empty_like(a)
        if self.lib.ldg_cx_process(self.h, a.shape[0], a.ctypes.data, out.ctypes.data) != LDG_OK:
            raise LDGError('ldg_cx_process failed')
        return out

    def __del__(self):
        if getattr(self, 'h', None):
            self.lib.ldg_cx_destroy(self.h)
            self.h = None
