/*
 * libldgpu -- MI355X (gfx950) LaserDisc RF -> .tbc decode: public C ABI.
 *
 * Plain C, plain pointers and sizes; no C++ or torch types cross this boundary.
 * Every entry point returns an int status (LDG_OK == 0) and never throws.
 *
 * The ABI is the seam a drop-in replaces in the reference ld-decode snapshot:
 *
 *   reference seam (file:line)                          replaced by
 *   ---------------------------------------------------  --------------------------------
 *   loader plugin  loader(infile, sample, readlen)      ldg_set_capture (GPU unpack of
 *     lddutils.py:117-229, set lddecode.py:53-58          u8 / s16 / .r30 / .lds)
 *   RFDecode(system) filter build                       ldg_create + ldg_set_filters
 *     lddecode_core.py:119-279
 *   RFDecode.demod(infile, start, 1e6, mtf)             ldg_decode_reads (demod part)
 *     lddecode_core.py:373-427
 *   FieldNTSC/FieldPAL(rf, rawdecode, 0, ...)           ldg_decode_reads (field part):
 *     lddecode_core.py:889-1191                            per read -> ldg_field_info +
 *                                                          device-resident dspicture
 *   Field.downscale(audio) -> downscale_audio           ldg_field_audio
 *     lddecode_core.py:431-484, 809-810
 *   Framer.formatoutput(fields)                         ldg_assemble_frames
 *     lddecode_core.py:1238-1252
 *   comb-ntsc stdin/stdout frame stream, dim=2          ldg_comb_ntsc
 *     comb-ntsc.cxx:834-892, 1099-1117
 *   PAL Y/C (build-defined adaptation of                 ldg_comb_pal
 *     attic2/comb-pal.cxx:234-654, 820-917)
 *   cx-expander stdin/stdout (.pcm post-chain)          ldg_cx_process
 *     cx-expander.cxx:34-117
 *   comb-ntsc -d 3 -F [-c core] [-r range] (3D, no      ldg_comb_ntsc3d
 *     optical flow) comb-ntsc.cxx:369-412, 834-892, 983-993, 1077-1082
 *
 * The Python host (ld-decode_amd/ldgpu) keeps readfield/readframe/mergevbi,
 * the read-position / MTF / audio-offset chains and the file writers, and
 * calls these through ctypes.
 */
#ifndef LDGPU_H
#define LDGPU_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LDG_OK 0
#define LDG_EINVAL (-1)
#define LDG_EDEVICE (-2)
#define LDG_ENOMEM (-3)
#define LDG_ESTATE (-4)

#define LDG_SYSTEM_NTSC 0
#define LDG_SYSTEM_PAL 1

#define LDG_FMT_U8 0  /* unsigned 8-bit (cxadc)                 lddutils.py:143-144 */
#define LDG_FMT_S16 1 /* signed 16-bit LE (.r16)                lddutils.py:146-147 */
#define LDG_FMT_R30 2 /* 3 x 10-bit per LE uint32 (ddpack)      lddutils.py:150-173 */
#define LDG_FMT_LDS 3 /* 4 x 10-bit per 5 bytes (DD .lds)       lddutils.py:195-229 */

/* Per-read field status: why a Field is (not) valid. */
#define LDG_FS_VALID 0    /* Field.valid == True                                  */
#define LDG_FS_NO_VSYNC 1 /* len(vsyncs) == 0            lddecode_core.py:909-912 */
#define LDG_FS_SHORT 2    /* 1 vsync / too few peaks      lddecode_core.py:913-924 */
#define LDG_FS_LINELOCS 3 /* 'unable to decode frame'     lddecode_core.py:935-941 */
#define LDG_FS_TBC 4      /* 'Unable to decode frame, skipping' :1043-1048,1178-1191 */
#define LDG_FS_EOF 5      /* a block of the read lies beyond the capture window    */
#define LDG_FS_CRASH 6    /* the reference raises uncaught here (documented)       */
#define LDG_FS_PENDING 7  /* internal                                               */
#define LDG_FS_MIGRATED 8 /* the read's per-CU odd-half park was overwritten between its
                           * store and its reload (another demod workgroup ran on the CU
                           * while this one was switched out: compute-wave save/restore
                           * on a shared GPU): its result is void, decode the read again */
#define LDG_FS_VCUT 9     /* a field kernel needed the video channel past the read's video
                           * cut (ldg_set_video_cut): its result is void, decode the read
                           * again in full (ldg_decode_reads_async2, full[i] = 1)          */

#define LDG_VBI_NONE (-2147483647 - 1) /* Python None in Field.vbi */

#define LDG_MAX_VSYNCS 16

/* Everything the host needs from one Field, lddecode_core.py:889-957,1165-1191. */
typedef struct ldg_field_info {
  int32_t status;       /* LDG_FS_*                                   */
  int32_t npeaks;       /* len(Field.peaklist)                        */
  int32_t nvsync;       /* len(Field.vsyncs)                          */
  int32_t istop;        /* Field.istop                                */
  int32_t linecount;    /* Field.linecount (262/263, 312/313)         */
  int32_t nlines;       /* len(Field.linelocs) = linecount + 4        */
  int64_t n_out;        /* demod samples in this read                 */
  int64_t nextfieldoffset; /* Field.nextfieldoffset (relative to the read's block start) */
  int64_t tbcstart;     /* Field.tbcstart                             */
  double med_hsync;     /* Field.med_hsync                            */
  double hsync_tol;     /* Field.hsync_tolerance                      */
  int32_t vsync[LDG_MAX_VSYNCS][3]; /* Field.vsyncs rows (peak idx, line0, istop/vote) */
  int32_t linecode[3][6];           /* Field.linecode[philips_codelines[i]] nibbles     */
  int32_t linecode_ok[3];           /* 1 = decoded, 0 = None                            */
  int32_t vbi_minutes, vbi_seconds, vbi_clvframe, vbi_framenr, vbi_status, vbi_isclv;
  int32_t burst_group;  /* NTSC burst phase group of the final refine pass */
  int32_t log_flags;    /* what the reference prints while building this Field:
                         * bit q (q < 16): "vsync vote needed q"    lddecode_core.py:620
                         * LDG_LOG_NO_VSYNC: "no/corrupt VSYNC found, jumping forward"  :918 */
  int32_t pad_;
  int64_t readsample;   /* the read's start: the requested one, or where a start probe moved it
                         * (ldg_decode_reads_async2, LDG_READ_PROBE) */
} ldg_field_info;

#define LDG_LOG_NO_VSYNC (1 << 16)

typedef struct ldg_ctx ldg_ctx;

typedef struct ldg_config {
  int32_t system;    /* LDG_SYSTEM_NTSC / LDG_SYSTEM_PAL      */
  int32_t device;    /* HIP device ordinal                     */
  int32_t max_reads; /* device read slots (and max reads per ldg_decode_reads call) */
  int32_t max_frames;/* frames per ldg_assemble_frames call    */
} ldg_config;

/* Scalars of the filter set / system constants (lddecode_core.py:30-117,119-279). */
typedef struct ldg_params {
  double freq_hz, freq, ire0, hz_ire, vsync_ire;
  double sync_lo, sync_hi; /* iretohz(-55), iretohz(-25) */
  double freq_arf, audio_lowfreq, audio_lfreq, audio_rfreq;
  double line_period, fsc_mhz;
  int32_t linelen, outlinelen, frame_lines, audio_lo0;
  int32_t codelines[3];
  int32_t pad_;
} ldg_params;

/* Filter tables, complex128 interleaved (re, im):
 *   rfvideo[16384], mtf[16384], fvideo[16384], fvideo05[16384], fvideoburst[16384],
 *   fvideopilot[16384] (PAL; may be NULL for NTSC), fpsync[16384],
 *   audio_lfilt[1024], audio_rfilt[1024], audio_lpf2[4096];
 * (fvideoburst, fvideopilot and fpsync are checked against `iir`, not used per sample)
 * real float64: mtf_logabs[16384] = log|MTF|, mtf_arg[16384] = arg MTF. */
typedef struct ldg_filters {
  const double *rfvideo, *mtf, *fvideo, *fvideo05, *fvideoburst, *fvideopilot, *fpsync;
  const double *audio_lfilt, *audio_rfilt, *audio_lpf2;
  const double *mtf_logabs, *mtf_arg;
  /* The butter(1) designs the tables sample (lddecode_core.py:204-214), 13 doubles:
   * FPsync {b0, b1, a1}, Fburst {b0, b1, b2, a1, a2}, Fpilot {b0, b1, b2, a1, a2}
   * (zeros for NTSC).  The demod filters sync, burst and pilot as these
   * recurrences; ldg_set_filters checks fpsync = B/A and fvideoburst
   * (fvideopilot) = fvideo * B/A on every bin and fails with LDG_EINVAL otherwise. */
  const double *iir;
  /* Optional: the 65 taps of F05 (firwin(65, 0.5 MHz), lddecode_core.py:199-202).
   * When given, ldg_set_filters checks fvideo05 = fvideo * DFT(taps) on every bin
   * (NULL: no check). */
  const double *f05_fir;
} ldg_filters;

int ldg_create(const ldg_config* cfg, ldg_ctx** out);
int ldg_destroy(ldg_ctx* ctx);
/* Human-readable description of the last error on this context. */
const char* ldg_last_error(const ldg_ctx* ctx);
int ldg_set_filters(ldg_ctx* ctx, const ldg_params* p, const ldg_filters* f);

/* Make samples [first_sample, first_sample + nsamples) of a capture resident in
 * HBM.  `data` points at the raw bytes of that window in the given format
 * (first_sample must be a multiple of 3 for .r30 and of 4 for .lds).
 * is_device != 0: `data` is already a device pointer (used in place). */
int ldg_set_capture(ldg_ctx* ctx, const void* data, int64_t nsamples, int fmt, int64_t first_sample,
                    int is_device);

/* ---- streamed capture (replaces RFDecode's per-block loader calls,
 * lddecode_core.py:373-392 -> lddutils.py:131-229, for a capture of any length) ----
 * ldg_stream_open makes the file at `path` (format fmt, as ldg_set_capture) the capture,
 * streamed from storage by a reader thread through pinned staging into a ring of
 * ring_bytes in HBM (device memory independent of the file's length; rounded down to
 * the reader's chunk), starting at first_sample's packing group.  Decodes then read it
 * as a resident capture, with two rules:
 *   - a launch waits until the samples its reads need have been read (overlapped:
 *     the reader runs ahead as far as the ring allows);
 *   - the host releases what it will not read again: ldg_stream_release(below) lets
 *     the reader overwrite samples below `below` once the launches issued so far have
 *     finished.  A launch whose reads end past the ring's reach (ldg_stream_window
 *     out[1]) fails with LDG_ESTATE; reads starting below the released point come back
 *     LDG_FS_EOF.
 * ldg_stream_seek restarts the stream at another sample (no decode outstanding).  Opening
 * a file while a stream of the same ring_bytes is open reuses its ring (no decode
 * outstanding).  The chunks' copies rotate over four copy streams (LDG_STREAM_COPIES
 * sets 1 - 4), one host-to-device DMA engine each.
 * ldg_set_capture, ldg_synth_capture and ldg_destroy close the stream. */
int ldg_stream_open(ldg_ctx* ctx, const char* path, int fmt, int64_t ring_bytes, int64_t first_sample);
int ldg_stream_release(ldg_ctx* ctx, int64_t below_sample);
int ldg_stream_seek(ldg_ctx* ctx, int64_t first_sample);
/* out[0..3]: the lowest sample a launch may read, the highest block end it may reach,
 * the samples read so far, the capture's total samples. */
int ldg_stream_window(ldg_ctx* ctx, int64_t* out4);
/* Up to n doubles: bytes read, seconds in read(2), chunks, launches that waited for data,
 * seconds they waited, seconds the reader waited for ring space, seeks, ring bytes, chunk
 * bytes, seconds the reader waited for a staging buffer's copy.  Returns the count written. */
int ldg_stream_stats(ldg_ctx* ctx, double* out, int n);
int ldg_stream_close(ldg_ctx* ctx);

/* Demodulate and analyse n field reads: read i starts at read_starts[i] (the
 * `start` argument of RFDecode.demod, readlen 1,000,000) with MTF level
 * mtf[i] and is stored in device slot slots[i] (0 <= slot < max_reads,
 * distinct; slots == NULL means slot i).  Fills info[i].  A slot keeps its
 * read (demod channels, line locations, .tbc lines) until it is reused, so a
 * host may cache reads across calls. */
int ldg_decode_reads(ldg_ctx* ctx, int n, const int64_t* read_starts, const double* mtf, const int32_t* slots,
                     ldg_field_info* info);
/* The same in two halves: launch without waiting, then wait and fetch the
 * records of the OLDEST outstanding call.  Up to eight calls may be outstanding:
 * a call's demod overlaps the field kernels of the calls before it, and with
 * three outstanding the demods run back to back.  Slots of
 * outstanding calls must be distinct and are not readable until their wait.
 * Output work (frames, audio, archive, comb) runs on other streams, so a host
 * can replay and output one batch while the next two decode. */
int ldg_decode_reads_async(ldg_ctx* ctx, int n, const int64_t* read_starts, const double* mtf,
                           const int32_t* slots);
/* The same with per-read flags (full may be NULL; in/out):
 *   LDG_READ_FULL  exempts read i from the video cut;
 *   LDG_READ_PROBE marks read_starts[i] as a prediction: a probe demodulates the one
 *     block centred on it and moves the read to the sync peak it finds within
 *     0.3 lines (the start the previous field's nextfieldoffset gives when the
 *     prediction is a sample or two off).  The read's actual start comes back in
 *     its record (ldg_field_info.readsample).  Speculative planning only: the
 *     caller still accepts a read only at the exact start its chain reaches.  On
 *     return the flag is left set exactly for the reads that were probed (a probe
 *     block outside the resident capture, or a stage-isolation run without the
 *     demod, clears it): the caller tracks only those as probes in flight. */
#define LDG_READ_FULL 1
#define LDG_READ_PROBE 2
int ldg_decode_reads_async2(ldg_ctx* ctx, int n, const int64_t* read_starts, const double* mtf,
                            const int32_t* slots, uint8_t* full);
/* Video cut (0, the default: none): the demod of later decodes stops each block whose
 * outputs start at or past `out_samples` (read output index: sample start - 1024) after
 * the sync channel -- the video, burst and pilot channels are not computed there.  A
 * field whose lines reach past the cut comes back LDG_FS_VCUT: decode it again with
 * full[i] = 1.  With a cut past the field (NTSC: ~10 lines before its vsync + 266
 * lines), a read skips its tail blocks' video IFFT and stores. */
int ldg_set_video_cut(ldg_ctx* ctx, int64_t out_samples);
int ldg_decode_reads_wait(ldg_ctx* ctx, ldg_field_info* info);

/* 48 kHz audio for fields in the given slots with the given starting time
 * offsets.  pcm receives, per field, 2*count int16 samples at
 * pcm + i * pcm_stride; counts[i], next_offsets[i] are returned. */
int ldg_field_audio(ldg_ctx* ctx, int n, const int32_t* slots, const double* offsets, int16_t* pcm,
                    int64_t pcm_stride, int32_t* counts, double* next_offsets);

/* ldg_field_audio in two halves (one outstanding): launch, so the kernel and
 * the copies overlap the host's next batch, then collect into the caller's
 * arrays (as ldg_field_audio would have filled them). */
int ldg_field_audio_async(ldg_ctx* ctx, int n, const int32_t* slots, const double* offsets);
int ldg_field_audio_collect(ldg_ctx* ctx, int16_t* pcm, int64_t pcm_stride, int32_t* counts, double* next_offsets);

/* Field archive (field-group sharding): keep the inputs of
 * ldg_field_audio of n live slots (field record, final line locations, 625 kHz
 * audio) at archive entries first..first+n-1, so a field's 48 kHz audio can be
 * computed after its read slot is reused -- once a shard learns its exact
 * starting audio time offset from the shards before it. */
int ldg_archive_fields(ldg_ctx* ctx, int n, const int32_t* slots, int64_t first);
/* ldg_field_audio over archive entries (any number: more than max_reads run in one
 * launch on buffers of their own).  pcm_stride 0: the fields' samples packed one
 * after another (pcm holds at least n * 2048 int16; field i's 2 * counts[i] samples
 * follow field i - 1's). */
int ldg_archive_audio(ldg_ctx* ctx, int n, const int64_t* entries, const double* offsets, int16_t* pcm,
                      int64_t pcm_stride, int32_t* counts, double* next_offsets);
/* The 48 kHz time-offset chain of downscale_audio (lddecode_core.py:432-437,484)
 * over n fields of line counts linecounts[] from o0: out[0] = o0, out[k + 1] =
 * np.arange(out[k], frametime_k + gap, gap)[-1] - frametime_k, in numpy's float
 * arange arithmetic (host code; a shard replays the earlier shards' transitions
 * with it).  LDG_EINVAL when a range is empty (the reference's IndexError). */
int ldg_audio_offsets(double o0, int64_t n, const double* linecounts, double line_period, double* out);

/* Interleave field pairs (top slot, bottom slot) into .tbc frames
 * (outlinelen x frame_lines uint16).  out_is_device: `out` is a device pointer. */
int ldg_assemble_frames(ldg_ctx* ctx, int n, const int32_t* top_slots, const int32_t* bottom_slots,
                        uint16_t* out, int out_is_device);

/* Debug / parity access to the per-read device arrays of a live slot.
 * what: 0..4 demod channels (demod, demod_05, demod_sync, demod_burst, demod_pilot)
 *       [float64, n_out] (demod_05, demod_sync and demod_burst are expanded on request from
 *       their compact forms); 10,11: audio_left/right after phase 2 [float64];
 *       20..24: linelocs1, linelocs2, linelocs3, linelocs4, final linelocs [float64];
 *       30: burstlevel [float32]; 31: linebad [int8]; 40: dspicture [uint16]; 41: peaklist [int32];
 *       50: the last ldg_comb_ntsc[3d] call's burst-level EMA per line (lines 38..524 of each
 *       frame) [float64]; 51: the comb's carried EMA state [float64] (50 and 51 ignore `slot`).
 * Copies up to `cap` bytes to host `dst`; returns bytes copied (>= 0) or an error. */
int64_t ldg_debug_read(ldg_ctx* ctx, int slot, int what, void* dst, int64_t cap);

/* Parity access to the demod's RF filter for one MTF level: RFVideo * MTF**mtf
 * (RFVideo alone at mtf == 0: demodblock skips the product, lddecode_core.py:290-293),
 * as the kernel ldg_k_rf_table builds it for a decode call.  dst: 16384 complex
 * values (re, im interleaved), natural bin order. */
int ldg_debug_rf_table(ldg_ctx* ctx, double mtf, double* dst);

/* 2D NTSC comb (comb-ntsc.cxx dim=2 defaults, comb-ntsc.cxx:834-892) on n
 * 910x525 .tbc frames, rgb48 744x480 out (the frames comb-ntsc writes to
 * stdout, :704-733, :894-938).  State (the burst-level EMA aburstlev,
 * :560-566) persists in ctx across calls exactly as across frames of one
 * reference comb process; ldg_comb_reset starts a new process.
 * io_is_device != 0: frames / rgb_out are device pointers; frames == NULL takes
 * the context's frame buffer (ldg_assemble_frames with out == NULL), rgb_out ==
 * NULL keeps the result in the context. */
int ldg_comb_ntsc(ldg_ctx* ctx, int n, const uint16_t* frames, uint16_t* rgb_out, int io_is_device);
int ldg_comb_reset(ldg_ctx* ctx);
/* comb-ntsc's options (main's getopt, comb-ntsc.cxx:972-1091) for every later
 * ldg_comb_ntsc / ldg_comb_ntsc_async / ldg_comb_ntsc3d call; NULL restores the
 * defaults.  Values as typed on the reference's command line (IRE, not scaled).
 * Output frames are 744 x linesout x 3 uint16. */
typedef struct ldg_comb_opts {
  double black_ire;    /* -I  setup removed in RGB conversion (default 7.5)          */
  double brightness;   /* -b  (default 236)                                          */
  double nr_y;         /* -n  luma noise-reduction clip, IRE (default 1; <= 0 off)   */
  double nr_c;         /* -N  chroma noise-reduction clip, IRE (default 0 = off)     */
  int32_t bw;          /* -B  black and white (I = Q = 0)                            */
  int32_t adaptive2d;  /* 1; -a toggles (Split2D weights fixed at 1)                 */
  int32_t colorlpf;    /* 1; -L toggles (FilterIQ off)                               */
  int32_t colorlpf_hq; /* 1; -Q toggles (Q through f_colorlpq)                       */
  int32_t linesout;    /* 480; -v: 525 (from line 20: the VBI rows; the last 20 black) */
  int32_t debug_line;  /* -l  line (f_debugline + 25) blacked out; -1000 none        */
  int32_t wide;        /* -W  910-wide output rows from x 0 (default 0: 744 from 78) */
  int32_t opticalflow; /* ldg_comb_ntsc3d: 1 = comb-ntsc -d 3 (with optical flow, the
                          reference's default; BUILD-DEFINED Farneback),
                          0 = -d 3 -F */
} ldg_comb_opts;
int ldg_comb_set_opts(ldg_ctx* ctx, const ldg_comb_opts* opts);
/* Start the comb from a given burst-level EMA (comb-ntsc.cxx:560-566; -1 = not
 * yet initialised, as after ldg_comb_reset): a field-group shard's comb starts
 * from the state the previous shard's frames end in (ldgpu/shard.py). */
int ldg_comb_set_state(ldg_ctx* ctx, double aburstlev);
/* Asynchronous form for a fused pipeline: comb the first n frames of the
 * context's frame buffer (the last ldg_assemble_frames into it) into its rgb
 * buffer on the comb's own stream, overlapped with the next ldg_decode_reads.
 * The context alternates two frame buffers, so the next assembly does not wait
 * for this comb; the one after it (into the same buffer) does.  ldg_sync waits
 * for all outstanding work.  ldg_comb_async is the same for the context's
 * system: the NTSC 2D comb, or for PAL the build-defined Y/C decoder of
 * ldg_comb_pal (576 x 1057 rgb48 per frame). */
int ldg_comb_ntsc_async(ldg_ctx* ctx, int n);
int ldg_comb_async(ldg_ctx* ctx, int n);
/* 3D NTSC comb without optical flow, as `comb-ntsc -d 3 -F -c core -r range`
 * (Process with f = 1 and Split3D(opt_flow = false), comb-ntsc.cxx:369-412,
 * 834-892).  The reference combs frame k once frame k+1 has been read, so a
 * process outputs nothing for its first two frames and never outputs its last
 * one: this call takes n host frames, writes *n_out rgb48 frames to host
 * rgb_out (room for n is enough) and holds the last two inputs in ctx for the
 * next call.  core_ire / range_ire < 0 take the -F defaults 1.25 / 5.5 IRE.
 * Shares the burst-level EMA with ldg_comb_ntsc (one process is either 2D or
 * 3D); ldg_comb_reset also drops the held frames. */
int ldg_comb_ntsc3d(ldg_ctx* ctx, int n, const uint16_t* frames, uint16_t* rgb_out, int* n_out, double core_ire,
                    double range_ire);
/* PAL Y/C decoder (SURVEY §8 f, row F2), BUILD-DEFINED: the snapshot has no
 * PAL comb for the 1135x625 .tbc geometry; this is attic2/comb-pal.cxx's dim=2
 * path (Split1D / Split2D over lines +-4 / SplitIQ / AdjustY / Y-NR / burst
 * angle rotation / V-switch flip / YUV->RGB) adapted to it (oracle/combpal.cpp
 * states the choices).  n host frames of 1135x625 uint16 in, n rgb48 frames of
 * 1057x576 out; the burst-level EMA carries across calls (ldg_comb_reset). */
int ldg_comb_pal(ldg_ctx* ctx, int n, const uint16_t* frames, uint16_t* rgb_out);
/* (ldg_output_async with rgb_host on a PAL context runs this decoder on the
 * device frames: 576 x 1057 rgb48 per frame.) */
int ldg_sync(ldg_ctx* ctx);

/* The CLI's output path without host round trips: interleave n field pairs into
 * .tbc frames in HBM (as ldg_assemble_frames), comb them there when rgb_host is
 * non-NULL (the 2D NTSC comb, ldg_comb_set_opts' options, state as ldg_comb_ntsc;
 * on a PAL context the Y/C decoder of ldg_comb_pal, 576 x 1057 rgb48 per frame),
 * and copy the frames (and rgb48) to the host buffers asynchronously on the
 * output stream, overlapped with the next decode.  The buffers must stay valid
 * (pinned memory from ldg_host_alloc for full copy speed) until the matching
 * ldg_output_wait: each call waits for the OLDEST outstanding ldg_output_async's
 * copies (first in, first out; at most 4 outstanding, LDG_ESTATE past that), so
 * the host can issue batch k+1 before handing batch k to its sink. */
int ldg_output_async(ldg_ctx* ctx, int n, const int32_t* top_slots, const int32_t* bottom_slots, uint16_t* tbc_host,
                     uint16_t* rgb_host);
int ldg_output_wait(ldg_ctx* ctx);
/* Page-locked host memory (hipHostMalloc) for ldg_output_async's buffers. */
int ldg_host_alloc(int64_t nbytes, void** out);
int ldg_host_free(void* p);

/* ---- in-library kernel timing (HIP events on the context's stream) ------------- */
typedef struct ldg_kernel_stat {
  char name[48];
  int64_t launches;
  double total_ms; /* sum of per-launch event durations */
} ldg_kernel_stat;
/* on == 1: record a start/stop event pair around every kernel launch; on == 2:
 * around the demod only (the roofline kernel; two events per call instead of
 * ~30); 0: off.  Resets the stats. */
int ldg_profile_enable(ldg_ctx* ctx, int on);
/* Copy up to max per-kernel records; returns the number of kernels recorded. */
int ldg_profile_read(ldg_ctx* ctx, ldg_kernel_stat* out, int max);
/* The demod launches' execution spans since ldg_profile_enable (first workgroup
 * start to last workgroup end on the device's constant-rate clock, what a
 * kernel trace reports): count and summed milliseconds. */
int ldg_profile_spans(ldg_ctx* ctx, double* total_ms, int64_t* count);
/* The union of those spans (time with at least one demod launch executing; two
 * demod streams overlap consecutive launches) and the launch count. */
int ldg_profile_spans_union(ldg_ctx* ctx, double* union_ms, int64_t* count);
/* Every profiled demod launch in issue order, four doubles each: execution start,
 * end, and the host's issue time, in ms on the device's constant-rate clock from
 * the first launch's start (issue times mapped by a calibration taken in
 * ldg_profile_enable, a few microseconds uncertain; NaN start / end for a launch
 * that ran no workgroup), then the issue time in ms on the host's monotonic clock.
 * Returns the number of rows written (<= max) or < 0. */
int ldg_profile_span_table(ldg_ctx* ctx, double* out, int max);

/* Benchmark roofline leg (not a reference interface): the demod kernel alone
 * (symbol ldg_k_demod_iso, so a kernel trace separates it from the pipeline's
 * ldg_k_demod) over n live slots, `iters` launches back to back on one stream;
 * *ms_per_launch = the mean HIP-event duration of a launch.  The slots' demod
 * outputs are recomputed in place (a host read cache should be dropped). */
int ldg_demod_isolated(ldg_ctx* ctx, int n, const int32_t* slots, int iters, double* ms_per_launch);
/* The same leg by variant: 0 = ldg_k_demod_iso (as above, every block in full),
 * 1 = ldg_k_demod_iso_cut, the shipped body of ldg_k_demod (blocks past a read's
 * video cut stop after the sync channel) under its own symbol.  LDG_EINVAL for
 * other variants. */
int ldg_demod_isolated_ex(ldg_ctx* ctx, int n, const int32_t* slots, int iters, int variant, double* ms_per_launch);

/* ---- benchmark / test tooling (not a reference interface) ----------------------
 * Synthesise an NTSC LaserDisc RF capture directly into this context's HBM
 * capture buffer (same signal model as ldgpu/synth.py), then make it the
 * current capture (first_sample 0).  fir: 63 band-limit taps; emph: b0, b1, a1
 * of the pre-emphasis IIR; codes: 3 Philips code words per frame. */
typedef struct ldg_synth_params {
  int32_t fmt;          /* LDG_FMT_* of the generated capture */
  int32_t pad_;
  int64_t nsamples;
  uint64_t seed;
  double noise;         /* Gaussian sigma relative to the unit video carrier */
  double start_line;    /* capture starts this many lines into frame 0 */
} ldg_synth_params;
int ldg_synth_capture(ldg_ctx* ctx, const ldg_synth_params* p, const double* fir63, const double* emph,
                      const uint32_t* codes, int64_t ncodeframes);
/* Copy nbytes of the resident capture starting at byte offset to dst (host memory
 * or a device buffer of the same device). */
int64_t ldg_capture_download(ldg_ctx* ctx, void* dst, int64_t offset, int64_t nbytes);

/* CX expander for the .pcm stream (cx-expander.cxx:9-117): host code, one
 * sequential chain (the channels are coupled through the peak followers).
 * ldg_cx_process takes n stereo frames of uint16 (L, R interleaved; the
 * reference reads the stream as unsigned and subtracts 32768) and writes n
 * expanded stereo frames; state persists across calls like one cx process.
 * The reference drops a trailing partial 1024-frame block (:105-113): that is
 * the caller's (cx_expander.py's) job. */
typedef struct ldg_cx ldg_cx;
int ldg_cx_create(ldg_cx** out);
int ldg_cx_destroy(ldg_cx* cx);
int ldg_cx_process(ldg_cx* cx, int64_t n, const uint16_t* in, uint16_t* out);

/* Library / device identification. */
const char* ldg_version(void);
int ldg_device_count(void);
/* Free and total device memory of `device` (hipMemGetInfo): what a context holds. */
int ldg_device_memory(int device, int64_t* free_bytes, int64_t* total_bytes);

#ifdef __cplusplus
}
#endif
#endif /* LDGPU_H */
