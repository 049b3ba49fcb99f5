// Shared host/device definitions for libldgpu (not part of the public ABI).
#pragma once
#include <stdint.h>

namespace ldg {

// Overlap-save geometry of RFDecode.demod (lddecode_core.py:120-122,145,373-410).
constexpr int BLOCKLEN = 16384;
constexpr int BLOCKCUT = 1024;
constexpr int BLOCKCUT_END = 32;                      // F05_offset
constexpr int BLOCKSTEP = BLOCKLEN - BLOCKCUT - BLOCKCUT_END;   // 15328
constexpr int HALF = BLOCKLEN / 2;                     // 8192-point complex FFTs
constexpr int MAX_BLOCKS_PER_READ = 66;
constexpr int PARK_SLOTS = 2048;                       // demod odd-half parks: one per physical CU (demod.hip)
constexpr int PARK_EXTRA = 64;                         // spare parks (a CU's park held by a switched-out workgroup)
constexpr int PARK_SCRATCH = PARK_SLOTS + PARK_EXTRA;  // the shared scratch park (no owner)
constexpr int PARK_TOTAL = PARK_SCRATCH + 1;
constexpr int PARK_OWNERS = PARK_SLOTS + PARK_EXTRA;   // owner words
constexpr int READLEN = 1000000;
constexpr int MAX_NOUT = READLEN + 1026 + 16;          // end - start + 1 (+ slack)
constexpr int AUDIO_DIV1 = 16;                         // 40 MHz -> 2.5 MHz (blocklen / 1024)
constexpr int AUDIO_BLOCK = 1024;
constexpr int MAX_NAUDIO = MAX_NOUT / AUDIO_DIV1 + 16;
constexpr int AUDIO_DIV2 = 4;                          // 2.5 MHz -> 625 kHz
constexpr int AUDIO2_BLOCK = 4096;
constexpr int MAX_NAUDIO2 = MAX_NAUDIO / AUDIO_DIV2 + 16;
constexpr int MAX_PEAKS = 2048;
constexpr int MAX_VSYNCS = 16;
constexpr int MAX_LINES = 320;                         // linecount + 4 <= 317 (PAL)
constexpr int MAX_OUTW = 1135;                         // PAL 4fsc line
constexpr int LINENUM_OFF = 1024;                      // dict key offset for compute_linelocs
constexpr int LINENUM_SPAN = 2048;

// demod channel order (rec-array fields of lddecode_core.py:314-316)
enum Chan { CH_DEMOD = 0, CH_05 = 1, CH_SYNC = 2, CH_BURST = 3, CH_PILOT = 4 };
constexpr int MAX_CHAN = 5;

// Field status codes (reason a Field is not valid; lddecode_core.py:909-941,1043-1048,1178-1191)
enum FieldStatus {
  FS_VALID = 0,
  FS_NO_VSYNC = 1,        // len(vsyncs) == 0
  FS_SHORT = 2,           // one vsync / too few peaks after the second
  FS_LINELOCS = 3,        // exception in compute_linelocs / refine_linelocs_hsync
  FS_TBC = 4,             // exception in burst/pilot refine or final downscale
  FS_EOF = 5,             // a block of this read lies beyond the capture (reference: crash / None)
  FS_CRASH = 6,           // reference would raise uncaught (e.g. vsync within first 11 peaks)
  FS_PENDING = 7,
  FS_MIGRATED = 8,        // the demod workgroup changed CU mid-block (its park was not private): decode again
  FS_VCUT = 9,            // a field kernel needed a video sample past the read's video cut: decode again in full
};

// Per-read descriptor, written by the host before a batch.
struct ReadDesc {
  int64_t readsample;     // 'start' argument of demod() (lddecode_core.py:373)
  int64_t s0;             // first block sample (start - blockcut, or 0)
  int64_t end;            // int(start + length) + 1
  int32_t n_out;          // end - s0 + 1 (video samples)
  int32_t n_blocks;
  int32_t n_audio;        // ((end - s0) // 16) + 1
  int32_t n_audio2;       // n_audio // 4
  int32_t filt_slot;      // index of the RF filter table (RFVideo * MTF**mtf)
  int32_t pad_;
  int64_t vcut;           // demod outputs from here on need no video / burst / pilot channel
                          // (blocks at or past it stop after the sync channel; a field kernel
                          // that reaches past it flags FS_VCUT)
};

// System/filter scalars (lddecode_core.py:30-117, 119-279)
struct SysConst {
  double freq_hz;         // 40e6
  double freq;            // 40 (MHz; rf.freq)
  double ire0, hz_ire, vsync_ire;
  double sync_lo, sync_hi;        // iretohz(-55), iretohz(-25)
  double freq_arf;                // 2.5e6
  double audio_lowfreq;
  double audio_lfreq, audio_rfreq;
  double line_period;             // us
  double fsc_mhz;
  double sy_b0, sy_p;             // FPsync recurrence (iir.hpp): b0, p = -a1
  double bu_b0, bu_b1, bu_b2, bu_a1, bu_a2;   // Fburst recurrence
  int32_t system;                 // 0 NTSC, 1 PAL
  int32_t linelen;                // rf.linelen (2542 / 2560)
  int32_t outlinelen;             // 910 / 1135
  int32_t frame_lines;            // 525 / 625
  int32_t n_chan;                 // 4 NTSC, 5 PAL
  int32_t audio_lo0;              // audio_fdslice_lo.start (791)
  int32_t codelines[3];           // philips_codelines
  int32_t pad_;
};

// Sync-channel tiles: for every 32 consecutive demod_sync outputs of a read
// (tile t = outputs [32 t, 32 t + 32); overlap-save blocks keep 15328 = 32 * 479
// outputs, so a tile never straddles two blocks) the maximum and the index of
// its first occurrence, np.argmax order (a NaN is the maximum, the first NaN
// wins).  The demod writes them beside the channel; get_syncpeaks' window
// argmax then reads whole tiles plus the two ragged ends.
struct SyncTile {
  double v;
  int64_t idx;             // absolute output index (INT64_MAX: tile has no output)
};
constexpr int64_t STILE_PER_SLOT = MAX_NOUT / 32 + 2;

// (v, vi) comes before (b, bi) in np.argmax order
__device__ __forceinline__ bool am_beats(double v, int64_t vi, double b, int64_t bi) {
  const bool vn = v != v, bn = b != b;
  if (vn || bn) return vn && (!bn || vi < bi);
  return v > b || (v == b && vi < bi);
}

// Latency-bound kernels (a wave per read / per line, one lane per recurrence)
// share CUs with the FP64-throughput demod; raise their wave priority so the
// SIMD arbiter issues their serial chains first (demod waves fill the gaps).
__device__ __forceinline__ void prio_latency() { __builtin_amdgcn_s_setprio(3); }

}  // namespace ldg

// The optical-flow fields of the 3D comb with flow (flow.hip, comb.hip): 252 x 840
// luma fields, rows 23 + field + 2 y and columns 70..909 of a 525 x 910 frame.
namespace ldg {
namespace flow {
constexpr int FR = 252, FC = 840, FY0 = 23, FX0 = 70;
}  // namespace flow
}  // namespace ldg

// Per-kernel phase stamps (profiling builds only, -DLDG_STAMPS; tools/kstamps.py):
// thread 0 of the first KST_BLOCKS workgroups of kernel K records the shader
// clock at phase boundary i (after a workgroup barrier).
// K: 0 comb_rows, 1 final_lines, 2 burst_field, 3 sync, 4 burst_lines, 5 philips.
#ifdef LDG_STAMPS
constexpr int KST_KERNELS = 6, KST_BLOCKS = 4096, KST_PHASES = 16;
__device__ unsigned long long g_kst[KST_KERNELS][KST_BLOCKS][KST_PHASES];
#define KSTAMP(K, i)                                                               \
  do {                                                                             \
    __syncthreads();                                                               \
    if (threadIdx.x == 0 && blockIdx.x < KST_BLOCKS)                               \
      g_kst[K][blockIdx.x][i] = __builtin_readcyclecounter();                      \
  } while (0)
#else
#define KSTAMP(K, i) \
  do {               \
  } while (0)
#endif
