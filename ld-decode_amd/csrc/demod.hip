// RF demodulation: one 1024-thread workgroup per 16384-sample overlap-save block.
//
// Restates, per block, RFDecode.demodblock + the block copy of RFDecode.demod
// (lddecode_core.py:288-330, 373-422) and unwrap_hilbert (lddutils.py:320-334)
// as ONE fused kernel: every intermediate lives in LDS/registers and only the
// kept part [1024, 1024+copylen) of each channel is written to HBM.
//
// Real 16384-point transforms are done as 8192-point complex FFTs plus a
// split/merge step; the complex 16384-point analytic-signal IFFT is done as
// its radix-2 decimation-in-frequency halves (even/odd outputs).  FP64 end to
// end (1 LSB of .tbc = 33.9 Hz).
//
// Per block, 8192-point FFTs: raw R2C, analytic even, analytic odd, demod R2C,
// C2R 0.5 MHz, C2R video = 6 (NTSC and PAL).  The sync, burst and pilot
// channels, whose filters are sampled butter(1) designs, are their periodic
// recurrences in the time domain (iir.hpp); sync and burst are stored compact,
// as per-chunk states the field kernels expand (chan.hpp).
#include <hip/hip_runtime.h>
#include "common.hpp"
#include "fft8k.hpp"
#include "iir.hpp"
#include "chan.hpp"

using namespace ldg;

namespace {

constexpr int T = 1024;
constexpr int M = HALF;           // 8192

__device__ __forceinline__ double load_sample(const uint8_t* __restrict__ cap, int fmt, int64_t rel) {
  if (fmt == 0) return (double)cap[rel];
  if (fmt == 1) return (double)reinterpret_cast<const int16_t*>(cap)[rel];
  if (fmt == 2) {   // .r30: 3 x 10 bit per LE uint32, low bits first (lddutils.py:150-173)
    const int64_t w = rel / 3;
    const int sh = 10 * (int)(rel - 3 * w);
    return (double)((reinterpret_cast<const uint32_t*>(cap)[w] >> sh) & 0x3ffu);
  }
  // .lds: 4 x 10 bit in 5 bytes, MSB first (lddutils.py:195-229)
  const int64_t g = rel >> 2;
  const int k = (int)(rel & 3);
  const uint8_t* b = cap + 5 * g;
  uint32_t v;
  if (k == 0) v = ((uint32_t)b[0] << 2) | (b[1] >> 6);
  else if (k == 1) v = ((uint32_t)(b[1] & 0x3f) << 4) | (b[2] >> 4);
  else if (k == 2) v = ((uint32_t)(b[2] & 0x0f) << 6) | (b[3] >> 2);
  else v = ((uint32_t)(b[3] & 0x03) << 8) | b[4];
  return (double)v;
}

// X[k] of a real 2M-point signal from Z = FFT_M(x[2m] + i x[2m+1]):
// X = (A + conj B)/2 + w * (-i/2)(A - conj B), A = Z[k], B = Z[M-k], w = W_2M^k.
__device__ __forceinline__ double2 rsplit(double2 A, double2 B, double2 w) {
  const double2 e = make_double2(0.5 * (A.x + B.x), 0.5 * (A.y - B.y));
  const double2 d = make_double2(A.x - B.x, A.y + B.y);
  const double2 o = make_double2(0.5 * d.y, -0.5 * d.x);
  return cadd(e, cmul(w, o));
}

// Inverse of rsplit: half-spectrum (P[k], P[M-k]) -> Z[k] whose M-point IFFT
// interleaves the real 2M-point result.
__device__ __forceinline__ double2 cmerge(double2 Pk, double2 Pkp, double2 w) {
  const double2 e = make_double2(0.5 * (Pk.x + Pkp.x), 0.5 * (Pk.y - Pkp.y));
  const double2 d = make_double2(Pk.x - Pkp.x, Pk.y + Pkp.y);
  const double2 o = cmulc(d, w);
  return make_double2(e.x - 0.5 * o.y, e.y + 0.5 * o.x);
}

// unwrap_hilbert's unwrap + fold, elementwise: the principal phase difference
// folded into [0, tau) (lddutils.py:321-333; differences vs. the cumulative
// form are O(1e-13 rad)).
__device__ __forceinline__ double fold_tau(double d) {
  constexpr double TAU = 6.283185307179586;
  return d < 0.0 ? d + TAU : d;
}

// Half-spectrum pair slots over the digit-reversed spectrum layout that
// fft8k_dif produces (fft8k.hpp): thread tid owns slots c = 0..3 and thread 0
// also slot 4, 4097 slots covering the bins k in [0, M] as pairs (k, M-k).
// Slot c < 3 (and c == 3 for tid < 512) takes sub-array q = 1..7 position
// 512 q + j, whose partner M-k sits at 512 (16-q) + 511 - j: contiguous (and
// reversed) across lanes.  The rest pair up sub-array 8 with itself and
// sub-array 0 (k = 16 k', a 512-point digit-reversed array) with itself.
//   p, pp: LDS positions of k and of M-k (pp == p for k = 0, whose partner is
//   the Nyquist bin M, and for k = M/2); gp: table index of M-k (M for k = 0).
struct Slot {
  int p, pp, gp;
};

__device__ __forceinline__ Slot slot_of(int tid, int c) {
  if (c < 3 || (c == 3 && tid < 512)) {
    const int i = tid + 1024 * c, q = 1 + (i >> 9), j = i & 511;
    const int pp = 512 * (16 - q) + 511 - j;
    return {512 * q + j, pp, pp};
  }
  if (c == 3 && tid < 768) {
    const int j = tid - 512;
    return {4096 + j, 4607 - j, 4607 - j};
  }
  const int z = c == 4 ? 256 : tid - 768;
  int p, pp;
  if (z < 192) {
    const int sb = 1 + (z >> 6), jj = z & 63;
    p = 64 * sb + jj;
    pp = 64 * (8 - sb) + 63 - jj;
  } else if (z < 224) {
    p = 256 + (z - 192);
    pp = 319 - (z - 192);
  } else if (z < 248) {
    const int w = z - 224, u = 1 + (w >> 3), v = w & 7;
    p = 8 * u + v;
    pp = 8 * (8 - u) + 7 - v;
  } else if (z < 252) {
    p = 32 + (z - 248);
    pp = 39 - (z - 248);
  } else if (z < 255) {
    p = z - 251;
    pp = 8 - p;
  } else if (z == 255) {
    return {0, 0, M};
  } else {
    return {4, 4, 4};
  }
  return {p, pp, pp};
}

// This workgroup's physical CU: (XCC, SE, SH, CU) from HW_REG_XCC_ID / HW_REG_HW_ID
// (gfx9 HW_ID: CU_ID [11:8], SH_ID [12], SE_ID [15:13]), < PARK_SLOTS (common.hpp).
// One park per CU is private only while two demod workgroups can never share a CU
// (also across the two demod streams' concurrent launches): the transform buffer
// alone is more than half of the CU's 160 KiB of LDS.
static_assert(sizeof(double2) * HALF > 160 * 1024 / 2, "demod workgroups must not share a CU");
__device__ __forceinline__ int cu_slot() {
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
  const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
  return (int)(((xcc & 7u) << 8) | (((hw >> 13) & 7u) << 5) | (((hw >> 12) & 1u) << 4) | ((hw >> 8) & 15u));
}

// Opaque copy of tid: stops the compiler from hoisting per-lane twiddle loads
// and addresses that repeat across the kernel's transforms (and spilling them).
__device__ __forceinline__ int fresh(int tid) { asm volatile("" : "+v"(tid)); return tid; }

__device__ __forceinline__ bool pair_live(int tid, int c) { return c < 4 || tid == 0; }

// W_2M^(M-k) = -conj(W_2M^k)
__device__ __forceinline__ double2 tw_mirror(double2 w) { return make_double2(-w.x, w.y); }

// Timing probe only (-DLDG_PROBE_NOSTORE): the channel stores are skipped, results are garbage.
// Timing probes only (-DLDG_PROBE=bits): 1 no atan2, 2 no video transform,
// 4 no IIR scans, 8 no raw transform, 16 no filter/park phase, 32 no merges,
// 64 no split of the raw and demod spectra, 128 no filter-table loads in the
// filter phase, 256 no park stores.  Results are garbage.
#ifdef LDG_PROBE
constexpr int kProbe = LDG_PROBE;
#else
constexpr int kProbe = 0;
#endif
#ifdef LDG_PROBE_NOSTORE
constexpr bool kProbeNoStore = true;
#else
constexpr bool kProbeNoStore = false;
#endif

// Store the pair of samples 2m, 2m+1 of a channel (o indexed by block position)
// if kept ([BLOCKCUT, BLOCKCUT + copylen)); the wave-uniform test keeps the
// common case (a wave's 64 pairs all kept or all dropped) branch-free.
// A channel's 16-byte store, non-temporal ("nt": streamed, the lines still land
// in L2 for the field kernels; -1.9% demod time against plain stores in an
// interleaved A/B, "sc1" +13%).  Through the compiler's builtin, not inline asm:
// an asm store is opaque to the hazard recognizer, which then does not keep
// VALU writes off the store's data VGPRs until the store has read them (round 3:
// under another register allocation whole waves' stores landed corrupted now
// and then, tools/nondet_probe.py).
__device__ __forceinline__ void st_pair(double* a, double2 z) {
  typedef double v2d __attribute__((ext_vector_type(2)));
  const v2d zv = {z.x, z.y};
  __builtin_nontemporal_store(zv, reinterpret_cast<v2d*>(a));
}
// The odd-half park's stores (read back by LDS-DMA on the same CU): plain
// stores ("nt" measured +1.5%, "sc0" even).
__device__ __forceinline__ void st_park(double2* a, double2 z) { *a = z; }
// The parks' owner words: PARK_SLOTS + PARK_EXTRA 64-bit words after the parks and the
// scratch park (ospill + PARK_TOTAL * M); word u = the tag of the workgroup holding park
// u, 0 when free (see demod_body).
__device__ __forceinline__ unsigned long long* park_owner(double2* ospill) {
  return reinterpret_cast<unsigned long long*>(ospill + (int64_t)PARK_TOTAL * M);
}
__device__ __forceinline__ void store_pair(double* o, int m, double2 z, int copylen) {
  const int p = 2 * m;
  const int pw0 = 2 * (m & ~63);
  if (pw0 >= BLOCKCUT && pw0 + 127 < BLOCKCUT + copylen) {
    st_pair(o + p, z);
  } else if (pw0 + 127 >= BLOCKCUT && pw0 < BLOCKCUT + copylen) {
    const bool in0 = p >= BLOCKCUT && p < BLOCKCUT + copylen;
    const bool in1 = p + 1 >= BLOCKCUT && p + 1 < BLOCKCUT + copylen;
    if (in0 && in1) *reinterpret_cast<double2*>(o + p) = z;
    else if (in0) o[p] = z.x;
    else if (in1) o[p + 1] = z.y;
  }
}

// Store a channel's kept samples [BLOCKCUT, BLOCKCUT + copylen) from the chunk
// layout in LDS (pair m = t + 1024 q per lane: coalesced 16-byte stores).
// o is indexed by block position.
__device__ __forceinline__ void store_chan(const double2* sx, double* o, int t, int copylen) {
  if (kProbeNoStore) return;
#pragma unroll
  for (int q = 0; q < 8; q++) {
    const int m = t + 1024 * q;
    store_pair(o, m, sx[SWC(m)], copylen);
  }
}

// atan(i / 64), i = 0..64 (the fast_atan2 table; copied to LDS per workgroup)
__constant__ double c_atan64[65] = {
    0.0, 0.015623728620476831, 0.031239833430268277, 0.046840712915969654,
    0.06241880999595735, 0.0779666338315423, 0.09347678115858947, 0.1089419569898658,
    0.12435499454676144, 0.13970887428916365, 0.15499674192394097, 0.1702119252854744,
    0.18534794999569476, 0.2003985538258785, 0.21535769969773805, 0.23021958727684372,
    0.24497866312686414, 0.2596296294082575, 0.2741674511196588, 0.2885873618940774,
    0.3028848683749714, 0.31705575320914703, 0.3310960767041321, 0.34500217720710513,
    0.35877067027057225, 0.3723984466767542, 0.38588266939807375, 0.39922076957525254,
    0.4124104415973873, 0.42544963737004227, 0.43833655985795783, 0.4510696559885235,
    0.4636476090008061, 0.4760693303227612, 0.48833395105640554, 0.5004408131472942,
    0.5123894603107377, 0.5241796287829132, 0.5358112379604637, 0.5472843809874369,
    0.5585993153435624, 0.5697564534829784, 0.5807563535676704, 0.5915997103351114,
    0.6022873461349642, 0.6128202021652414, 0.6231993299340659, 0.6334258829691446,
    0.6435011087932844, 0.6534263411807619, 0.6632029927060933, 0.6728325475937632,
    0.6823165548747481, 0.6916566218531999, 0.7008544078844502, 0.7099116184635249,
    0.7188299996216245, 0.7276113326265107, 0.7362574289814281, 0.7447701257160751,
    0.7531512809621944, 0.7614027698055784, 0.7695264804056583, 0.7775243103733478,
    0.7853981633974483};

// np.angle(y + i x) = atan2(y, x) in (-pi, pi] for the FM demod (lddutils.py:320-334),
// FP64, max abs error 4.4e-16 rad (2e7 random points against libm, incl. axes and
// zeros; atan2(+-0, -0) returns +-0, not +-pi).  About a third of the
// instructions of the library atan2: r = min/max of |x|, |y| is rounded to
// c = i/64, atan(r) = atan(c) + atan(t), t = (r - c) / (1 + r c) = (n - c d)/(d + c n),
// |t| <= 1/128, so atan(t) to O(t^9) = 1e-20 is t - t^3/3 + t^5/5 - t^7/7.
__device__ __forceinline__ double fast_atan2(double y, double x, const double* s_atan) {
  const double ax = fabs(x), ay = fabs(y);
  const bool sw = ay > ax;
  const double num = sw ? ax : ay, den = sw ? ay : ax;
  const bool zero = !(den > 0.0);
  int i = (int)__builtin_rint(num * __builtin_amdgcn_rcp(den) * 64.0);
  i = zero ? 0 : min(max(i, 0), 64);
  const double c = (double)i * (1.0 / 64);
  const double n = __fma_rn(-c, den, num);
  const double d = __fma_rn(c, num, den);
  double r = __builtin_amdgcn_rcp(d);
  r = __fma_rn(r, __fma_rn(-d, r, 1.0), r);
  const double t = zero ? 0.0 : n * r;
  const double t2 = t * t;
  const double pl = __fma_rn(__fma_rn(-1.0 / 7, t2, 1.0 / 5), t2, -1.0 / 3);
  double th = s_atan[i] + __fma_rn(t * t2, pl, t);
  if (sw) th = 1.57079632679489661923 - th;
  if (x < 0.0) th = 3.14159265358979323846 - th;
  return copysign(th, y);
}

constexpr bool kFastAtan2 = true;

struct Pairs {
  double2 a[5], b[5];   // value at k and at M-k of each pair slot
};

// Half-spectrum of the real signal just transformed by fft8k_dif, for my slots.
// twk[p] = W_2M^(dr_nat(p)).
__device__ __forceinline__ void split_pairs(const CBuf x, const double2* __restrict__ twk, int tid, Pairs& X) {
  tid = fresh(tid);
#pragma unroll
  for (int c = 0; c < 5; c++) {
    if (!pair_live(tid, c)) continue;
    const Slot sl = slot_of(tid, c);
    const double2 A = x[sl.p], B = x[sl.pp];
    const double2 wk = twk[sl.p];
    X.a[c] = rsplit(A, B, wk);
    X.b[c] = rsplit(B, A, tw_mirror(wk));
  }
}

// Write merge(D * G) for my slots into LDS, digit-reversed (input of fft8k_dit).
// G: a filter in digit-reversed order (G[p] = filter[dr_nat(p)], G[M] = filter[M]).
__device__ __forceinline__ void merge_pairs(const CBuf x, const double2* __restrict__ twk,
                                            const double2* __restrict__ G, int tid, const Pairs& D) {
  tid = fresh(tid);
#pragma unroll
  for (int c = 0; c < 5; c++) {
    if (!pair_live(tid, c)) continue;
    const Slot sl = slot_of(tid, c);
    const double2 wk = twk[sl.p];
    const double2 Pk = cmul(D.a[c], G[sl.p]);
    const double2 Pkp = cmul(D.b[c], G[sl.gp]);
    x[sl.p] = cmerge(Pk, Pkp, wk);
    if (sl.pp != sl.p) x[sl.pp] = cmerge(Pkp, Pk, tw_mirror(wk));
  }
}

}  // namespace

// In-kernel phase stamps (profiling builds only: -DLDG_STAMPS, tools/demod_stamps.py):
// thread 0 of the first LDG_STAMP_BLOCKS workgroups records the shader clock
// at each phase boundary.
#ifdef LDG_STAMPS
constexpr int LDG_STAMP_BLOCKS = 8192;
__device__ unsigned long long g_stamps[LDG_STAMP_BLOCKS][32];
#define STAMP(i)                                                                   \
  do {                                                                             \
    __syncthreads();                                                               \
    if (threadIdx.x == 0 && blockIdx.x < LDG_STAMP_BLOCKS)                         \
      g_stamps[blockIdx.x][i] = __builtin_readcyclecounter();                      \
  } while (0)
#else
#define STAMP(i) \
  do {           \
  } while (0)
#endif

// grid: n_reads * MAX_BLOCKS_PER_READ workgroups of 1024 threads.
// ospill: PARK_TOTAL x 8192 double2 parks (one per physical CU, spares, scratch) + owner words.
// cap: the resident capture samples [cap_first, cap_first + cap_nsamp); ring = 0: cap holds
// them from its start; ring > 0 (a streamed capture, ldg_stream_open): cap is a ring of
// `ring` bytes (a multiple of every format's packing group) where the capture's byte b lives
// at b mod ring, followed by a mirror of its first bytes, so one block is contiguous.
#define LDG_DEMOD_PARAMS                                                                                          \
  const int32_t *__restrict__ smap, const ReadDesc *__restrict__ reads, const uint8_t *__restrict__ cap,          \
      int64_t cap_first, int64_t cap_nsamp, int64_t ring, int fmt, const double2 *__restrict__ tw,               \
      const double2 *__restrict__ twk, const double2 *__restrict__ rf_filt, const double2 *__restrict__ g_video,  \
      const double2 *__restrict__ g_05, const double *__restrict__ iir, const double2 *__restrict__ a_lfilt,      \
      const double2 *__restrict__ a_rfilt, SysConst C, double *__restrict__ video, int64_t vread_stride,          \
      int64_t vchan_stride, double *__restrict__ audio1, int64_t aread_stride, int64_t achan_stride,              \
      int32_t *__restrict__ status, double2 *__restrict__ ospill, unsigned long long park_epoch,                 \
      SyncTile *__restrict__ stiles,                                                                             \
      double2 *__restrict__ aslice, double *__restrict__ sst, uint32_t *__restrict__ sbits,                      \
      double4 *__restrict__ bst, unsigned long long *__restrict__ span
#define LDG_DEMOD_ARGS                                                                                            \
  smap, reads, cap, cap_first, cap_nsamp, ring, fmt, tw, twk, rf_filt, g_video, g_05, iir, a_lfilt, a_rfilt, C, video, \
      vread_stride, vchan_stride, audio1, aread_stride, achan_stride, status, ospill, park_epoch, stiles, aslice,  \
      sst, sbits,                                                                                                 \
      bst, span
// PROBE: one workgroup per probe read (slot smap[blockIdx.x], its block 0 only):
// ldg_k_demod_probe, below.
template <bool CUT, bool PROBE = false>
__device__ __forceinline__ void demod_body(LDG_DEMOD_PARAMS) {
  __shared__ double2 s_x[M];          // 128 KiB: the 8192-point transforms
  __shared__ uint16_t s_bits[BLOCKLEN / 16];   // sync detector bits
  __shared__ double2 s_tw[TW_LDS_N];           // per-lane FFT twiddles (fft8k.hpp)
  __shared__ IIRAux s_aux;
  __shared__ double s_atan[65];
  const CBuf X_{s_x};
  const int tid = threadIdx.x;
  if (tid < 65) s_atan[tid] = c_atan64[tid];   // ordered by the first transform's barrier
  s_tw[tw_lds_pos(tid)] = tw[2 * tid];
  const TwLds twl{s_tw};
  STAMP(0);
  // profiling: the launch's execution span on the constant-rate clock (first
  // workgroup start, last workgroup end), what a kernel trace reports
  if (span && tid == 0) atomicMax(&span[0], ~(unsigned long long)__builtin_amdgcn_s_memrealtime());
  const int slot = PROBE ? smap[blockIdx.x] : smap[blockIdx.x / MAX_BLOCKS_PER_READ];
  const int b = PROBE ? 0 : blockIdx.x % MAX_BLOCKS_PER_READ;
  const ReadDesc rd = reads[slot];
  if (b >= rd.n_blocks) return;

  const int64_t i0 = rd.s0 + (int64_t)b * BLOCKSTEP;
  const int off = b * BLOCKSTEP;
  const int copylen = (off + (BLOCKLEN - BLOCKCUT) > rd.n_out) ? rd.n_out - off : BLOCKSTEP;
  int64_t rel0 = i0 - cap_first;
  if (rel0 < 0 || rel0 + BLOCKLEN > cap_nsamp) {
    if (tid == 0) status[slot] = FS_EOF;
    return;
  }
  if (ring) {
    // streamed capture: the block's first packing group at its ring position, the block
    // read from there (contiguous through the ring's mirrored head)
    const int spg = fmt == 2 ? 3 : fmt == 3 ? 4 : 1, bpg = fmt == 1 ? 2 : fmt == 2 ? 4 : fmt == 3 ? 5 : 1;
    const int64_t g = i0 / spg;
    cap += (g * bpg) % ring;
    rel0 = i0 - g * spg;
  }
  double* vout = video + (int64_t)slot * vread_stride + off - BLOCKCUT;   // index by block position p
  const double2* F = rf_filt + (int64_t)rd.filt_slot * BLOCKLEN;
  // odd-half park, in LDS image order (park[u] = the value for LDS slot u), so
  // it returns to LDS by LDS-DMA (global_load_lds) without a register pass.
  // One park per physical CU (one demod workgroup per CU at a time: 128 KiB of
  // LDS), so consecutive workgroups on a CU rewrite the same 128 KiB and it
  // stays cache-resident instead of streaming 1 GB per launch through HBM.
  //
  // The park is owned exclusively from its claim to its release: its owner word goes
  // from 0 to this workgroup's tag (unique per launch and workgroup) by compare-and-swap,
  // and back to 0 once the reload has completed.  A CU's park is free whenever a
  // workgroup starts there, unless compute-wave save/restore (a shared or oversubscribed
  // GPU) switched out the workgroup that holds it: the claimant then takes one of
  // PARK_EXTRA spare parks, and with all of those held too it runs on the scratch park
  // (shared, unowned) and flags its read FS_MIGRATED (the host decodes it again).  No
  // workgroup can store into a park another one holds, so a read not flagged is exact.
  __shared__ int s_park;
  const int my_cu = cu_slot();
  unsigned long long* const owners = park_owner(ospill);
  const unsigned long long my_tag = (park_epoch << 32) | (unsigned long long)blockIdx.x;
  int my_park = -1;                                 // (thread 0) the park this workgroup holds
  if (tid == 0) {
    if (atomicCAS(owners + my_cu, 0ull, my_tag) == 0ull) my_park = my_cu;
    for (int e = 0; e < PARK_EXTRA && my_park < 0; e++) {
      const int u = PARK_SLOTS + ((my_cu + e) & (PARK_EXTRA - 1));
      if (atomicCAS(owners + u, 0ull, my_tag) == 0ull) my_park = u;
    }
    s_park = my_park;                               // read after the first transform's barriers
  }
  constexpr double TAU = 6.283185307179586;

  // ---- 1. raw samples -> z[m] = x[2m] + i x[2m+1]; forward FFT ---------------
  if (fmt == 0 || fmt == 1) {
    // thread t takes samples [16 t, 16 t + 16) with 16-byte loads (unaligned
    // global access): z[8 t + r] = (x[16 t + 2 r], x[16 t + 2 r + 1])
    double x[16];
    if (fmt == 0) {
      uint4 w;
      __builtin_memcpy(&w, cap + rel0 + 16 * tid, 16);
      const uint32_t wd[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int i = 0; i < 16; i++) x[i] = (double)((wd[i >> 2] >> (8 * (i & 3))) & 0xffu);
    } else {
      uint4 w[2];
      __builtin_memcpy(w, reinterpret_cast<const int16_t*>(cap) + rel0 + 16 * tid, 32);
      const uint32_t wd[8] = {w[0].x, w[0].y, w[0].z, w[0].w, w[1].x, w[1].y, w[1].z, w[1].w};
#pragma unroll
      for (int i = 0; i < 16; i++) x[i] = (double)(int16_t)(wd[i >> 1] >> (16 * (i & 1)));
    }
#pragma unroll
    for (int r = 0; r < 8; r++) X_[8 * tid + r] = make_double2(x[2 * r], x[2 * r + 1]);
  } else {
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int m = tid + T * q;
      X_[m] = make_double2(load_sample(cap, fmt, rel0 + 2 * m), load_sample(cap, fmt, rel0 + 2 * m + 1));
    }
  }
  STAMP(1);
  if (!(kProbe & 8)) fft8k_dif<false>(s_x, tw, twl, tid);
  else __syncthreads();
  STAMP(2);
  const bool park_lost = s_park < 0;
  double2* const park = ospill + (int64_t)(park_lost ? PARK_SCRATCH : s_park) * M;

  // ---- 2. analytic-signal spectra and the audio carrier slices ---------------
  // Y = X * RFVideo*MTF^m; the 16384-point IFFT of Y is done as its even/odd
  // (radix-2 DIF) halves: even half -> LDS, odd half -> ospill.  The audio
  // slices (lddecode_core.py:321-328, audio_fdslice lo [a0,a0+512), hi
  // mirrored) go to the separate 32 KiB audio buffer.  X dies here.
  // Spectra are digit-reversed here (fft8k.hpp); F and the filters are stored
  // in the same order (F[p] = bin dr_nat(p), F[M + p] = bin M + dr_nat(p)).
  {
    Pairs X;
    if (!(kProbe & 64)) split_pairs(X_, twk, tid, X);
    else for (int c = 0; c < 5; c++) { X.a[c] = X_[tid + 1024 * c]; X.b[c] = X.a[c]; }
    {
      // audio carrier slices (lddecode_core.py:321-328): thread t < 512 takes
      // bin k = a0 + t into slot j = t; thread t >= 512 the mirrored bin
      // k = a0 + 1 + (t - 512), conjugated, into slot j = a0 + 1024 - k
      const int t = fresh(tid);
      const int a0 = C.audio_lo0;
      const bool mir = t >= 512;
      const int k = mir ? a0 + 1 + (t - 512) : a0 + t;
      const int j = mir ? a0 + 1024 - k : t;
      double2 xk = rsplit(X_[dr_pos(k)], X_[dr_pos(M - k)], tw[k]);
      if (mir) xk = conj2(xk);
      const double2 al = cmul(xk, a_lfilt[j]), ar = cmul(xk, a_rfilt[j]);
      // per slot (a later call's demod must not overwrite slices ldg_k_audio1 has not read)
      double2* as = aslice + ((int64_t)slot * MAX_BLOCKS_PER_READ + b) * 2048;   // left [0,1024), right [1024,2048)
      as[j] = al;
      as[1024 + j] = ar;
    }
    __syncthreads();
    const int t = fresh(tid);
#pragma unroll
    for (int c = 0; c < 5; c++) {
      if (!pair_live(t, c) || (kProbe & 16)) continue;
      const Slot sl = slot_of(t, c);
      auto Fv = [&](int i) { return (kProbe & 128) ? make_double2(1.0 + i * 1e-9, 0.5) : F[i]; };
      const double2 wk = twk[sl.p];
      const double2 yk = cmul(X.a[c], Fv(sl.p));
      const double2 yk2 = cmul(conj2(X.b[c]), Fv(M + sl.p));
      X_[sl.p] = cadd(yk, yk2);
      if (!(kProbe & 256)) {
        const double2 o = cmulc(csub(yk, yk2), wk);
        st_park(park + SW(sl.p), o);
      }
      if (sl.pp != sl.p) {
        const double2 ykp = cmul(X.b[c], Fv(sl.pp));
        const double2 ykp2 = cmul(conj2(X.a[c]), Fv(M + sl.pp));
        X_[sl.pp] = cadd(ykp, ykp2);
        if (!(kProbe & 256)) st_park(park + SW(sl.pp), cmulc(csub(ykp, ykp2), tw_mirror(wk)));
      }
    }
  }

  STAMP(3);
  // (audio phase 1 -- 2 x IFFT1024 -> FM demod -- runs in ldg_k_audio1 on the
  // slices above: the demod keeps 128 KiB of LDS, so kernels with up to 32 KiB
  // share its CUs)
  // ---- 4. analytic IFFTs (even, odd) -> instantaneous phase --------------------
  // One loop body for both halves: one copy of the inverse FFT in the code (the
  // kernel would outgrow the instruction cache with every transform inlined).
  double the[8], tho[8];
#pragma clang loop unroll(disable)
  for (int h = 0; h < 2; h++) {
    STAMP(4 + 2 * h);
    // release the park: every wave's reload completed before the barrier that ended the
    // even half (vmcnt(0)), so no later store into it can reach this block's data
    if (h == 1 && tid == 0 && my_park >= 0)
      __hip_atomic_store(owners + my_park, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    double2 zr[8];
    fft8k_dit<true, true>(s_x, tw, twl, tid, zr);
    if (h == 0) {
      // the odd half returns to LDS while the even half's angles are computed:
      // every wave's park stores are complete (vmcnt) before any wave reads them
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const int t = fresh(tid);
      const int wbase = __builtin_amdgcn_readfirstlane(t & ~63);
#pragma unroll
      for (int i = 0; i < 8; i++)
        __builtin_amdgcn_global_load_lds((const void*)(park + T * i + t),
                                         (__attribute__((address_space(3))) void*)(s_x + T * i + wbase), 16, 0, 0);
    }
    STAMP(5 + 2 * h);
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const double2 z = zr[q];
      const double a = (kProbe & 1) ? z.y * 0.5 + z.x : kFastAtan2 ? fast_atan2(z.y, z.x, s_atan) : atan2(z.y, z.x);
      if (h) tho[q] = a;
      else the[q] = a;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

  }
  double* ph = reinterpret_cast<double*>(s_x);    // plain (unswizzled) phase scratch
#pragma unroll
  for (int q = 0; q < 8; q++) ph[tid + T * q] = tho[q];
  __syncthreads();

  STAMP(8);
  // ---- 5. FM demod (Hz) -> demod spectrum D (parked in ospill) ----------------------------------
  {
    const double hzk = C.freq_hz / TAU;
    double d0[8], d1[8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int m = tid + T * q;
      const double prev = m ? ph[m - 1] : 0.0;
      d0[q] = m ? fold_tau(the[q] - prev) * hzk : 0.0;
      d1[q] = fold_tau(tho[q] - the[q]) * hzk;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 8; q++) X_[tid + T * q] = make_double2(d0[q], d1[q]);
  }
  STAMP(9);
  fft8k_dif<false>(s_x, tw, twl, tid);
  STAMP(10);
  Pairs D;
  if (!(kProbe & 64)) split_pairs(X_, twk, tid, D);
  else for (int c = 0; c < 5; c++) { D.a[c] = X_[tid + 1024 * c]; D.b[c] = D.a[c]; }
  __syncthreads();
  STAMP(11);

  // ---- 6. output channels.
  //  a. demod_05 = C2R(D * FVideo05), rolled by -32 (lddecode_core.py:302-303),
  //     and its sync detector bits inrange(., iretohz(-55), iretohz(-25)) (:308)
  //     into an LDS bitmask;
  //  b. demod_sync: ifft(fft(bits) * FPsync) (:310) as the periodic recurrence
  //     of FPsync's butter(1) design (iir.hpp), not two more transforms;
  //  c. demod = C2R(D * FVideo);
  //  d. demod_burst (and PAL demod_pilot): FVideoBurst = FVideo * Fburst
  //     (:204-209), so the periodic recurrence of Fburst over demod (iir.hpp).
  const double inv = 1.0 / (double)M;
  double pl1, pt1, p151, p311;
  double2* sx = s_x;                             // chunk layout SWC (iir.hpp) from here on
  {
    if (!(kProbe & 32)) merge_pairs(X_, twk, g_05, tid, D);
    STAMP(12);
    double2 zr[8];                               // outputs at natural positions t + T q
    fft8k_dit<true, true>(s_x, tw, twl, tid, zr);
    STAMP(13);
    const int t = fresh(tid);
    // the sync scan's per-lane powers, loaded ahead of this phase's stores
    pl1 = iir[IIR_P1 + (t & 63)];
    pt1 = iir[IIR_P1 + t];
    p151 = iir[IIR_P1 + scan_d15(t & 63)];
    p311 = iir[IIR_P1 + scan_d31(t & 63)];
    // demod_05 is stored at full rate for refine_linelocs_hsync and the PAL pilot
    // windows (rebuilding those windows by the 65-tap FIR in the field kernels
    // instead measured 3.6% slower end to end, profiles/r03_z_d05_ab.txt)
    double* o = vout + (int64_t)CH_05 * vchan_stride;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int m = t + T * q;
      const double v0 = zr[q].x * inv, v1 = zr[q].y * inv;
      if (!kProbeNoStore) {
        // block position p lands at rolled position (p - 32) mod 16384 (even: p0 + 1 never wraps);
        // the wave's 64 pairs are all kept or all dropped except at the block ends
        const int p0 = (2 * m - BLOCKCUT_END) & (BLOCKLEN - 1);
        const int pw0 = (2 * (m & ~63) - BLOCKCUT_END) & (BLOCKLEN - 1);
        if (pw0 >= BLOCKCUT && pw0 + 127 < BLOCKCUT + copylen) {
          st_pair(o + p0, make_double2(v0, v1));
        } else {
          const bool in0 = p0 >= BLOCKCUT && p0 < BLOCKCUT + copylen;
          const bool in1 = p0 + 1 >= BLOCKCUT && p0 + 1 < BLOCKCUT + copylen;
          if (in0 && in1) *reinterpret_cast<double2*>(o + p0) = make_double2(v0, v1);
          else if (in0) o[p0] = v0;
          else if (in1) o[p0 + 1] = v1;
        }
      }
      // detector bits at UNROLLED block positions 2m, 2m + 1; lanes 8j..8j+7 (pairs
      // of 16 consecutive samples) OR their bits into lane 8j+7 (DPP row shifts)
      const uint32_t f0 = (v0 >= C.sync_lo && v0 <= C.sync_hi) ? 1u : 0u;
      const uint32_t f1 = (v1 >= C.sync_lo && v1 <= C.sync_hi) ? 1u : 0u;
      int xb = (int)((f0 | (f1 << 1)) << (2 * (t & 7)));
      xb |= __builtin_amdgcn_mov_dpp(xb, 0x111, 0xf, 0xf, true);   // row_shr:1
      xb |= __builtin_amdgcn_mov_dpp(xb, 0x112, 0xf, 0xf, true);   // row_shr:2
      xb |= __builtin_amdgcn_mov_dpp(xb, 0x114, 0xf, 0xf, true);   // row_shr:4
      if ((t & 7) == 7) s_bits[m >> 3] = (uint16_t)xb;
    }
  }
  __syncthreads();
  STAMP(14);
  {
    // sync: thread t owns ROLLED positions [16 t, 16 t + 16) = unrolled [16 t + 32, +16)
    const int t = fresh(tid);
    const uint32_t cur = s_bits[(t + 2) & 1023], prv = (uint32_t)s_bits[(t + 1) & 1023] >> 15;
    double y[IIR_CHUNK];
    double st_in = 0.0;
    if (!(kProbe & 4)) iir1_bits(cur, prv, iir, &s_aux, t, pl1, pt1, p151, p311, y, &st_in);
    else for (int i = 0; i < IIR_CHUNK; i++) y[i] = (double)((cur >> i) & 1) * pl1;
    // the compact channel (chan.hpp): the kept chunks' entering states and bits
    if (16 * t >= BLOCKCUT && 16 * t < BLOCKCUT + copylen) {
      const int64_t g = (int64_t)slot * CHUNKS_PER_SLOT + (off >> 4) + (t - BLOCKCUT / 16);
      sst[g] = st_in;
      sbits[g] = cur | (prv << 16);
    }
    // sync tiles (common.hpp SyncTile): tile j = outputs [off + 32 j, +32) =
    // block positions [1024 + 32 j, +32) = chunks of threads 64 + 2 j (+1); np.argmax
    // order, the lower half wins ties
    {
      const int j = (t >> 1) - 32, hf = t & 1;
      const int ntile = (copylen + 31) / 32;
      double v = -__builtin_inf();
      int64_t vi = 0x7fffffffffffffffLL;
      const int64_t n0 = (int64_t)off + 32 * j;
      if (j >= 0 && j < ntile) {
#pragma unroll
        for (int i = 0; i < IIR_CHUNK; i++) {
          const int e = 16 * hf + i;
          if (e < copylen - 32 * j && am_beats(y[i], n0 + e, v, vi)) { v = y[i]; vi = n0 + e; }
        }
      }
      const double ov = __shfl_xor(v, 1);
      const int64_t oi = __shfl_xor(vi, 1);
      if (am_beats(ov, oi, v, vi)) { v = ov; vi = oi; }
      if (j >= 0 && j < ntile && hf == 0) {
        SyncTile tt;
        tt.v = v;
        tt.idx = vi;
        stiles[(int64_t)slot * STILE_PER_SLOT + (n0 >> 5)] = tt;
      }
    }
  }
  STAMP(15);
  // past the read's video cut nothing reads the video, burst or pilot channel (the
  // field kernels check, FS_VCUT): the block ends after the sync channel
  if (CUT && (int64_t)off >= rd.vcut) {
    if (tid == 0 && park_lost) status[slot] = FS_MIGRATED;
    if (span && tid == 0) atomicMax(&span[1], (unsigned long long)__builtin_amdgcn_s_memrealtime());
    return;
  }
  double4 mlb, mtb, m15b, m31b;
  {
    if (!(kProbe & 32)) merge_pairs(X_, twk, g_video, tid, D);
    STAMP(16);
    double2 zr[8];
    if (!(kProbe & 2)) fft8k_dit<true, true>(s_x, tw, twl, tid, zr);
    else { __syncthreads(); for (int q = 0; q < 8; q++) zr[q] = s_x[tid + 1024 * q]; __syncthreads(); }
    STAMP(17);
    const int t = fresh(tid);
    mlb = iir2_pow(iir + IIR_MB, t & 63);     // the burst scan's powers, ahead of the stores
    mtb = iir2_pow(iir + IIR_MB, t);
    m15b = iir2_pow(iir + IIR_MB, scan_d15(t & 63));
    m31b = iir2_pow(iir + IIR_MB, scan_d31(t & 63));
    double* o = vout + (int64_t)CH_DEMOD * vchan_stride;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int m = t + T * q;
      const double2 z = make_double2(zr[q].x * inv, zr[q].y * inv);
      sx[SWC(m)] = z;
      if (!kProbeNoStore) store_pair(o, m, z, copylen);
    }
  }
  __syncthreads();
  STAMP(18);
  {
    const int t = fresh(tid);
    double x[IIR_CHUNK];
#pragma unroll
    for (int c = 0; c < 8; c++) {
      const double2 z = sx[SWC(8 * t + c)];
      x[2 * c] = z.x;
      x[2 * c + 1] = z.y;
    }
    const double2 h = sx[SWC((8 * t - 1) & (M - 1))];
    double y[IIR_CHUNK];
    double2 s_in = make_double2(0.0, 0.0);
    if (!(kProbe & 4)) iir2(x, h.y, h.x, iir + 3, iir + IIR_MB, &s_aux, t, mlb, mtb, m15b, m31b, y, &s_in);
    // the compact burst channel (chan.hpp): the kept chunks' entering states
    if (16 * t >= BLOCKCUT && 16 * t < BLOCKCUT + copylen) {
      const int64_t g = (int64_t)slot * CHUNKS_PER_SLOT + (off >> 4) + (t - BLOCKCUT / 16);
      bst[g] = make_double4(s_in.x, s_in.y, h.y, h.x);
    }
    if (C.n_chan > 4) {
      // PAL pilot from the same demod samples (still in x); iir2's barriers order
      // every thread's reads of sx above before the writes below
      double2 p_in;
      iir2(x, h.y, h.x, iir + 8, iir + IIR_MP, &s_aux, t, iir2_pow(iir + IIR_MP, t & 63), iir2_pow(iir + IIR_MP, t),
           iir2_pow(iir + IIR_MP, scan_d15(t & 63)), iir2_pow(iir + IIR_MP, scan_d31(t & 63)), y, &p_in);
#pragma unroll
      for (int c = 0; c < 8; c++) sx[SWC(8 * t + c)] = make_double2(y[2 * c], y[2 * c + 1]);
      __syncthreads();
      store_chan(sx, vout + (int64_t)CH_PILOT * vchan_stride, t, copylen);
    }
  }
  STAMP(19);
  if (tid == 0 && park_lost) status[slot] = FS_MIGRATED;
  if (span && tid == 0) atomicMax(&span[1], (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

extern "C" __global__ __launch_bounds__(1024) void ldg_k_demod(LDG_DEMOD_PARAMS) { demod_body<true>(LDG_DEMOD_ARGS); }

// The same kernel under its own name for the benchmark's isolated roofline leg
// (ldg_demod_isolated): its dispatches run alone on the GPU, so a kernel trace's
// per-dispatch average of this symbol is the figure bench.py measures with HIP
// events, undisturbed by the field kernels that co-run with ldg_k_demod.  It
// demodulates every block in full (no video cut): the leg times whole reads.
extern "C" __global__ __launch_bounds__(1024) void ldg_k_demod_iso(LDG_DEMOD_PARAMS) { demod_body<false>(LDG_DEMOD_ARGS); }
// The shipped body (video cut) for the same leg: ldg_demod_isolated_ex variant 1.
extern "C" __global__ __launch_bounds__(1024) void ldg_k_demod_iso_cut(LDG_DEMOD_PARAMS) { demod_body<true>(LDG_DEMOD_ARGS); }

// ---------------------------------------------------------------------------
// Read-start probes (speculative planning, not a reference stage).  A read's
// start is the previous field's nextfieldoffset: the absolute position of one
// sync peak, the argmax of demod_sync over a window of the previous read
// (lddecode_core.py:497-516, 926, 1204).  The planner predicts starts it has
// not decoded from the field period; on a capture whose sync peaks jitter by a
// sample or two (PAL: the trailing edge of the 0.5 MHz video through the
// -55..-25 IRE window falls on either side of a sample) those predictions miss
// and the read is decoded again.  A probe demodulates the one overlap-save
// block centred on a predicted start and takes the argmax of its demod_sync
// over +-0.3 lines around it: the peak the previous read's walk finds there
// (the peak is a sample position in the capture; other block alignments move
// demod_sync by far less than the peak's margin over its neighbours).  The
// read is then decoded from that start.  A probe can only change where a
// speculative read starts: the replay accepts a read only at the exact start
// the reference's chain reaches, so a wrong probe costs a decode, never a
// result.
constexpr int PROBE_C = BLOCKSTEP / 2;    // output index of the predicted start in the probe's block

extern "C" __global__ __launch_bounds__(1024) void ldg_k_demod_probe(LDG_DEMOD_PARAMS) {
  demod_body<true, true>(LDG_DEMOD_ARGS);
}

// One wave per probe: the argmax (first maximum) of the probe block's demod_sync
// over [PROBE_C - halfwin, PROBE_C + halfwin]; if its level passes the reference's
// peak test (> .2) the read in the same slot is moved to start there (its
// geometry as ldg_decode_reads_async2 sets it up).  The slot's status returns to
// 0: the probe's demod wrote into the read's own channels, which its full demod
// rewrites before any field kernel reads them.
extern "C" __global__ __launch_bounds__(64) void ldg_k_probe_pick(const int32_t* __restrict__ psm,
                                                                 const ReadDesc* __restrict__ preads,
                                                                 ReadDesc* __restrict__ reads,
                                                                 int32_t* __restrict__ status,
                                                                 const double* __restrict__ sst,
                                                                 const uint32_t* __restrict__ sbits, SysConst C,
                                                                 int halfwin) {
  const int slot = psm[blockIdx.x];
  const int lane = threadIdx.x;
  const bool eof = status[slot] == FS_EOF;
  const SyncSrc ds(sst, sbits, slot, C);
  double best = -1.0;
  int bi = 0x7fffffff;
  if (!eof) {
    for (int o = PROBE_C - halfwin + lane; o <= PROBE_C + halfwin; o += 64) {
      const double v = ds[o];
      if (v > best) { best = v; bi = o; }      // ascending o per lane: first maximum
    }
  }
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) {
    const double ov = __shfl_xor(best, m);
    const int oi = __shfl_xor(bi, m);
    if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
  }
  if (lane == 0) {
    if (!eof && best > 0.2) {
      ReadDesc r = reads[slot];
      const int64_t start = preads[slot].readsample + bi;
      r.readsample = start;
      r.end = start + READLEN + 1;
      r.s0 = start > BLOCKCUT ? start - BLOCKCUT : 0;
      r.n_out = (int32_t)(r.end - r.s0 + 1);
      r.n_blocks = (int32_t)((r.end - r.s0 + BLOCKSTEP - 1) / BLOCKSTEP);
      r.n_audio = (int32_t)((r.end - r.s0) / AUDIO_DIV1 + 1);
      r.n_audio2 = r.n_audio / AUDIO_DIV2;
      if (r.n_out <= MAX_NOUT && r.n_blocks <= MAX_BLOCKS_PER_READ) reads[slot] = r;
    }
    status[slot] = 0;
  }
}

// ---------------------------------------------------------------------------
// Audio phase 1 (lddecode_core.py:321-328): per overlap-save block, the two
// carrier slices the demod filtered (aslice, 2 x 1024 bins) -> 1024-point IFFT
// -> unwrap_hilbert at 2.5 MHz + the low carrier -> the block's kept audio
// samples.  grid: n_reads * MAX_BLOCKS_PER_READ workgroups of A1_T threads
// (threads [0, A1_T/2) left, [A1_T/2, A1_T) right), 32 KiB of LDS: a 1024-point
// radix-8 Stockham pass has 128 butterflies, so 128 threads per transform are
// all busy and four workgroups share a CU.
constexpr int A1_T = 256;
constexpr int A1_H = A1_T / 2;
constexpr int A1_P = 1024 / A1_H;      // points per thread
extern "C" __global__ __launch_bounds__(A1_T) void ldg_k_audio1(
    const int32_t* __restrict__ smap, const ReadDesc* __restrict__ reads, const double2* __restrict__ tw, SysConst C,
    const double2* __restrict__ aslice, double* __restrict__ audio1, int64_t aread_stride, int64_t achan_stride,
    const int32_t* __restrict__ status) {
  __shared__ double2 s_a[2048];
  const CBuf A_{s_a};
  const int tid = threadIdx.x;
  const int slot = smap[blockIdx.x / MAX_BLOCKS_PER_READ];
  const int b = blockIdx.x % MAX_BLOCKS_PER_READ;
  const ReadDesc rd = reads[slot];
  if (b >= rd.n_blocks || status[slot] == FS_EOF) return;
  const int off = b * BLOCKSTEP;
  const int copylen = (off + (BLOCKLEN - BLOCKCUT) > rd.n_out) ? rd.n_out - off : BLOCKSTEP;
  constexpr double TAU = 6.283185307179586;
  const double2* as = aslice + ((int64_t)slot * MAX_BLOCKS_PER_READ + b) * 2048;
  __shared__ double s_atan[65];
  if (tid < 65) s_atan[tid] = c_atan64[tid];   // ordered by the transform's first barrier
#pragma unroll
  for (int q = 0; q < 2048 / A1_T; q++) A_[tid + A1_T * q] = as[tid + A1_T * q];
  {
    const int g = tid / A1_H, lt = tid % A1_H;
    const CBuf ga = A_ + (g ? 1024 : 0);
    fft_lds<1024, A1_H, true>(ga, tw, lt);
    double th[A1_P];
#pragma unroll
    for (int e = 0; e < A1_P; e++) {
      const double2 z = ga[lt + A1_H * e];
      th[e] = kFastAtan2 ? fast_atan2(z.y, z.x, s_atan) : atan2(z.y, z.x);
    }
    __syncthreads();
    double* gth = reinterpret_cast<double*>(s_a) + (g ? 1024 : 0);     // plain (unswizzled) phase scratch
#pragma unroll
    for (int e = 0; e < A1_P; e++) gth[lt + A1_H * e] = th[e];
    __syncthreads();
    double* aout = audio1 + (int64_t)slot * aread_stride + (int64_t)g * achan_stride;
    const int kept = copylen / AUDIO_DIV1;
#pragma unroll
    for (int e = 0; e < A1_P; e++) {
      const int p = lt + A1_H * e;
      const double prev = p ? gth[p - 1] : 0.0;
      const double d = p ? fold_tau(th[e] - prev) : 0.0;
      const double v = d * (C.freq_arf / TAU) + C.audio_lowfreq;
      const int j = p - BLOCKCUT / AUDIO_DIV1;
      if (j >= 0 && j < kept) aout[off / AUDIO_DIV1 + j] = v;
    }
    // zero the tail the reference leaves at 0 (np.zeros) after the last block
    if (b == rd.n_blocks - 1) {
      const int last = (off + copylen) / AUDIO_DIV1;
      for (int j = last + lt; j < rd.n_audio; j += A1_H) aout[j] = 0.0;
    }
  }
}

// ---------------------------------------------------------------------------
// Audio phase 2 (lddecode_core.py:335-371): per (read, block, channel) a
// 16384-point real FFT of the 2.5 MHz audio, bins [0:2048]+[14336:16384]
// times audio_lpf2, 4096-point IFFT, real part / 4.
// grid: n_reads * AUDIO2_WG workgroups of 1024 threads: (block j < 4, channel)
// per read (a read's 2.5 MHz audio, at most MAX_NAUDIO samples, spans first +
// two middle + last blocks; the static_assert below holds that bound).
constexpr int AUDIO2_JMAX = 4;
constexpr int AUDIO2_WG = 2 * AUDIO2_JMAX;
static_assert((MAX_NAUDIO - 2 * (BLOCKLEN - 64 * AUDIO_DIV2) + (BLOCKLEN - 64 * AUDIO_DIV2) - 1) /
                          (BLOCKLEN - 64 * AUDIO_DIV2) + 2 <= AUDIO2_JMAX,
              "audio phase 2: a read needs more blocks than the grid has");
extern "C" __global__ __launch_bounds__(1024) void ldg_k_audio2(
    const int32_t* __restrict__ smap, const ReadDesc* __restrict__ reads, const double2* __restrict__ tw, const double2* __restrict__ lpf2,
    const double* __restrict__ audio1, int64_t aread_stride, int64_t achan_stride,
    double* __restrict__ audio2, int64_t a2read_stride, int64_t a2chan_stride, const int32_t* __restrict__ status) {
  __shared__ double2 s_x[M];
  __shared__ double2 s_tw[TW_LDS_N];
  const CBuf X_{s_x};
  const int tid = threadIdx.x;
  s_tw[tw_lds_pos(tid)] = tw[2 * tid];
  const TwLds twl{s_tw};
  const int ch = blockIdx.x & 1;
  const int j = (blockIdx.x >> 1) & (AUDIO2_JMAX - 1);
  const int slot = smap[blockIdx.x / AUDIO2_WG];
  if (status[slot] == FS_EOF) return;
  const ReadDesc rd = reads[slot];
  const int n_in = rd.n_audio, n_out = rd.n_audio2;
  constexpr int SKIP = 64;
  constexpr int JUMP = BLOCKLEN - SKIP * AUDIO_DIV2;     // 16128
  const int span = n_in - JUMP - JUMP;
  const int n_mid = span > 0 ? (span + JUMP - 1) / JUMP : 0;
  if (j > n_mid + 1) return;
  const int start = (j == 0) ? 0 : (j <= n_mid ? JUMP * j : n_in - BLOCKLEN - 1);
  const double* src = audio1 + (int64_t)slot * aread_stride + (int64_t)ch * achan_stride + start;
#pragma unroll
  for (int q = 0; q < 8; q++) {
    const int m = tid + T * q;
    X_[m] = make_double2(src[2 * m], src[2 * m + 1]);
  }
  fft8k_dif<false>(s_x, tw, twl, tid);     // digit-reversed out (fft8k.hpp)
  // X[k] for k in [0, 2048]
  double2 xa, xb, xc = make_double2(0, 0);
  {
    const int k1 = tid, k2 = tid + 1024;
    xa = rsplit(X_[dr_pos(k1)], X_[dr_pos((M - k1) & (M - 1))], tw[k1]);
    xb = rsplit(X_[dr_pos(k2)], X_[dr_pos(M - k2)], tw[k2]);
    if (tid == 0) xc = rsplit(X_[dr_pos(2048)], X_[dr_pos(M - 2048)], tw[2048]);
  }
  __syncthreads();
  // S[j] = X[j] (j < 2048); S[j] = conj(X[4096 - j]) (j >= 2048); times lpf2
  {
    const int ks[2] = {tid, tid + 1024};
    const double2 xs[2] = {xa, xb};
#pragma unroll
    for (int e = 0; e < 2; e++) {
      const int k = ks[e];
      X_[k] = cmul(xs[e], lpf2[k]);
      if (k >= 1) {
        const int jj = AUDIO2_BLOCK - k;
        X_[jj] = cmul(conj2(xs[e]), lpf2[jj]);
      }
    }
    if (tid == 0) X_[2048] = cmul(conj2(xc), lpf2[2048]);
  }
  fft_lds<AUDIO2_BLOCK, 512, true>(X_, tw, tid);   // threads >= 512 only join barriers
  double* dst = audio2 + (int64_t)slot * a2read_stride + (int64_t)ch * a2chan_stride;
  const double scale = 1.0 / (double)AUDIO2_BLOCK / (double)AUDIO_DIV2;
  const int last_start = n_out - (AUDIO2_BLOCK - SKIP);
#pragma unroll
  for (int e = 0; e < 4; e++) {
    const int p = tid + 1024 * e;
    const double v = X_[p].x * scale;
    int o;
    if (j == 0) {
      o = p;
      if (o >= last_start) continue;
    } else if (j <= n_mid) {
      if (p < SKIP) continue;
      o = AUDIO2_BLOCK + (AUDIO2_BLOCK - SKIP) * (j - 1) + (p - SKIP);
      if (o >= last_start) continue;
    } else {
      if (p < SKIP) continue;
      o = last_start + (p - SKIP);
    }
    if (o >= 0 && o < n_out) dst[o] = v;
  }
}

// Profiling: the device's constant-rate clock, read once (ldg_profile_enable's
// host-to-device clock calibration; out zeroed beforehand).
extern "C" __global__ void ldg_k_clock(unsigned long long* out) {
  if (threadIdx.x == 0) atomicMax(out, (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

// RF filter table for one mtf level: RFVideo * MTF**m (lddecode_core.py:290-293).
// m == 1 uses MTF itself (numpy's integer-power path); other m use
// exp(m*log|MTF|) * cis(m*arg MTF) (cpow = cexp(m*clog)).  m == 0: RFVideo.
extern "C" __global__ void ldg_k_rf_table(const double2* __restrict__ rfvideo, const double2* __restrict__ mtf,
                                           const double* __restrict__ mtf_logabs, const double* __restrict__ mtf_arg,
                                           const double* __restrict__ mtfs, double2* __restrict__ tables) {
  // grid: (BLOCKLEN / 256, n_tables); table y has mtf level mtfs[y].  Entry o
  // holds bin dr_nat(o) (o < M) or M + dr_nat(o - M): the order of the demod's
  // digit-reversed spectra.
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= BLOCKLEN) return;
  const int k = o < M ? dr_nat(o) : M + dr_nat(o - M);
  const double m = mtfs[blockIdx.y];
  double2* out = tables + (size_t)blockIdx.y * BLOCKLEN;
  const double2 r = rfvideo[k];
  double2 p;
  if (m == 0.0) {
    out[o] = r;
    return;
  }
  if (m == 1.0) p = mtf[k];
  else {
    const double mag = exp(m * mtf_logabs[k]);
    double s, c;
    sincos(m * mtf_arg[k], &s, &c);
    p = make_double2(mag * c, mag * s);
  }
  out[o] = cmul(r, p);
}
