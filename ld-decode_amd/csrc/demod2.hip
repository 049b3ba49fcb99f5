// RF demodulation, register-resident: one 512-thread workgroup per 16384-sample
// overlap-save block, two workgroups per CU.
//
// The same computation as demod.hip (RFDecode.demodblock + the block copy of
// RFDecode.demod, lddecode_core.py:288-330, 373-422; unwrap_hilbert,
// lddutils.py:320-334), with the same outputs (full-rate demod / demod_05 /
// PAL demod_pilot, compact sync and burst, sync tiles, audio slices), laid out
// for a workgroup that keeps its 8192-point transforms in REGISTERS
// (fft8k_h.hpp: 16 points per thread) and uses 64 KiB of LDS: a CU holds two
// demod workgroups, so one's barriers and LDS round trips overlap the other's
// FP64 work (the 1024-thread LDS design waited at barriers half the time, with
// nothing to switch to).
//
// Per block: raw R2C (forward transform + real split), the analytic spectrum as
// its even / odd DIF halves, two inverse transforms -> atan2 -> FM demod ->
// forward transform + split -> the demod_05 and video C2R spectra (merge) -> two
// inverse transforms.  A workgroup's registers hold one 8192-point array; the
// second array of each pair (the analytic odd half, the even half's phases,
// the video spectrum) waits in a park: a 320 KiB slot of a per-context pool,
// claimed by atomic bit at the start and released at the end, so it is private
// to the workgroup by construction (no CU-residency assumption).  Each thread
// parks and reloads only its own entries, in register order (coalesced).
//
// Spectral tables are stored per layout position (pos_of): F = RFVideo * MTF^m
// at the position's bin k and at k + 8192 (ldg_k_rf_table2), W_16384^k (twks),
// and the C2R filters (FVideo05, FVideo) at k and at 8192 - k (g2).
#include <hip/hip_runtime.h>
#include "common.hpp"
#include "fft8k_h.hpp"
#include "iir2h.hpp"
#include "chan.hpp"

using namespace ldg;

namespace {

#ifndef LDG_D2_WAVES
#define LDG_D2_WAVES 4                   // waves per SIMD: two 512-thread workgroups per CU
#endif
#ifndef D2_STOP
#define D2_STOP 99                       // (register-pressure experiments: return after phase D2_STOP)
#endif
constexpr int T5 = h8k::T;               // 512
constexpr int M5 = HALF;                 // 8192
// park slot layout (double2 units): the analytic odd half, the even half's phases
// (8192 doubles), the merged video spectrum
constexpr int P2_O = 0, P2_TH = 8192, P2_V = 12288;
constexpr int P2_N = 20480;              // 320 KiB per slot
constexpr int P2_WORDS = 64;             // claim bitmap words
constexpr int P2_SLOTS = 32 * P2_WORDS;  // slots per context

// Claim a free park slot (a bit of the bitmap), starting at word `key`.
__device__ int park2_claim(unsigned* bm, int key) {
  for (int probe = 0;; probe++) {
    const int wi = (key + probe) & (P2_WORDS - 1);
    unsigned cur = __hip_atomic_load(bm + wi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (~cur) {
      const int bit = __builtin_ctz(~cur);
      const unsigned old = atomicOr(bm + wi, 1u << bit);
      if (!(old & (1u << bit))) return wi * 32 + bit;
      cur = old | (1u << bit);
    }
    if (probe >= P2_WORDS) __builtin_amdgcn_s_sleep(16);   // every slot busy (never with <= 2 workgroups per CU)
  }
}

__device__ __forceinline__ void park2_release(unsigned* bm, int slot) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");        // this workgroup's park accesses are complete
  atomicAnd(bm + (slot >> 5), ~(1u << (slot & 31)));
}

__device__ __forceinline__ int cu_key() {
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
  const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
  return (int)((xcc & 7u) * 9u + ((hw >> 8) & 15u) + 3u * ((hw >> 13) & 7u));
}

// X[k] of the real 16384-point signal from Z = FFT_8192(x[2m] + i x[2m+1]):
// X = (A + conj B)/2 + w (-i/2)(A - conj B), A = Z[k], B = Z[M-k], w = W_2M^k.
__device__ __forceinline__ double2 rsplit2(double2 A, double2 B, double2 w) {
  const double2 e = make_double2(0.5 * (A.x + B.x), 0.5 * (A.y - B.y));
  const double2 d = make_double2(A.x - B.x, A.y + B.y);
  const double2 o = make_double2(0.5 * d.y, -0.5 * d.x);
  return cadd(e, cmul(w, o));
}
// Inverse of rsplit2: half spectrum (P[k], P[M-k]) -> Z[k] of the C2R's 8192-point IFFT.
__device__ __forceinline__ double2 cmerge2(double2 Pk, double2 Pkp, double2 w) {
  const double2 e = make_double2(0.5 * (Pk.x + Pkp.x), 0.5 * (Pk.y - Pkp.y));
  const double2 d = make_double2(Pk.x - Pkp.x, Pk.y + Pkp.y);
  const double2 o = cmulc(d, w);
  return make_double2(e.x - 0.5 * o.y, e.y + 0.5 * o.x);
}
__device__ __forceinline__ double2 tw_mirror2(double2 w) { return make_double2(-w.x, w.y); }   // W^(M-k) = -conj W^k

// Opaque copy (fresh per phase): table loads and addresses of a phase are not
// hoisted above its barriers into an earlier phase (register pressure).
__device__ __forceinline__ int fr(int x) {
  asm volatile("" : "+v"(x));
  return x;
}

__device__ __forceinline__ void sqd(double& x) { asm volatile("" : "+v"(x)); }
// pin z, and emit every memory access before this point here (the compiler would
// otherwise sink a loop's park stores to its end, keeping all their data live)
__device__ __forceinline__ void pinm(double2& z) { asm volatile("" : "+v"(z.x), "+v"(z.y)::"memory"); }

__device__ __forceinline__ double fold_tau2(double d) {
  constexpr double TAU = 6.283185307179586;
  return d < 0.0 ? d + TAU : d;
}

// wave 0's partners: sub-array 0 (bins 16 j) pairs j with (512 - j) mod 512, sub-array
// 1 (bins 8 + 16 j) j with 511 - j; the scratch holds a sub-array as [d][lane]
__device__ __forceinline__ int w0_partner(int s, int l, int d) {
  if (s == 1) return (7 - d) * 64 + (63 - l);
  const int j = ((l >> 3) + 8 * (l & 7)) + 64 * d;
  const int jp = (512 - j) & 511, jl = jp & 63;
  return (jp >> 6) * 64 + ((jl >> 3) + 8 * (jl & 7));
}

// Store the pair of samples 2m, 2m+1 of a channel (o indexed by block position) if
// kept ([BLOCKCUT, BLOCKCUT + copylen)); wave-uniform fast path as demod.hip.
__device__ __forceinline__ void st_pair2(double* o, int p, double2 z) {
  typedef double v2d __attribute__((ext_vector_type(2)));
  const v2d zv = {z.x, z.y};
  __builtin_nontemporal_store(zv, &h8k::at(reinterpret_cast<v2d*>(o), (unsigned)p >> 1));
}
__device__ __forceinline__ void store_pair2(double* o, int m, double2 z, int copylen) {
  const int p = 2 * m;
  const int pw0 = 2 * (m & ~63);
  if (pw0 >= BLOCKCUT && pw0 + 127 < BLOCKCUT + copylen) {
    st_pair2(o, p, z);
  } else if (pw0 + 127 >= BLOCKCUT && pw0 < BLOCKCUT + copylen) {
    const bool in0 = p >= BLOCKCUT && p < BLOCKCUT + copylen;
    const bool in1 = p + 1 >= BLOCKCUT && p + 1 < BLOCKCUT + copylen;
    if (in0 && in1) h8k::at(reinterpret_cast<double2*>(o), (unsigned)p >> 1) = z;
    else if (in0) h8k::at(o, p) = z.x;
    else if (in1) h8k::at(o, p + 1) = z.y;
  }
}

// demod_05 is rolled by -32 (lddecode_core.py:302-303): block position p holds unrolled p + 32.
__device__ __forceinline__ void store_pair05(double* o, int m, double2 z, int copylen) {
  const int p0 = (2 * m - BLOCKCUT_END) & (BLOCKLEN - 1);
  const int pw0 = (2 * (m & ~63) - BLOCKCUT_END) & (BLOCKLEN - 1);
  if (pw0 >= BLOCKCUT && pw0 + 127 < BLOCKCUT + copylen) {
    st_pair2(o, p0, z);
  } else {
    const bool in0 = p0 >= BLOCKCUT && p0 < BLOCKCUT + copylen;
    const bool in1 = p0 + 1 >= BLOCKCUT && p0 + 1 < BLOCKCUT + copylen;
    if (in0 && in1) h8k::at(reinterpret_cast<double2*>(o), (unsigned)p0 >> 1) = z;
    else if (in0) h8k::at(o, p0) = z.x;
    else if (in1) h8k::at(o, p0 + 1) = z.y;
  }
}

}  // namespace

// grid: n_reads * MAX_BLOCKS_PER_READ workgroups of 512 threads.
// rf2: [filt_slot][16384] (F at pos, F at pos's bin + 8192); twks: [8192]; g2, g2m:
// [8192] double4 (FVideo05, FVideo) at pos's bin / at 8192 - bin; parks: P2_SLOTS x P2_N
// double2; pbm: the claim bitmap (P2_WORDS words).
#define LDG_DEMOD2_PARAMS                                                                                       \
  const int32_t *__restrict__ smap, const ReadDesc *__restrict__ reads, const uint8_t *__restrict__ cap,        \
      int64_t cap_first, int64_t cap_nsamp, int fmt, const double2 *__restrict__ tw,                           \
      const double2 *__restrict__ twks, const double2 *__restrict__ rf2, const double4 *__restrict__ g2,        \
      const double4 *__restrict__ g2m, const double *__restrict__ iir, const double2 *__restrict__ a_lfilt,    \
      const double2 *__restrict__ a_rfilt, SysConst C, double *__restrict__ video, int64_t vread_stride,        \
      int64_t vchan_stride, int32_t *__restrict__ status, double2 *__restrict__ parks, unsigned *__restrict__ pbm, \
      SyncTile *__restrict__ stiles, double2 *__restrict__ aslice, double *__restrict__ sst,                    \
      uint32_t *__restrict__ sbits, double4 *__restrict__ bst, unsigned long long *__restrict__ span
#define LDG_DEMOD2_ARGS                                                                                         \
  smap, reads, cap, cap_first, cap_nsamp, fmt, tw, twks, rf2, g2, g2m, iir, a_lfilt, a_rfilt, C, video,         \
      vread_stride, vchan_stride, status, parks, pbm, stiles, aslice, sst, sbits, bst, span

template <bool CUT, bool PAL>
__device__ __forceinline__ void demod2_body(LDG_DEMOD2_PARAMS) {
  __shared__ double2 ex[h8k::EX];                 // 64 KiB: exchanges, wave scratch, staging
  __shared__ uint16_t s_bits[BLOCKLEN / 16];       // sync detector bits (unrolled positions)
  __shared__ IIRAux2 s_aux;
  __shared__ double s_atan[65];
  __shared__ double2 s_edge[2];                   // video (x[16382], x[16383]), (x[8190], x[8191])
  __shared__ int s_park;
  const int tid = threadIdx.x;
  if (tid < 65) s_atan[tid] = c_atan64[tid];      // ordered by the first transform's barriers
  if (span && tid == 0) atomicMax(&span[0], ~(unsigned long long)__builtin_amdgcn_s_memrealtime());
  const int slot = smap[blockIdx.x / MAX_BLOCKS_PER_READ];
  const int b = blockIdx.x % MAX_BLOCKS_PER_READ;
  const ReadDesc rd = reads[slot];
  if (b >= rd.n_blocks) return;
  const int64_t i0 = rd.s0 + (int64_t)b * BLOCKSTEP;
  const int off = b * BLOCKSTEP;
  const int copylen = (off + (BLOCKLEN - BLOCKCUT) > rd.n_out) ? rd.n_out - off : BLOCKSTEP;
  const int64_t rel0 = i0 - cap_first;
  if (rel0 < 0 || rel0 + BLOCKLEN > cap_nsamp) {
    if (tid == 0) status[slot] = FS_EOF;
    return;
  }
  // past the read's video cut nothing reads the video, burst or pilot channel (the
  // field kernels check, FS_VCUT): the block ends after the sync channel
  const bool vcut = CUT && (int64_t)off >= rd.vcut;
  if (tid == 0) s_park = park2_claim(pbm, cu_key());
  double* vout = video + (int64_t)slot * vread_stride + off - BLOCKCUT;   // index by block position p
  const double2* F = rf2 + (int64_t)rd.filt_slot * BLOCKLEN;
  constexpr double TAU = 6.283185307179586;
  int t = tid;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6), l = tid & 63;

  // ---- 1. raw samples, natural layout: v[r] = (x[2m], x[2m+1]), m = t + 512 r ----
  double2 v[16];
  if (fmt == 0) {
    if (!(rel0 & 1)) {
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const uint32_t u = *reinterpret_cast<const uint16_t*>(cap + rel0 + 2 * (t + T5 * r));
        v[r] = make_double2((double)(u & 0xffu), (double)(u >> 8));
      }
    } else {
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const uint8_t* p = cap + rel0 + 2 * (t + T5 * r);
        v[r] = make_double2((double)p[0], (double)p[1]);
      }
    }
  } else if (fmt == 1) {
    const int16_t* c16 = reinterpret_cast<const int16_t*>(cap) + rel0;
#pragma unroll
    for (int r = 0; r < 16; r++) v[r] = make_double2((double)c16[2 * (t + T5 * r)], (double)c16[2 * (t + T5 * r) + 1]);
  } else {
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int64_t s = rel0 + 2 * (t + T5 * r);
      double a0, a1;
      if (fmt == 2) {
        const uint32_t* c32 = reinterpret_cast<const uint32_t*>(cap);
        a0 = (double)((c32[s / 3] >> (10 * (int)(s % 3))) & 0x3ffu);
        a1 = (double)((c32[(s + 1) / 3] >> (10 * (int)((s + 1) % 3))) & 0x3ffu);
      } else {
        auto lds10 = [&](int64_t q) {
          const uint8_t* bb = cap + 5 * (q >> 2);
          const int k = (int)(q & 3);
          uint32_t u;
          if (k == 0) u = ((uint32_t)bb[0] << 2) | (bb[1] >> 6);
          else if (k == 1) u = ((uint32_t)(bb[1] & 0x3f) << 4) | (bb[2] >> 4);
          else if (k == 2) u = ((uint32_t)(bb[2] & 0x0f) << 6) | (bb[3] >> 2);
          else u = ((uint32_t)(bb[3] & 0x03) << 8) | bb[4];
          return (double)u;
        };
        a0 = lds10(s);
        a1 = lds10(s + 1);
      }
      v[r] = make_double2(a0, a1);
    }
  }
  h8k::fwd<false>(v, ex, tw, t);

  if (D2_STOP <= 1) { for (int i = 0; i < 16; i++) reinterpret_cast<double2*>(vout)[i * T5 + tid] = v[i]; return; }
  // ---- 2. real split, analytic spectrum halves, audio carrier slices --------------
  // Y = X * F (F = RFVideo * MTF^m); the 16384-point IFFT of Y as its DIF halves:
  // E[k] = Y[k] + Y[k+M] (inverse-transformed in registers), O[k] = (Y[k] - Y[k+M])
  // conj(W^k) (parked).  Y[k+M] = conj(X[M-k]) F[k+M].
  double2* mine = ex + 512 * w;
  const int pslot = __builtin_amdgcn_readfirstlane(s_park);   // (set before the transform's barriers)
  double2* park = parks + (int64_t)pslot * P2_N;
  const int a0 = C.audio_lo0;
  {
  const int l = fr(tid & 63), t = fr(tid);
  double2* as = aslice + ((int64_t)slot * MAX_BLOCKS_PER_READ + b) * 2048;   // left [0,1024), right [1024,2048)
  // one bin: X at bin k (Xk) and at M - k (Xm) -> E (returned), O (parked at register i), audio slices
  // (aud: the register can hold an audio-slice bin -- bins < 2048 -- so the branch is
  // compiled only there)
  auto analytic = [&](double2 Xk, double2 Xm, double2 wk, int pos, int k, int i, bool aud) -> double2 {
    const double2 y = cmul(Xk, h8k::at(F, pos)), yh = cmul(conj2(Xm), h8k::at(F, M5 + pos));
    h8k::at(park, P2_O + i * T5 + t) = cmulc(csub(y, yh), wk);
    if (aud && __builtin_expect(k >= a0 && k <= a0 + 512, 0)) {
      // audio_fdslice (lddecode_core.py:321-328): lo slot k - a0, hi (mirrored, conj) a0 + 1024 - k
      if (k < a0 + 512) {
        h8k::at(as, k - a0) = cmul(Xk, h8k::at(a_lfilt, k - a0));
        h8k::at(as, 1024 + k - a0) = cmul(Xk, h8k::at(a_rfilt, k - a0));
      }
      if (k > a0) {
        const int j = a0 + 1024 - k;
        h8k::at(as, j) = cmul(conj2(Xk), h8k::at(a_lfilt, j));
        h8k::at(as, 1024 + j) = cmul(conj2(Xk), h8k::at(a_rfilt, j));
      }
    }
    return cadd(y, yh);
  };
  if (w > 0) {
#pragma unroll
    for (int d = 0; d < 8; d++) {
      // one bin pair at a time (its loads issued after the previous pair's results:
      // interleaving all eight pairs would not fit the 128 registers)
      const int l = fr(tid & 63);
      const int p0 = h8k::pos_of(w, 0, l, d), p1 = h8k::pos_of(w, 1, l, 7 - d);
      const double2 A = v[d], B = v[15 - d];
      const double2 wk = h8k::at(twks, p0);
      const double2 Xk = rsplit2(A, B, wk), Xm = rsplit2(B, A, tw_mirror2(wk));
      v[d] = analytic(Xk, Xm, wk, p0, h8k::bin_of(w, 0, l, d), d, d < 2);
      v[15 - d] = analytic(Xm, Xk, tw_mirror2(wk), p1, h8k::bin_of(w, 1, l, 7 - d), 15 - d, d >= 6);
      h8k::pin(v[d]);
      pinm(v[15 - d]);
    }
  } else {
#pragma unroll
    for (int s = 0; s < 2; s++) {
#pragma unroll
      for (int d = 0; d < 8; d++) mine[d * 64 + l] = v[8 * s + d];
      h8k::wsync();
#pragma unroll
      for (int d = 0; d < 8; d++) {
        const int l = fr(tid & 63);
        const double2 P = mine[w0_partner(s, l, d)];   // (read before this register is overwritten: wave order)
        const int p = h8k::pos_of(0, s, l, d);
        const double2 wk = h8k::at(twks, p);
        const double2 Xk = rsplit2(v[8 * s + d], P, wk), Xm = rsplit2(P, v[8 * s + d], tw_mirror2(wk));
        v[8 * s + d] = analytic(Xk, Xm, wk, p, h8k::bin_of(0, s, l, d), 8 * s + d, d < 2);
        pinm(v[8 * s + d]);
      }
    }
  }

  }

  if (D2_STOP <= 2) { for (int i = 0; i < 16; i++) h8k::at(park, i * T5 + tid) = v[i]; return; }
  // ---- 3. analytic IFFT halves -> instantaneous phase -> FM demod (Hz) ------------
  double th[16];
  h8k::inv<true>(v, ex, tw, t);                   // even samples y[2m]
  {
    const int t = fr(tid);
#pragma unroll
    for (int r = 0; r < 16; r++) {
      double2 z = v[r];
      h8k::pin(z);                                // one atan2 at a time (registers)
      double a = fast_atan2(z.y, z.x, s_atan);
      sqd(a);
      h8k::at(reinterpret_cast<double*>(park + P2_TH), r * T5 + t) = a;
    }
  }
  {
    const int t = fr(tid);
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = h8k::at(park, P2_O + i * T5 + t);    // this thread's own parked entries
  }
  h8k::inv<true>(v, ex, tw, t);                   // odd samples y[2m + 1]
#pragma unroll
  for (int r = 0; r < 16; r++) {
    double2 z = v[r];
    h8k::pin(z);
    th[r] = fast_atan2(z.y, z.x, s_atan);
    sqd(th[r]);
  }
  {
    const int t = fr(tid);
    double* ph = reinterpret_cast<double*>(ex);   // the odd phases, for the previous sample of 2m
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; r++) ph[t + T5 * r] = th[r];
    __syncthreads();
    const double hzk = C.freq_hz / TAU;
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int m = t + T5 * r;
      const double the = h8k::at(reinterpret_cast<const double*>(park + P2_TH), r * T5 + t);
      const double prev = m ? ph[m - 1] : 0.0;
      v[r] = make_double2(m ? fold_tau2(the - prev) * hzk : 0.0, fold_tau2(th[r] - the) * hzk);
    }
  }
  h8k::fwd<false>(v, ex, tw, t);

  if (D2_STOP <= 3) { for (int i = 0; i < 16; i++) h8k::at(park, i * T5 + tid) = v[i]; return; }
  // ---- 4. demod spectrum D (split) -> C2R spectra of demod_05 and video (merge) ------
  // P[k] = merge(D[k] G[k], D[M-k] G[M-k]); the video's is parked (unless past the cut)
  {
  const int l = fr(tid & 63), t = fr(tid);
  if (w > 0) {
#pragma unroll
    for (int d = 0; d < 8; d++) {
      const int l = fr(tid & 63), t = fr(tid);
      const int p0 = h8k::pos_of(w, 0, l, d), p1 = h8k::pos_of(w, 1, l, 7 - d);
      const double2 A = v[d], B = v[15 - d];
      const double2 wk = h8k::at(twks, p0), wm = tw_mirror2(wk);
      const double2 Dk = rsplit2(A, B, wk), Dm = rsplit2(B, A, wm);
      const double4 Gk = h8k::at(g2, p0), Gm = h8k::at(g2, p1);
      const double2 fk = cmul(Dk, make_double2(Gk.x, Gk.y)), fm = cmul(Dm, make_double2(Gm.x, Gm.y));
      v[d] = cmerge2(fk, fm, wk);
      v[15 - d] = cmerge2(fm, fk, wm);
      if (!vcut) {
        const double2 gk = cmul(Dk, make_double2(Gk.z, Gk.w)), gm = cmul(Dm, make_double2(Gm.z, Gm.w));
        h8k::at(park, P2_V + d * T5 + t) = cmerge2(gk, gm, wk);
        h8k::at(park, P2_V + (15 - d) * T5 + t) = cmerge2(gm, gk, wm);
      }
      h8k::pin(v[d]);
      pinm(v[15 - d]);
    }
  } else {
#pragma unroll
    for (int s = 0; s < 2; s++) {
#pragma unroll
      for (int d = 0; d < 8; d++) mine[d * 64 + l] = v[8 * s + d];
      h8k::wsync();
#pragma unroll
      for (int d = 0; d < 8; d++) {
        const int l = fr(tid & 63), t = fr(tid);
        const double2 P = mine[w0_partner(s, l, d)];
        const int p = h8k::pos_of(0, s, l, d);
        const double2 wk = h8k::at(twks, p);
        const double2 Dk = rsplit2(v[8 * s + d], P, wk), Dm = rsplit2(P, v[8 * s + d], tw_mirror2(wk));
        const double4 Gk = h8k::at(g2, p), Gm = h8k::at(g2m, p);
        v[8 * s + d] = cmerge2(cmul(Dk, make_double2(Gk.x, Gk.y)), cmul(Dm, make_double2(Gm.x, Gm.y)), wk);
        if (!vcut)
          h8k::at(park, P2_V + (8 * s + d) * T5 + t) =
              cmerge2(cmul(Dk, make_double2(Gk.z, Gk.w)), cmul(Dm, make_double2(Gm.z, Gm.w)), wk);
        pinm(v[8 * s + d]);
      }
    }
  }

  }

  if (D2_STOP <= 4) { for (int i = 0; i < 16; i++) h8k::at(park, i * T5 + tid) = v[i]; return; }
  // ---- 5. demod_05 (C2R), its sync detector bits -> demod_sync (periodic IIR) ------
  const double inv = 1.0 / (double)M5;
  h8k::inv<true>(v, ex, tw, t);
  {
    const int t = fr(tid);
    double* o = vout + (int64_t)CH_05 * vchan_stride;
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int m = t + T5 * r;
      const double v0 = v[r].x * inv, v1 = v[r].y * inv;
      store_pair05(o, m, make_double2(v0, v1), copylen);
      // detector bits at unrolled block positions 2m, 2m + 1 (lddecode_core.py:308);
      // lanes 8j..8j+7 (16 consecutive samples) OR into lane 8j+7
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
  {
    const int l = fr(tid & 63), t = fr(tid);
    // sync: chunk c (ROLLED block positions [16 c, 16 c + 16) = unrolled [16 c + 32, +16)),
    // thread t owns chunks t (half A) and t + 512 (half B)
    const double* pw = iir + IIR_P1;
    const double b0 = iir[0], p = -iir[2];
    uint32_t cur[2], prv[2];
    double e[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int c = t + 512 * h;
      cur[h] = s_bits[(c + 2) & 1023];
      prv[h] = (uint32_t)s_bits[(c + 1) & 1023] >> 15;
      double st = 0.0;
      uint32_t pv = prv[h];
#pragma unroll
      for (int i = 0; i < IIR_CHUNK; i++) {
        const uint32_t x = (cur[h] >> i) & 1u;
        st = __fma_rn(p, st, b0 * (double)(x + pv));
        pv = x;
      }
      e[h] = st;
    }
    double sin_[2];
    iir1_scan2(e[0], e[1], pw, &s_aux, t, pw[l], pw[t], pw[scan_d15(l)], pw[scan_d31(l)], pw[512], &sin_[0], &sin_[1]);
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int c = t + 512 * h;
      // the compact channel (chan.hpp): the kept chunks' entering states and bits
      if (16 * c >= BLOCKCUT && 16 * c < BLOCKCUT + copylen) {
        const int64_t g = (int64_t)slot * CHUNKS_PER_SLOT + (off >> 4) + (c - BLOCKCUT / 16);
        sst[g] = sin_[h];
        sbits[g] = cur[h] | (prv[h] << 16);
      }
      // sync tiles (common.hpp SyncTile): tile j = outputs [off + 32 j, +32) = chunks 64 + 2 j
      // (+1): adjacent threads of one half; np.argmax order, the lower half wins ties
      const int j = (c >> 1) - 32, hf = c & 1;
      const int ntile = (copylen + 31) / 32;
      double vm = -__builtin_inf();
      int64_t vi = 0x7fffffffffffffffLL;
      const int64_t n0 = (int64_t)off + 32 * j;
      double st = sin_[h];
      uint32_t pv = prv[h];
#pragma unroll
      for (int i = 0; i < IIR_CHUNK; i++) {
        const uint32_t x = (cur[h] >> i) & 1u;
        st = sync_step(st, x, pv, b0, p);
        pv = x;
        const int ei = 16 * hf + i;
        if (j >= 0 && j < ntile && ei < copylen - 32 * j && am_beats(st, n0 + ei, vm, vi)) {
          vm = st;
          vi = n0 + ei;
        }
      }
      const double ov = __shfl_xor(vm, 1);
      const int64_t oi = __shfl_xor(vi, 1);
      if (am_beats(ov, oi, vm, vi)) {
        vm = ov;
        vi = oi;
      }
      if (j >= 0 && j < ntile && hf == 0) {
        SyncTile tt;
        tt.v = vm;
        tt.idx = vi;
        stiles[(int64_t)slot * STILE_PER_SLOT + (n0 >> 5)] = tt;
      }
    }
  }
  if (D2_STOP <= 5) { for (int i = 0; i < 16; i++) h8k::at(park, i * T5 + tid) = v[i]; return; }
  if (vcut) {
    __syncthreads();
    if (tid == 0) park2_release(pbm, pslot);
    if (span && tid == 0) atomicMax(&span[1], (unsigned long long)__builtin_amdgcn_s_memrealtime());
    return;
  }

  // ---- 6. video (C2R) -> demod channel; demod_burst (and PAL demod_pilot) ----------
  {
    const int t = fr(tid);
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = h8k::at(park, P2_V + i * T5 + t);
  }
  h8k::inv<true>(v, ex, tw, t);
  const int t6 = fr(tid), l6 = fr(tid & 63);
  {
    const int t = t6;
    double* o = vout + (int64_t)CH_DEMOD * vchan_stride;
#pragma unroll
    for (int r = 0; r < 16; r++) {
      v[r] = make_double2(v[r].x * inv, v[r].y * inv);
      store_pair2(o, t + T5 * r, v[r], copylen);
    }
  }
  // the chunk layout through LDS in two halves: chunk t6 of half h = samples
  // [8192 h + 16 t6, +16) = pairs m = 4096 h + 8 t6 + c, c < 8
  if (t6 == T5 - 1) {
    s_edge[0] = v[15];                              // (x[16382], x[16383])
    s_edge[1] = v[7];                               // (x[8190], x[8191])
  }
  double x[2][16];
  double2 hx[2];
#pragma unroll
  for (int h = 0; h < 2; h++) {
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 8; r++) ex[SWC(t6 + T5 * r)] = v[8 * h + r];
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 8; c++) {
      const double2 z = ex[SWC(8 * t6 + c)];
      x[h][2 * c] = z.x;
      x[h][2 * c + 1] = z.y;
    }
    hx[h] = t6 ? ex[SWC(8 * t6 - 1)] : s_edge[h ? 1 : 0];
  }
  {
    const double* pw = iir + IIR_MB;
    const double2 zero = make_double2(0.0, 0.0);
    const double2 eA = sos_chunk(x[0], hx[0].y, hx[0].x, zero, iir + 3, nullptr);
    const double2 eB = sos_chunk(x[1], hx[1].y, hx[1].x, zero, iir + 3, nullptr);
    double2 s_in[2];
    iir2_scan2(eA, eB, pw, &s_aux, t6, &s_in[0], &s_in[1]);
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int c = t6 + 512 * h;
      // the compact burst channel (chan.hpp): the kept chunks' entering states
      if (16 * c >= BLOCKCUT && 16 * c < BLOCKCUT + copylen) {
        const int64_t g = (int64_t)slot * CHUNKS_PER_SLOT + (off >> 4) + (c - BLOCKCUT / 16);
        bst[g] = make_double4(s_in[h].x, s_in[h].y, hx[h].y, hx[h].x);
      }
    }
    if (PAL) {
      // PAL pilot from the same demod samples, stored at full rate from the chunk layout
      const double* pp = iir + IIR_MP;
      const double2 fA = sos_chunk(x[0], hx[0].y, hx[0].x, zero, iir + 8, nullptr);
      const double2 fB = sos_chunk(x[1], hx[1].y, hx[1].x, zero, iir + 8, nullptr);
      double2 p_in[2];
      iir2_scan2(fA, fB, pp, &s_aux, t6, &p_in[0], &p_in[1]);
      double* o = vout + (int64_t)CH_PILOT * vchan_stride;
#pragma unroll
      for (int h = 0; h < 2; h++) {
        double y[IIR_CHUNK];
        sos_chunk(x[h], hx[h].y, hx[h].x, p_in[h], iir + 8, y);
        const int p0 = 16 * (t6 + 512 * h);
#pragma unroll
        for (int i = 0; i < IIR_CHUNK; i += 2) {
          const int p = p0 + i;
          if (p >= BLOCKCUT && p + 1 < BLOCKCUT + copylen) st_pair2(o, p, make_double2(y[i], y[i + 1]));
          else if (p >= BLOCKCUT && p < BLOCKCUT + copylen) h8k::at(o, p) = y[i];
          else if (p + 1 >= BLOCKCUT && p + 1 < BLOCKCUT + copylen) h8k::at(o, p + 1) = y[i + 1];
        }
      }
    }
  }
  __syncthreads();
  if (tid == 0) park2_release(pbm, pslot);
  if (span && tid == 0) atomicMax(&span[1], (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

extern "C" __global__ __launch_bounds__(512, LDG_D2_WAVES) void ldg_k_demod2(LDG_DEMOD2_PARAMS) {
  demod2_body<true, false>(LDG_DEMOD2_ARGS);
}
extern "C" __global__ __launch_bounds__(512, LDG_D2_WAVES) void ldg_k_demod2_pal(LDG_DEMOD2_PARAMS) {
  demod2_body<true, true>(LDG_DEMOD2_ARGS);
}
// the roofline leg's variants (ldg_demod_isolated): every block in full (no video cut)
extern "C" __global__ __launch_bounds__(512, LDG_D2_WAVES) void ldg_k_demod2_iso(LDG_DEMOD2_PARAMS) {
  demod2_body<false, false>(LDG_DEMOD2_ARGS);
}
extern "C" __global__ __launch_bounds__(512, LDG_D2_WAVES) void ldg_k_demod2_iso_pal(LDG_DEMOD2_PARAMS) {
  demod2_body<false, true>(LDG_DEMOD2_ARGS);
}

// RF filter table for one mtf level in the register layout: entry pos < M holds
// RFVideo * MTF**m at bin_of(pos), entry M + pos at that bin + M (lddecode_core.py:290-293;
// the arithmetic of ldg_k_rf_table).
extern "C" __global__ void ldg_k_rf_table2(const double2* __restrict__ rfvideo, const double2* __restrict__ mtf,
                                           const double* __restrict__ mtf_logabs, const double* __restrict__ mtf_arg,
                                           const double* __restrict__ mtfs, double2* __restrict__ tables) {
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= BLOCKLEN) return;
  const int pos = o & (M5 - 1);
  const int l = pos & 63, d = (pos >> 6) & 7, s = (pos >> 9) & 1, w = pos >> 10;
  const int k = h8k::bin_of(w, s, l, d) + (o >= M5 ? M5 : 0);
  const double m = mtfs[blockIdx.y];
  double2* out = tables + (size_t)blockIdx.y * BLOCKLEN;
  const double2 r = rfvideo[k];
  if (m == 0.0) {
    out[o] = r;
    return;
  }
  double2 p;
  if (m == 1.0) p = mtf[k];
  else {
    const double mag = exp(m * mtf_logabs[k]);
    double s_, c_;
    sincos(m * mtf_arg[k], &s_, &c_);
    p = make_double2(mag * c_, mag * s_);
  }
  out[o] = cmul(r, p);
}
