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
// one C2R per output filter (video, burst, [pilot], 0.5 MHz), sync R2C, sync
// C2R  = 9 (NTSC) / 10 (PAL); plus 2 x 1024-point audio IFFTs.
#include <hip/hip_runtime.h>
#include "common.hpp"
#include "fft.hpp"

using namespace ldg;

namespace {

constexpr int T = 1024;
constexpr int M = HALF;           // 8192
constexpr int LDSN = M + M / 8;   // padded

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

struct Pairs {
  double2 a[5], b[5];   // value at k and at M-k of each pair slot
};

__device__ __forceinline__ int pair_k(int tid, int q) { return q < 4 ? tid + 1024 * q : 4096; }
__device__ __forceinline__ bool pair_live(int tid, int q) { return q < 4 || tid == 0; }

// Half-spectrum of the real signal currently transformed in LDS, for my pairs.
__device__ __forceinline__ void split_pairs(const double* re, const double* im, const double2* __restrict__ tw,
                                            int tid, Pairs& X) {
#pragma unroll
  for (int q = 0; q < 5; q++) {
    if (!pair_live(tid, q)) continue;
    const int k = pair_k(tid, q), kp = M - k;
    const double2 A = make_double2(re[PAD(k)], im[PAD(k)]);
    const double2 B = make_double2(re[PAD(kp & (M - 1))], im[PAD(kp & (M - 1))]);
    X.a[q] = rsplit(A, B, tw[k]);
    X.b[q] = rsplit(B, A, tw[kp]);
  }
}

// Write merge(D * G) for my pairs into LDS (input of a C2R inverse FFT).
__device__ __forceinline__ void merge_filtered(double* re, double* im, const double2* __restrict__ tw,
                                               const double2* __restrict__ G, int tid, const Pairs& D) {
#pragma unroll
  for (int q = 0; q < 5; q++) {
    if (!pair_live(tid, q)) continue;
    const int k = pair_k(tid, q), kp = M - k;
    const double2 Pk = cmul(D.a[q], G[k]);
    const double2 Pkp = cmul(D.b[q], G[kp]);
    const double2 zk = cmerge(Pk, Pkp, tw[k]);
    re[PAD(k)] = zk.x; im[PAD(k)] = zk.y;
    if (kp < M && kp != k) {
      const double2 zkp = cmerge(Pkp, Pk, tw[kp]);
      re[PAD(kp)] = zkp.x; im[PAD(kp)] = zkp.y;
    }
  }
}

}  // namespace

// grid: n_reads * MAX_BLOCKS_PER_READ workgroups of 1024 threads.
extern "C" __global__ __launch_bounds__(1024) void ldg_k_demod(
    const int32_t* __restrict__ smap, const ReadDesc* __restrict__ reads, const uint8_t* __restrict__ cap, int64_t cap_first, int64_t cap_nsamp,
    int fmt, const double2* __restrict__ tw, const double2* __restrict__ rf_filt,
    const double2* __restrict__ g_video, const double2* __restrict__ g_05, const double2* __restrict__ g_burst,
    const double2* __restrict__ g_pilot, const double2* __restrict__ g_psync,
    const double2* __restrict__ a_lfilt, const double2* __restrict__ a_rfilt, SysConst C,
    double* __restrict__ video, int64_t vread_stride, int64_t vchan_stride,
    double* __restrict__ audio1, int64_t aread_stride, int64_t achan_stride, int32_t* __restrict__ status) {
  __shared__ double s_re[LDSN];
  __shared__ double s_im[LDSN];
  const int tid = threadIdx.x;
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
  double* vout = video + (int64_t)slot * vread_stride + off - BLOCKCUT;   // index by block position p
  const double2* F = rf_filt + (int64_t)rd.filt_slot * BLOCKLEN;
  constexpr double TAU = 6.283185307179586;

  // ---- 1. raw samples -> z[m] = x[2m] + i x[2m+1]; forward FFT ---------------
#pragma unroll
  for (int q = 0; q < 8; q++) {
    const int m = tid + T * q;
    s_re[PAD(m)] = load_sample(cap, fmt, rel0 + 2 * m);
    s_im[PAD(m)] = load_sample(cap, fmt, rel0 + 2 * m + 1);
  }
  fft_lds<M, T, false>(s_re, s_im, tw, tid);

  Pairs X;
  split_pairs(s_re, s_im, tw, tid, X);
  __syncthreads();

  // ---- 2. audio phase 1: carrier slices -> 2 x IFFT1024 -> FM demod ------------
  // lddecode_core.py:321-328; slices audio_fdslice (lo [a0,a0+512), hi mirrored).
  {
    const int a0 = C.audio_lo0;
    double* LR = s_re;            // left at [0,1024), right at [1024,2048) (padded)
    double* LI = s_im;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int k = pair_k(tid, q);
      const double2 xk = X.a[q];
      if (k >= a0 && k < a0 + 512) {
        const int j = k - a0;
        const double2 l = cmul(xk, a_lfilt[j]), r = cmul(xk, a_rfilt[j]);
        LR[PAD(j)] = l.x; LI[PAD(j)] = l.y;
        LR[PAD(1024 + j)] = r.x; LI[PAD(1024 + j)] = r.y;
      }
      if (k > a0 && k <= a0 + 512) {
        const int j = a0 + 1024 - k;
        const double2 xc = conj2(xk);
        const double2 l = cmul(xc, a_lfilt[j]), r = cmul(xc, a_rfilt[j]);
        LR[PAD(j)] = l.x; LI[PAD(j)] = l.y;
        LR[PAD(1024 + j)] = r.x; LI[PAD(1024 + j)] = r.y;
      }
    }
    const int g = tid >> 9, lt = tid & 511;
    double* gre = s_re + (g ? PAD(1024) : 0);
    double* gim = s_im + (g ? PAD(1024) : 0);
    fft_lds<1024, 512, true>(gre, gim, tw, lt);
    double th[2];
#pragma unroll
    for (int e = 0; e < 2; e++) { const int p = lt + 512 * e; th[e] = atan2(gim[PAD(p)], gre[PAD(p)]); }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 2; e++) gre[PAD(lt + 512 * e)] = th[e];
    __syncthreads();
    double* aout = audio1 + (int64_t)slot * aread_stride + (int64_t)g * achan_stride;
    const int kept = copylen / AUDIO_DIV1;
#pragma unroll
    for (int e = 0; e < 2; e++) {
      const int p = lt + 512 * e;
      const double prev = p ? gre[PAD(p - 1)] : 0.0;
      const double d = p ? fold_tau(th[e] - prev) : 0.0;
      const double v = d * (C.freq_arf / TAU) + C.audio_lowfreq;
      const int j = p - BLOCKCUT / AUDIO_DIV1;
      if (j >= 0 && j < kept) aout[off / AUDIO_DIV1 + j] = v;
    }
    // zero the tail the reference leaves at 0 (np.zeros) after the last block
    if (b == rd.n_blocks - 1) {
      const int last = (off + copylen) / AUDIO_DIV1;
      for (int j = last + lt; j < rd.n_audio; j += 512) aout[j] = 0.0;
    }
    __syncthreads();
  }

  // ---- 3. analytic signal: Y = X * RFVideo*MTF^m; IFFT16384 via even/odd halves --
  Pairs O;
#pragma unroll
  for (int q = 0; q < 5; q++) {
    if (!pair_live(tid, q)) continue;
    const int k = pair_k(tid, q), kp = M - k;
    const double2 yk = cmul(X.a[q], F[k]);
    const double2 yk2 = cmul(conj2(X.b[q]), F[k + M]);
    const double2 ek = cadd(yk, yk2);
    O.a[q] = cmulc(csub(yk, yk2), tw[k]);
    s_re[PAD(k)] = ek.x; s_im[PAD(k)] = ek.y;
    if (kp < M && kp != k) {
      const double2 ykp = cmul(X.b[q], F[kp]);
      const double2 ykp2 = cmul(conj2(X.a[q]), F[kp + M]);
      const double2 ekp = cadd(ykp, ykp2);
      O.b[q] = cmulc(csub(ykp, ykp2), tw[kp]);
      s_re[PAD(kp)] = ekp.x; s_im[PAD(kp)] = ekp.y;
    }
  }
  fft_lds<M, T, true>(s_re, s_im, tw, tid);
  double the[8], tho[8];
#pragma unroll
  for (int q = 0; q < 8; q++) { const int m = tid + T * q; the[q] = atan2(s_im[PAD(m)], s_re[PAD(m)]); }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 5; q++) {
    if (!pair_live(tid, q)) continue;
    const int k = pair_k(tid, q), kp = M - k;
    s_re[PAD(k)] = O.a[q].x; s_im[PAD(k)] = O.a[q].y;
    if (kp < M && kp != k) { s_re[PAD(kp)] = O.b[q].x; s_im[PAD(kp)] = O.b[q].y; }
  }
  fft_lds<M, T, true>(s_re, s_im, tw, tid);
#pragma unroll
  for (int q = 0; q < 8; q++) { const int m = tid + T * q; tho[q] = atan2(s_im[PAD(m)], s_re[PAD(m)]); }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 8; q++) s_re[PAD(tid + T * q)] = tho[q];
  __syncthreads();

  // ---- 4. FM demod (Hz) -> demod spectrum D ----------------------------------
  {
    const double hzk = C.freq_hz / TAU;
    double d0[8], d1[8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int m = tid + T * q;
      const double prev = m ? s_re[PAD(m - 1)] : 0.0;
      d0[q] = m ? fold_tau(the[q] - prev) * hzk : 0.0;
      d1[q] = fold_tau(tho[q] - the[q]) * hzk;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 8; q++) { const int m = tid + T * q; s_re[PAD(m)] = d0[q]; s_im[PAD(m)] = d1[q]; }
  }
  fft_lds<M, T, false>(s_re, s_im, tw, tid);
  Pairs D;
  split_pairs(s_re, s_im, tw, tid, D);
  __syncthreads();

  const double inv = 1.0 / (double)M;
  auto emit = [&](int ch, const double2* G) {
    merge_filtered(s_re, s_im, tw, G, tid, D);
    fft_lds<M, T, true>(s_re, s_im, tw, tid);
    double* o = vout + (int64_t)ch * vchan_stride;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int m = tid + T * q;
      const int p = 2 * m;
      if (p >= BLOCKCUT && p < BLOCKCUT + copylen) o[p] = s_re[PAD(m)] * inv;
      if (p + 1 >= BLOCKCUT && p + 1 < BLOCKCUT + copylen) o[p + 1] = s_im[PAD(m)] * inv;
    }
    __syncthreads();
  };
  emit(CH_DEMOD, g_video);
  emit(CH_BURST, g_burst);
  if (C.n_chan > 4) emit(CH_PILOT, g_pilot);

  // ---- 5. 0.5 MHz channel (rolled by -F05_offset) and the sync detector --------
  merge_filtered(s_re, s_im, tw, g_05, tid, D);
  fft_lds<M, T, true>(s_re, s_im, tw, tid);
  {
    double v0[8], v1[8];
#pragma unroll
    for (int q = 0; q < 8; q++) { const int m = tid + T * q; v0[q] = s_re[PAD(m)] * inv; v1[q] = s_im[PAD(m)] * inv; }
    __syncthreads();
    double* o = vout + (int64_t)CH_05 * vchan_stride;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int m = tid + T * q;
      // value at block position p lands at rolled position (p - 32) mod 16384
      const int p0 = (2 * m - BLOCKCUT_END) & (BLOCKLEN - 1);
      const int p1 = (2 * m + 1 - BLOCKCUT_END) & (BLOCKLEN - 1);
      if (p0 >= BLOCKCUT && p0 < BLOCKCUT + copylen) o[p0] = v0[q];
      if (p1 >= BLOCKCUT && p1 < BLOCKCUT + copylen) o[p1] = v1[q];
      // inrange(demod_05, iretohz(-55), iretohz(-25)) as 0/1 doubles
      const int mz = (m - BLOCKCUT_END / 2) & (M - 1);
      s_re[PAD(mz)] = (v0[q] >= C.sync_lo && v0[q] <= C.sync_hi) ? 1.0 : 0.0;
      s_im[PAD(mz)] = (v1[q] >= C.sync_lo && v1[q] <= C.sync_hi) ? 1.0 : 0.0;
    }
  }
  fft_lds<M, T, false>(s_re, s_im, tw, tid);
  split_pairs(s_re, s_im, tw, tid, D);
  __syncthreads();
  emit(CH_SYNC, g_psync);
}

// ---------------------------------------------------------------------------
// Audio phase 2 (lddecode_core.py:335-371): per (read, block, channel) a
// 16384-point real FFT of the 2.5 MHz audio, bins [0:2048]+[14336:16384]
// times audio_lpf2, 4096-point IFFT, real part / 4.
// grid: n_reads * 8 * 2 workgroups of 1024 threads.
extern "C" __global__ __launch_bounds__(1024) void ldg_k_audio2(
    const int32_t* __restrict__ smap, const ReadDesc* __restrict__ reads, const double2* __restrict__ tw, const double2* __restrict__ lpf2,
    const double* __restrict__ audio1, int64_t aread_stride, int64_t achan_stride,
    double* __restrict__ audio2, int64_t a2read_stride, int64_t a2chan_stride, const int32_t* __restrict__ status) {
  __shared__ double s_re[LDSN];
  __shared__ double s_im[LDSN];
  const int tid = threadIdx.x;
  const int ch = blockIdx.x & 1;
  const int j = (blockIdx.x >> 1) & 7;
  const int slot = smap[blockIdx.x >> 4];
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
    s_re[PAD(m)] = src[2 * m];
    s_im[PAD(m)] = src[2 * m + 1];
  }
  fft_lds<M, T, false>(s_re, s_im, tw, tid);
  // X[k] for k in [0, 2048]
  double2 xa, xb, xc = make_double2(0, 0);
  {
    const int k1 = tid, k2 = tid + 1024;
    xa = rsplit(make_double2(s_re[PAD(k1)], s_im[PAD(k1)]),
                make_double2(s_re[PAD((M - k1) & (M - 1))], s_im[PAD((M - k1) & (M - 1))]), tw[k1]);
    xb = rsplit(make_double2(s_re[PAD(k2)], s_im[PAD(k2)]),
                make_double2(s_re[PAD(M - k2)], s_im[PAD(M - k2)]), tw[k2]);
    if (tid == 0)
      xc = rsplit(make_double2(s_re[PAD(2048)], s_im[PAD(2048)]),
                  make_double2(s_re[PAD(M - 2048)], s_im[PAD(M - 2048)]), tw[2048]);
  }
  __syncthreads();
  // S[j] = X[j] (j < 2048); S[j] = conj(X[4096 - j]) (j >= 2048); times lpf2
  {
    const int ks[2] = {tid, tid + 1024};
    const double2 xs[2] = {xa, xb};
#pragma unroll
    for (int e = 0; e < 2; e++) {
      const int k = ks[e];
      const double2 s = cmul(xs[e], lpf2[k]);
      s_re[PAD(k)] = s.x; s_im[PAD(k)] = s.y;
      if (k >= 1) {
        const int jj = AUDIO2_BLOCK - k;
        const double2 t = cmul(conj2(xs[e]), lpf2[jj]);
        s_re[PAD(jj)] = t.x; s_im[PAD(jj)] = t.y;
      }
    }
    if (tid == 0) {
      const double2 t = cmul(conj2(xc), lpf2[2048]);
      s_re[PAD(2048)] = t.x; s_im[PAD(2048)] = t.y;
    }
  }
  fft_lds<AUDIO2_BLOCK, 512, true>(s_re, s_im, tw, tid);   // threads >= 512 only join barriers
  double* dst = audio2 + (int64_t)slot * a2read_stride + (int64_t)ch * a2chan_stride;
  const double scale = 1.0 / (double)AUDIO2_BLOCK / (double)AUDIO_DIV2;
  const int last_start = n_out - (AUDIO2_BLOCK - SKIP);
#pragma unroll
  for (int e = 0; e < 4; e++) {
    const int p = tid + 1024 * e;
    const double v = s_re[PAD(p)] * scale;
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

// RF filter table for one mtf level: RFVideo * MTF**m (lddecode_core.py:290-293).
// m == 1 uses MTF itself (numpy's integer-power path); other m use
// exp(m*log|MTF|) * cis(m*arg MTF) (cpow = cexp(m*clog)).  m == 0: RFVideo.
extern "C" __global__ void ldg_k_rf_table(const double2* __restrict__ rfvideo, const double2* __restrict__ mtf,
                                           const double* __restrict__ mtf_logabs, const double* __restrict__ mtf_arg,
                                           double m, double2* __restrict__ out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= BLOCKLEN) return;
  const double2 r = rfvideo[k];
  double2 p;
  if (m == 0.0) { out[k] = r; return; }
  if (m == 1.0) p = mtf[k];
  else {
    const double mag = exp(m * mtf_logabs[k]);
    double s, c;
    sincos(m * mtf_arg[k], &s, &c);
    p = make_double2(mag * c, mag * s);
  }
  out[k] = cmul(r, p);
}
