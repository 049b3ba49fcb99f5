// Periodic steady state of a low-order recursive filter over one circular
// overlap-save block, in the time domain.
//
// The reference filters three demod channels with frequency responses that are
// freqz samples of IIR designs (lddutils.filtfft = freqz(b, a, 16384, whole),
// lddutils.py:256-257):
//   demod_sync  = ifft(fft(bits) * FPsync),          FPsync = butter(1, 50 kHz)   lddecode_core.py:211-214,310
//   demod_burst = ifft(D * FVideo * Fburst),         Fburst = butter(1, fsc+-0.1) :204-205,305
//   demod_pilot = ifft(D * FVideo * Fpilot)  (PAL),  Fpilot = butter(1, 3.7-3.8)  :207-209,313
// H(w_k) = B(e^-iw_k)/A(e^-iw_k) is the DFT of the filter's impulse response
// folded onto the 16384-sample circle, so ifft(fft(x) * H) is exactly the
// periodic solution of the recurrence A y = B x on the circular block.  That
// replaces an FFT + inverse FFT (sync) or an inverse FFT (burst, pilot, whose
// input demod = ifft(D * FVideo) is computed anyway) by one chunked linear scan.
//
// Work split: thread t of the 1024-thread workgroup owns samples [16t, 16t+16).
//   1. the chunk's recurrence from a zero state gives its end state e_t;
//   2. states entering each chunk: S_{t+1} = C^16 S_t + e_t, an affine scan
//      (Kogge-Stone over the wave, then over the 16 wave totals), C the
//      companion matrix of A;
//   3. the circle: the state entering sample 0 is the state after sample 16383,
//      i.e. the scan's total E (the exact value E / (1 - C^16384) differs by
//      |pole|^16384 < 1e-55 relative), added to chunk t as C^(16t) E;
//   4. the chunk's recurrence again from its true state gives the outputs.
// The powers C^(16 s), s = 0..1024, are built on the host (ldg_set_filters).
// Agreement with the FFT form is ~1e-14 relative (rounding of either method).
#pragma once
#include <hip/hip_runtime.h>

namespace ldg {

constexpr int IIR_CHUNK = 16;
// Layout of the host-built coefficient table (doubles):
//   [0..2]   FPsync  b0, b1, a1
//   [3..7]   Fburst  b0, b1, b2, a1, a2
//   [8..12]  Fpilot  b0, b1, b2, a1, a2  (PAL; zeros for NTSC)
//   IIR_P1:  p^(16 s), p = -a1 of FPsync, s = 0..1024
//   IIR_MB:  C^(16 s) of Fburst, row-major (m00, m01, m10, m11), s = 0..1024
//   IIR_MP:  the same for Fpilot
constexpr int IIR_NCOEF = 13;
constexpr int IIR_NPOW = 1025;
constexpr int IIR_P1 = 16;
constexpr int IIR_MB = IIR_P1 + 1040;
constexpr int IIR_MP = IIR_MB + 4 * 1028;
constexpr int IIR_TAB_N = IIR_MP + 4 * 1028;

// LDS scratch of a scan: wave totals and the states entering each wave.
struct IIRAux {
  double tot[16][2];
  double k[17][2];
};

// Chunk layout in LDS: double2 index u (samples 2u, 2u+1) lives at SWC(u).
// Conflict-free both for the pair-per-lane layout u = t + 1024 q (ds_write_b128 /
// ds_read_b128) and for the chunk-per-lane layout u = 8 t + c.
__device__ __forceinline__ constexpr int SWC(int u) { return u ^ ((u >> 3) & 15); }

// States entering each wave and the block total, from the per-wave inclusive
// totals (written to aux->tot by lane 63 of each wave).  ORD = state size.
template <int ORD>
__device__ __forceinline__ void iir_wave_carries(IIRAux* aux, const double* __restrict__ pw, int tid) {
  __syncthreads();
  if (tid < 64) {
    const int lane = tid;
    double k0 = lane < 16 ? aux->tot[lane][0] : 0.0;
    double k1 = (ORD == 2 && lane < 16) ? aux->tot[lane][1] : 0.0;
#pragma unroll
    for (int d = 1; d < 16; d <<= 1) {
      const double u0 = __shfl_up(k0, d);
      const double u1 = ORD == 2 ? __shfl_up(k1, d) : 0.0;
      if (lane >= d) {
        if constexpr (ORD == 1) {
          k0 = __fma_rn(pw[64 * d], u0, k0);
        } else {
          const double* m = pw + 4 * (64 * d);
          const double n0 = __fma_rn(m[0], u0, __fma_rn(m[1], u1, k0));
          const double n1 = __fma_rn(m[2], u0, __fma_rn(m[3], u1, k1));
          k0 = n0;
          k1 = n1;
        }
      }
    }
    if (lane < 16) {
      aux->k[lane + 1][0] = k0;
      if (ORD == 2) aux->k[lane + 1][1] = k1;
    }
    if (lane == 0) {
      aux->k[0][0] = 0.0;
      aux->k[0][1] = 0.0;
    }
  }
  __syncthreads();
}

// FPsync over the sync detector bits: y[n] = b0 (x[n] + x[n-1]) + p y[n-1].
// bits: bit i = x[16t + i]; xm1 = x[16t - 1].  y[i] = y[16t + i].
// pl, pt: the table's p^(16 lane), p^(16 t), loaded by the caller (ahead of
// its global stores: a load issued after them waits for them).
__device__ __forceinline__ void iir1_bits(uint32_t bits, uint32_t xm1, const double* __restrict__ tab, IIRAux* aux,
                                          int tid, double pl, double pt, double* y) {
  const double b0 = tab[0], p = -tab[2];
  const double* pw = tab + IIR_P1;
  const int lane = tid & 63, w = tid >> 6;
  double s = 0.0;
  uint32_t prev = xm1 & 1u;
#pragma unroll
  for (int i = 0; i < IIR_CHUNK; i++) {
    const uint32_t x = (bits >> i) & 1u;
    s = __fma_rn(p, s, b0 * (double)(x + prev));
    prev = x;
  }
  double e = s;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const double u = __shfl_up(e, d);
    if (lane >= d) e = __fma_rn(pw[d], u, e);
  }
  double st = __shfl_up(e, 1);
  if (lane == 0) st = 0.0;
  if (lane == 63) aux->tot[w][0] = e;
  iir_wave_carries<1>(aux, pw, tid);
  st = __fma_rn(pl, aux->k[w][0], st);
  st = __fma_rn(pt, aux->k[16][0], st);
  prev = xm1 & 1u;
#pragma unroll
  for (int i = 0; i < IIR_CHUNK; i++) {
    const uint32_t x = (bits >> i) & 1u;
    st = __fma_rn(p, st, b0 * (double)(x + prev));
    prev = x;
    y[i] = st;
  }
}

// Second-order section y[n] = b0 x[n] + b1 x[n-1] + b2 x[n-2] - a1 y[n-1] - a2 y[n-2]
// (cf = b0 b1 b2 a1 a2; pw = its C^(16 s) table).  x[i] = x[16t + i],
// xm1, xm2 = x[16t - 1], x[16t - 2] (circular).  y[i] = y[16t + i].
// ml, mt: C^(16 lane), C^(16 t) from the table, loaded by the caller.
__device__ __forceinline__ double4 iir2_pow(const double* __restrict__ pw, int s) {
  return *reinterpret_cast<const double4*>(pw + 4 * s);
}
__device__ __forceinline__ void iir2(const double* x, double xm1, double xm2, const double* __restrict__ cf,
                                     const double* __restrict__ pw, IIRAux* aux, int tid, double4 ml, double4 mt,
                                     double* y) {
  const double b0 = cf[0], b1 = cf[1], b2 = cf[2], a1 = cf[3], a2 = cf[4];
  const int lane = tid & 63, w = tid >> 6;
  double e0 = 0.0, e1 = 0.0;
  {
    double xa = xm1, xb = xm2;
#pragma unroll
    for (int i = 0; i < IIR_CHUNK; i++) {
      const double v = b0 * x[i] + b1 * xa + b2 * xb - a1 * e0 - a2 * e1;
      e1 = e0;
      e0 = v;
      xb = xa;
      xa = x[i];
    }
  }
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const double u0 = __shfl_up(e0, d), u1 = __shfl_up(e1, d);
    if (lane >= d) {
      const double* m = pw + 4 * d;
      const double n0 = __fma_rn(m[0], u0, __fma_rn(m[1], u1, e0));
      const double n1 = __fma_rn(m[2], u0, __fma_rn(m[3], u1, e1));
      e0 = n0;
      e1 = n1;
    }
  }
  double s0 = __shfl_up(e0, 1), s1 = __shfl_up(e1, 1);
  if (lane == 0) s0 = s1 = 0.0;
  if (lane == 63) {
    aux->tot[w][0] = e0;
    aux->tot[w][1] = e1;
  }
  iir_wave_carries<2>(aux, pw, tid);
  {
    const double K0 = aux->k[w][0], K1 = aux->k[w][1], E0 = aux->k[16][0], E1 = aux->k[16][1];
    s0 = __fma_rn(ml.x, K0, __fma_rn(ml.y, K1, s0));
    s1 = __fma_rn(ml.z, K0, __fma_rn(ml.w, K1, s1));
    s0 = __fma_rn(mt.x, E0, __fma_rn(mt.y, E1, s0));
    s1 = __fma_rn(mt.z, E0, __fma_rn(mt.w, E1, s1));
  }
  {
    double xa = xm1, xb = xm2;
#pragma unroll
    for (int i = 0; i < IIR_CHUNK; i++) {
      const double v = b0 * x[i] + b1 * xa + b2 * xb - a1 * s0 - a2 * s1;
      s1 = s0;
      s0 = v;
      xb = xa;
      xa = x[i];
      y[i] = v;
    }
  }
}

}  // namespace ldg
