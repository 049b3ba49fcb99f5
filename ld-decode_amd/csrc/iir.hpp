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
//      (Kogge-Stone over the wave by DPP row shifts and row broadcasts, then
//      over the 16 wave totals), C the companion matrix of A;
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

// Lane i of a wave reads x of another lane (DPP, no LDS round trip): CTRL
// 0x111..0x118 = row_shr:1..8 (lane i - d of its row of 16, 0 below the row
// start), 0x142 = row_bcast:15 (lane 15 of the previous row; rows ROWM),
// 0x143 = row_bcast:31 (lane 31), 0x138 = wave_shr:1 (lane i - 1; lane 0 reads 0).
template <int CTRL, int ROWM = 0xf>
__device__ __forceinline__ double dpp_f64(double x) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), CTRL, ROWM, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), CTRL, ROWM, 0xf, false);
  return __hiloint2double(hi, lo);
}

// Per-lane powers of the cross-row steps of the wave scans below: row_bcast:15
// adds lane 15 (47) to row 1 (3) at distance (lane & 15) + 1 chunks, row_bcast:31
// adds lane 31 to rows 2, 3 at distance lane - 31.
__device__ __forceinline__ int scan_d15(int lane) { return (lane & 15) + 1; }
__device__ __forceinline__ int scan_d31(int lane) { return lane >= 32 ? lane - 31 : 0; }

// One step of each recurrence, in the arithmetic the demod's outputs use; the
// field kernels rebuild sync / burst values from stored chunk states with the
// same steps (compact channels, chan.hpp), so the values are bit-identical.
__device__ __forceinline__ double sync_step(double st, uint32_t x, uint32_t prev, double b0, double p) {
  return __fma_rn(p, st, b0 * (double)(x + prev));
}
__device__ __forceinline__ double sos_step(double x, double xa, double xb, double s0, double s1, double b0, double b1,
                                           double b2, double a1, double a2) {
  return b0 * x + b1 * xa + b2 * xb - a1 * s0 - a2 * s1;
}

// LDS scratch of a scan: wave totals and the states entering each wave.
struct IIRAux {
  double tot[16][2];
  double k[17][2];
};

// Chunk layout in LDS: double2 index u (samples 2u, 2u+1) lives at SWC(u).
// Conflict-free both for the pair-per-lane layout u = t + 1024 q (ds_write_b128 /
// ds_read_b128) and for the chunk-per-lane layout u = 8 t + c.
__device__ __forceinline__ constexpr int SWC(int u) { return u ^ ((u >> 3) & 15); }

// One Kogge-Stone step of an affine scan with a wave-uniform power (table entry s):
// (k0, k1) += C^(16 s) (k0, k1) of the lane CTRL reads.
template <int CTRL, int ORD>
__device__ __forceinline__ void carry_step(double& k0, double& k1, const double* __restrict__ pw, int s) {
  const double u0 = dpp_f64<CTRL>(k0);
  if constexpr (ORD == 1) {
    k0 = __fma_rn(pw[s], u0, k0);
  } else {
    const double u1 = dpp_f64<CTRL>(k1);
    const double* m = pw + 4 * s;
    const double n0 = __fma_rn(m[0], u0, __fma_rn(m[1], u1, k0));
    const double n1 = __fma_rn(m[2], u0, __fma_rn(m[3], u1, k1));
    k0 = n0;
    k1 = n1;
  }
}
// The same with per-lane powers m (ORD 2: a row-major 2x2 matrix).
template <int CTRL, int ROWM>
__device__ __forceinline__ void carry_step_lane1(double& k0, double m) {
  k0 = __fma_rn(m, dpp_f64<CTRL, ROWM>(k0), k0);
}
template <int CTRL, int ROWM>
__device__ __forceinline__ void carry_step_lane2(double& k0, double& k1, double4 m) {
  const double u0 = dpp_f64<CTRL, ROWM>(k0), u1 = dpp_f64<CTRL, ROWM>(k1);
  const double n0 = __fma_rn(m.x, u0, __fma_rn(m.y, u1, k0));
  const double n1 = __fma_rn(m.z, u0, __fma_rn(m.w, u1, k1));
  k0 = n0;
  k1 = n1;
}

// States entering each wave and the block total, from the per-wave inclusive
// totals (written to aux->tot by lane 63 of each wave).  ORD = state size.
template <int ORD>
__device__ __forceinline__ void iir_wave_carries(IIRAux* aux, const double* __restrict__ pw, int tid) {
  __syncthreads();
  if (tid < 64) {
    const int lane = tid;
    double k0 = lane < 16 ? aux->tot[lane][0] : 0.0;
    double k1 = (ORD == 2 && lane < 16) ? aux->tot[lane][1] : 0.0;
    // inclusive scan over lanes 0..15 (one DPP row): lanes below d read 0
    carry_step<0x111, ORD>(k0, k1, pw, 64);
    carry_step<0x112, ORD>(k0, k1, pw, 128);
    carry_step<0x114, ORD>(k0, k1, pw, 256);
    carry_step<0x118, ORD>(k0, k1, pw, 512);
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
// p15, p31: p^(16 scan_d15(lane)), p^(16 scan_d31(lane)), also loaded by the caller.
// *st_in: the state entering the chunk (y[16t - 1]).
__device__ __forceinline__ void iir1_bits(uint32_t bits, uint32_t xm1, const double* __restrict__ tab, IIRAux* aux,
                                          int tid, double pl, double pt, double p15, double p31, double* y,
                                          double* st_in) {
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
  double e = s, e1 = 0.0;
  carry_step<0x111, 1>(e, e1, pw, 1);
  carry_step<0x112, 1>(e, e1, pw, 2);
  carry_step<0x114, 1>(e, e1, pw, 4);
  carry_step<0x118, 1>(e, e1, pw, 8);
  carry_step_lane1<0x142, 0xa>(e, p15);
  carry_step_lane1<0x143, 0xc>(e, p31);
  double st = dpp_f64<0x138>(e);        // exclusive: lane 0 reads 0
  if (lane == 63) aux->tot[w][0] = e;
  iir_wave_carries<1>(aux, pw, tid);
  st = __fma_rn(pl, aux->k[w][0], st);
  st = __fma_rn(pt, aux->k[16][0], st);
  *st_in = st;
  prev = xm1 & 1u;
#pragma unroll
  for (int i = 0; i < IIR_CHUNK; i++) {
    const uint32_t x = (bits >> i) & 1u;
    st = sync_step(st, x, prev, b0, p);
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
// m15, m31: C^(16 scan_d15(lane)), C^(16 scan_d31(lane)).
__device__ __forceinline__ void iir2(const double* x, double xm1, double xm2, const double* __restrict__ cf,
                                     const double* __restrict__ pw, IIRAux* aux, int tid, double4 ml, double4 mt,
                                     double4 m15, double4 m31, double* y, double2* s_in) {
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
  carry_step<0x111, 2>(e0, e1, pw, 1);
  carry_step<0x112, 2>(e0, e1, pw, 2);
  carry_step<0x114, 2>(e0, e1, pw, 4);
  carry_step<0x118, 2>(e0, e1, pw, 8);
  carry_step_lane2<0x142, 0xa>(e0, e1, m15);
  carry_step_lane2<0x143, 0xc>(e0, e1, m31);
  double s0 = dpp_f64<0x138>(e0), s1 = dpp_f64<0x138>(e1);   // exclusive: lane 0 reads 0
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
  *s_in = make_double2(s0, s1);
  {
    double xa = xm1, xb = xm2;
#pragma unroll
    for (int i = 0; i < IIR_CHUNK; i++) {
      const double v = sos_step(x[i], xa, xb, s0, s1, b0, b1, b2, a1, a2);
      s1 = s0;
      s0 = v;
      xb = xa;
      xa = x[i];
      y[i] = v;
    }
  }
}

}  // namespace ldg
