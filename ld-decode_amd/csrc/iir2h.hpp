// The periodic recurrences of iir.hpp (sync, burst, pilot) for the 512-thread
// demod (demod2.hip): 1024 chunks of 16 samples, thread t owning chunk t of
// half A (samples [0, 8192)) and chunk t of half B (samples [8192, 16384)).
// Both halves are scanned by the same instructions: the affine scans over the
// wave (DPP) run side by side, the wave carries put half A in DPP row 0 and
// half B in row 1 of one wave (rows scan independently).  Then
//   S_0   = T_B + C^(16*512) T_A        (the circle: the state after chunk 1023
//                                        from zero, as in iir.hpp)
//   S_512 = T_A + C^(16*512) S_0
// with T_h the half's total from a zero state, and a chunk's entering state is
// its half's exclusive prefix + C^(16 lane) K_h[wave] + C^(16 t) S_(0 | 512).
// Same step functions as iir.hpp (the field kernels rebuild values from the
// stored chunk states with them, bit-identically).
#pragma once
#include "iir.hpp"

namespace ldg {

struct IIRAux2 {
  double tot[2][8][2];    // [half][wave] inclusive wave totals
  double k[2][9][2];      // [half][w]: state entering wave w from zero at the half's start; [8]: half total
};

template <int ORD>
__device__ __forceinline__ void iir_wave_carries2(IIRAux2* aux, const double* __restrict__ pw, int tid) {
  __syncthreads();
  if (tid < 64) {
    const int h = (tid >> 4) & 1, i = tid & 15;
    const bool act = tid < 32 && i < 8;
    double k0 = act ? aux->tot[h][i][0] : 0.0;
    double k1 = (ORD == 2 && act) ? aux->tot[h][i][1] : 0.0;
    carry_step<0x111, ORD>(k0, k1, pw, 64);     // row-local: half A in lanes 0..15, half B in 16..31
    carry_step<0x112, ORD>(k0, k1, pw, 128);
    carry_step<0x114, ORD>(k0, k1, pw, 256);
    if (act) {
      aux->k[h][i + 1][0] = k0;
      if (ORD == 2) aux->k[h][i + 1][1] = k1;
    }
    if (tid < 32 && i == 0) {
      aux->k[h][0][0] = 0.0;
      aux->k[h][0][1] = 0.0;
    }
  }
  __syncthreads();
}

// First order (FPsync).  eA / eB: the chunks' end states from a zero state.  On
// return *sA / *sB are the states entering the two chunks.  pl, pt: p^(16 lane),
// p^(16 t); p15, p31: p^(16 scan_d15(lane)), p^(16 scan_d31(lane)); p512: p^(16*512).
__device__ __forceinline__ void iir1_scan2(double eA, double eB, const double* __restrict__ pw, IIRAux2* aux, int tid,
                                           double pl, double pt, double p15, double p31, double p512, double* sA,
                                           double* sB) {
  const int lane = tid & 63, w = tid >> 6;
  double z0 = 0.0;
  carry_step<0x111, 1>(eA, z0, pw, 1);
  carry_step<0x111, 1>(eB, z0, pw, 1);
  carry_step<0x112, 1>(eA, z0, pw, 2);
  carry_step<0x112, 1>(eB, z0, pw, 2);
  carry_step<0x114, 1>(eA, z0, pw, 4);
  carry_step<0x114, 1>(eB, z0, pw, 4);
  carry_step<0x118, 1>(eA, z0, pw, 8);
  carry_step<0x118, 1>(eB, z0, pw, 8);
  carry_step_lane1<0x142, 0xa>(eA, p15);
  carry_step_lane1<0x142, 0xa>(eB, p15);
  carry_step_lane1<0x143, 0xc>(eA, p31);
  carry_step_lane1<0x143, 0xc>(eB, p31);
  double a = dpp_f64<0x138>(eA), b = dpp_f64<0x138>(eB);   // exclusive: lane 0 reads 0
  if (lane == 63) {
    aux->tot[0][w][0] = eA;
    aux->tot[1][w][0] = eB;
  }
  iir_wave_carries2<1>(aux, pw, tid);
  const double TA = aux->k[0][8][0], TB = aux->k[1][8][0];
  const double S0 = __fma_rn(p512, TA, TB);
  const double S512 = __fma_rn(p512, S0, TA);
  a = __fma_rn(pl, aux->k[0][w][0], a);
  b = __fma_rn(pl, aux->k[1][w][0], b);
  *sA = __fma_rn(pt, S0, a);
  *sB = __fma_rn(pt, S512, b);
}

__device__ __forceinline__ double2 mat2(double4 m, double2 v, double2 acc) {
  return make_double2(__fma_rn(m.x, v.x, __fma_rn(m.y, v.y, acc.x)), __fma_rn(m.z, v.x, __fma_rn(m.w, v.y, acc.y)));
}

// Second order (Fburst / Fpilot): the same for 2-vector states (y[n], y[n-1]).
// pw: the C^(16 s) table; the per-lane powers C^(16 lane), C^(16 t), C^(16 scan_d15),
// C^(16 scan_d31) and C^(16*512) are loaded where they are used (registers).
__device__ __forceinline__ void iir2_scan2(double2 eA, double2 eB, const double* __restrict__ pw, IIRAux2* aux, int tid,
                                           double2* sA, double2* sB) {
  const int lane = tid & 63, w = tid >> 6;
  carry_step<0x111, 2>(eA.x, eA.y, pw, 1);
  carry_step<0x111, 2>(eB.x, eB.y, pw, 1);
  carry_step<0x112, 2>(eA.x, eA.y, pw, 2);
  carry_step<0x112, 2>(eB.x, eB.y, pw, 2);
  carry_step<0x114, 2>(eA.x, eA.y, pw, 4);
  carry_step<0x114, 2>(eB.x, eB.y, pw, 4);
  carry_step<0x118, 2>(eA.x, eA.y, pw, 8);
  carry_step<0x118, 2>(eB.x, eB.y, pw, 8);
  {
    const double4 m15 = iir2_pow(pw, scan_d15(lane));
    carry_step_lane2<0x142, 0xa>(eA.x, eA.y, m15);
    carry_step_lane2<0x142, 0xa>(eB.x, eB.y, m15);
  }
  {
    const double4 m31 = iir2_pow(pw, scan_d31(lane));
    carry_step_lane2<0x143, 0xc>(eA.x, eA.y, m31);
    carry_step_lane2<0x143, 0xc>(eB.x, eB.y, m31);
  }
  double2 a = make_double2(dpp_f64<0x138>(eA.x), dpp_f64<0x138>(eA.y));
  double2 b = make_double2(dpp_f64<0x138>(eB.x), dpp_f64<0x138>(eB.y));
  if (lane == 63) {
    aux->tot[0][w][0] = eA.x;
    aux->tot[0][w][1] = eA.y;
    aux->tot[1][w][0] = eB.x;
    aux->tot[1][w][1] = eB.y;
  }
  iir_wave_carries2<2>(aux, pw, tid);
  const double2 TA = make_double2(aux->k[0][8][0], aux->k[0][8][1]);
  const double2 TB = make_double2(aux->k[1][8][0], aux->k[1][8][1]);
  const double4 m512 = iir2_pow(pw, 512);
  const double2 S0 = mat2(m512, TA, TB);
  const double2 S512 = mat2(m512, S0, TA);
  const double4 ml = iir2_pow(pw, lane);
  a = mat2(ml, make_double2(aux->k[0][w][0], aux->k[0][w][1]), a);
  b = mat2(ml, make_double2(aux->k[1][w][0], aux->k[1][w][1]), b);
  const double4 mt = iir2_pow(pw, tid);
  *sA = mat2(mt, S0, a);
  *sB = mat2(mt, S512, b);
}

// A chunk's second-order recurrence from state s (x: its 16 samples; xm1, xm2 the
// two before it).  Returns the end state; y (if non-null) receives the outputs.
__device__ __forceinline__ double2 sos_chunk(const double* x, double xm1, double xm2, double2 s, const double* cf,
                                             double* y) {
  const double b0 = cf[0], b1 = cf[1], b2 = cf[2], a1 = cf[3], a2 = cf[4];
  double s0 = s.x, s1 = s.y, xa = xm1, xb = xm2;
#pragma unroll
  for (int i = 0; i < IIR_CHUNK; i++) {
    const double v = sos_step(x[i], xa, xb, s0, s1, b0, b1, b2, a1, a2);
    s1 = s0;
    s0 = v;
    xb = xa;
    xa = x[i];
    if (y) y[i] = v;
  }
  return make_double2(s0, s1);
}

}  // namespace ldg
