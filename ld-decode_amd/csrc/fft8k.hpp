// 8192-point FP64 FFT for one 1024-thread workgroup, four-step with
// wave-local inner stages.
//
// 8192 = 16 x 8 x 8 x 8.  Stage 1 is a radix-16 pass over stride 512.  It is
// the only stage that mixes data between waves.  Stages 2-4 are radix-8
// passes inside one 512-point sub-array, and wave q owns sub-array q.  So a
// transform has one workgroup barrier in its body, not two per pass (the
// Stockham fft_lds in fft.hpp has ten), and waves run their inner stages out
// of step: one wave's LDS stores overlap another wave's FP64 work.  There are
// four LDS round trips per point, not five.
//
// Layouts (same XOR swizzle as fft.hpp, through SW; the inner stages address
// the same physical slots SW(64 a + 8 b + c) = 64 a + 8 (b ^ (a & 1)) + (c ^ b)):
//   * fft8k_dif: the forward transform.  Natural order in, digit-reversed out:
//     bin k = q + 16 s + 128 u + 1024 v lands at position dr_pos(k) =
//     512 q + 64 s + 8 u + v.
//   * fft8k_dit: the inverse transform.  Digit-reversed in, natural order out.
// The demod only does pointwise spectral work between the two (filters, the
// real-FFT split/merge), so it never reorders: it indexes bins through dr_pos.
//
// Twiddles come from the same W[m] = exp(-2 pi i m / 16384) table.  Stage 1's
// twiddle W_8192^(q m) is applied inside stage 2, on stage 2's input for the
// DIF and on stage 2's output for the DIT.  It factors as W_8192^(q m2) (one
// per-lane load) times W_128^(q r), and W_128^(q r) is uniform across the wave
// (scalar loads).
#pragma once
#include "fft.hpp"

namespace ldg {

__host__ __device__ __forceinline__ constexpr int dr_pos(int k) {
  return ((k & 15) << 9) | (((k >> 4) & 7) << 6) | (((k >> 7) & 7) << 3) | ((k >> 10) & 7);
}
__host__ __device__ __forceinline__ constexpr int dr_nat(int p) {
  return ((p >> 9) & 15) | (((p >> 6) & 7) << 4) | (((p >> 3) & 7) << 7) | ((p & 7) << 10);
}

// Per-lane twiddles W[i] = exp(-2 pi i i / 16384) of the transforms' stages, from
// an LDS copy of the even entries i < 2048 (all a transform reads per lane:
// 32 l, 256 m3, 2 q m2; the wave-uniform W_128^(q r) stay scalar loads of the
// global table).  Global loads after a phase's global stores wait for those
// stores (gfx9's vmcnt counts both), so the transforms read no global memory
// per lane.  Entry k = i / 2 at tw_lds_pos(k): conflict-free for i = 32 l and
// 256 m3 under ds_read_b128's lane groups.
constexpr int TW_LDS_N = 1024;
__host__ __device__ __forceinline__ constexpr int tw_lds_pos(int k) { return k ^ ((k >> 4) & 15) ^ ((k >> 7) & 7); }
struct TwLds {
  const double2* t;   // LDS, TW_LDS_N entries
  __device__ __forceinline__ double2 operator()(int i) const { return t[tw_lds_pos(i >> 1)]; }
};

// a * W16^r (conjugate twiddle for the inverse), r = 0..7
template <bool INV> __device__ __forceinline__ double2 w16(double2 a, int r) {
  constexpr double C1 = 0.92387953251128675613, S1 = 0.38268343236508977173, R2 = 0.70710678118654752440;
  const double sg = INV ? -1.0 : 1.0;
  switch (r) {
    case 0: return a;
    case 1: return cmul(a, make_double2(C1, -sg * S1));
    case 2: return INV ? make_double2(R2 * (a.x - a.y), R2 * (a.x + a.y)) : make_double2(R2 * (a.x + a.y), R2 * (a.y - a.x));
    case 3: return cmul(a, make_double2(S1, -sg * C1));
    case 4: return mul_mi<INV>(a);
    case 5: return cmul(a, make_double2(-S1, -sg * C1));
    case 6: return INV ? make_double2(-R2 * (a.x + a.y), R2 * (a.x - a.y)) : make_double2(R2 * (a.y - a.x), -R2 * (a.x + a.y));
    default: return cmul(a, make_double2(-C1, -sg * S1));
  }
}

// Order LDS accesses of one wave across lanes (the hardware keeps a wave's LDS
// operations in order; this keeps the compiler from moving them).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

// stage-1 twiddle for the 8 points m2 + 64 r of sub-array q: v[r] *= W_8192^(q (m2 + 64 r))
template <bool INV>
__device__ __forceinline__ void stage1_twiddle(double2* v, const double2* __restrict__ tw, TwLds twl, int q, int m2) {
  if (q == 0) return;   // wave-uniform
  double2 g = twl(2 * q * m2);
  if (INV) g = conj2(g);
  v[0] = cmul(v[0], g);
#pragma unroll
  for (int r = 1; r < 8; r++) {
    double2 h = tw[128 * q * r];   // wave-uniform address: scalar load
    if (INV) h = conj2(h);
    v[r] = cmul(v[r], cmul(g, h));
  }
}

// Forward (INV=false) or inverse transform, natural order in, digit-reversed out.
// Begins and ends with a workgroup barrier, like fft_lds.
template <bool INV>
__device__ __forceinline__ void fft8k_dif(double2* __restrict__ s, const double2* __restrict__ tw, TwLds twl, int tid) {
  __syncthreads();
  {
    // stage 1: radix-16 over stride 512.  Thread pair (m, b): both read all 16
    // points, thread b produces the outputs q = 2 q1 + b.
    asm volatile("" : "+v"(tid));
    const int m = tid & 511;
    const int b = __builtin_amdgcn_readfirstlane(tid >> 9);
    const int sm = SW(m);
    double2 u[8];
#pragma unroll
    for (int r = 0; r < 8; r++) {
      const double2 a = s[sm + 512 * r], c = s[sm + 512 * (r + 8)];
      u[r] = b ? w16<INV>(csub(a, c), r) : cadd(a, c);
      if (r == 3) __builtin_amdgcn_sched_barrier(0);   // at most 8 loads in flight (register pressure)
    }
    dft8<INV>(u);
    __syncthreads();
#pragma unroll
    for (int q1 = 0; q1 < 8; q1++) s[512 * (2 * q1 + b) + sm] = u[q1];
  }
  __syncthreads();
  asm volatile("" : "+v"(tid));
  const int q = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l = tid & 63;
  double2* sub = s + 512 * q;
  double2 v[8];
  {
    // stage 2: radix 8 over stride 64 inside the sub-array (slot of 64 r + l:
    // 64 r + SW(l) with bit 3 flipped for odd r)
    const int swl = SW(l);
#pragma unroll
    for (int r = 0; r < 8; r++) v[r] = sub[64 * r + (swl ^ ((r & 1) << 3))];
    stage1_twiddle<INV>(v, tw, twl, q, l);
    dft8<INV>(v);
    twiddle_row_w<8, INV>(v, twl(32 * l));
#pragma unroll
    for (int r = 0; r < 8; r++) sub[64 * r + (swl ^ ((r & 1) << 3))] = v[r];
  }
  wave_lds_sync();
  {
    // stage 3: radix 8 over stride 8 inside each 64-point block (a = l >> 3)
    const int m3 = l & 7, a1 = (l >> 3) & 1;
    double2* p = sub + 64 * (l >> 3);
#pragma unroll
    for (int r = 0; r < 8; r++) v[r] = p[8 * (r ^ a1) + (m3 ^ r)];
    dft8<INV>(v);
    twiddle_row_w<8, INV>(v, twl(256 * m3));
#pragma unroll
    for (int r = 0; r < 8; r++) p[8 * (r ^ a1) + (m3 ^ r)] = v[r];
  }
  wave_lds_sync();
  {
    // stage 4: radix 8 on each 8 consecutive points
    const int x = l & 7;
    double2* p = sub + 8 * (l ^ ((l >> 3) & 1));
#pragma unroll
    for (int r = 0; r < 8; r++) v[r] = p[r ^ x];
    dft8<INV>(v);
#pragma unroll
    for (int r = 0; r < 8; r++) p[r ^ x] = v[r];
  }
  __syncthreads();
}

// Transform of a digit-reversed input (the transpose of fft8k_dif), natural order out.
// OUT_REGS: the last stage leaves its outputs in registers instead of LDS --
// thread tid holds natural positions tid + 1024 q in out[q], q < 8 (the layout a
// caller reading X_[tid + 1024 q] would get) -- saving an LDS round trip for an
// elementwise consumer.  The transform then ends with the barrier after its last
// LDS reads, so the caller may write s right away.
template <bool INV, bool OUT_REGS = false>
__device__ __forceinline__ void fft8k_dit(double2* __restrict__ s, const double2* __restrict__ tw, TwLds twl, int tid,
                                          double2* out = nullptr) {
  __syncthreads();
  {
    asm volatile("" : "+v"(tid));
    const int q = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int l = tid & 63;
    double2* sub = s + 512 * q;
    double2 v[8];
    {
      const int x = l & 7;
      double2* p = sub + 8 * (l ^ ((l >> 3) & 1));
#pragma unroll
      for (int r = 0; r < 8; r++) v[r] = p[r ^ x];
      dft8<INV>(v);
#pragma unroll
      for (int r = 0; r < 8; r++) p[r ^ x] = v[r];
    }
    wave_lds_sync();
    {
      const int m3 = l & 7, a1 = (l >> 3) & 1;
      double2* p = sub + 64 * (l >> 3);
#pragma unroll
      for (int r = 0; r < 8; r++) v[r] = p[8 * (r ^ a1) + (m3 ^ r)];
      twiddle_row_w<8, INV>(v, twl(256 * m3));
      dft8<INV>(v);
#pragma unroll
      for (int r = 0; r < 8; r++) p[8 * (r ^ a1) + (m3 ^ r)] = v[r];
    }
    wave_lds_sync();
    {
      const int swl = SW(l);
#pragma unroll
      for (int r = 0; r < 8; r++) v[r] = sub[64 * r + (swl ^ ((r & 1) << 3))];
      twiddle_row_w<8, INV>(v, twl(32 * l));
      dft8<INV>(v);
      stage1_twiddle<INV>(v, tw, twl, q, l);
#pragma unroll
      for (int r = 0; r < 8; r++) sub[64 * r + (swl ^ ((r & 1) << 3))] = v[r];
    }
  }
  __syncthreads();
  {
    // stage 1 transposed: radix-16 over the sub-arrays.  Thread b produces the
    // outputs r = 2 r1 + b.
    asm volatile("" : "+v"(tid));
    const int m = tid & 511;
    const int b = __builtin_amdgcn_readfirstlane(tid >> 9);
    const int sm = SW(m);
    double2 u[8];
#pragma unroll
    for (int q1 = 0; q1 < 8; q1++) {
      const double2 a = s[sm + 512 * q1], c = s[sm + 512 * (q1 + 8)];
      u[q1] = b ? w16<INV>(csub(a, c), q1) : cadd(a, c);
      if (q1 == 3) __builtin_amdgcn_sched_barrier(0);
    }
    dft8<INV>(u);
    __syncthreads();
    if constexpr (OUT_REGS) {
#pragma unroll
      for (int r1 = 0; r1 < 8; r1++) out[r1] = u[r1];
      return;
    } else {
#pragma unroll
      for (int r1 = 0; r1 < 8; r1++) s[sm + 512 * (2 * r1 + b)] = u[r1];
    }
  }
  __syncthreads();
}

}  // namespace ldg
