// 8192-point FP64 FFT for one 512-thread workgroup holding the data in
// REGISTERS, with 64 KiB of LDS: two workgroups share a CU (160 KiB of LDS),
// so one's barriers and LDS round trips overlap the other's arithmetic.
//
// 8192 = 16 x 512, 512 = 8 x 8 x 8.  Thread t (wave w = t / 64, lane l) holds
// 16 points:
//   * natural layout (transform input / inverse output): v[r] = x[t + 512 r];
//   * spectral layout (transform output / inverse input): wave w owns the two
//     512-point sub-arrays q0(w) = w and q1(w) = 16 - w (8 for w = 0) of the
//     bins k = q + 16 j, j = jl + 64 d with jl = (l >> 3) + 8 (l & 7):
//       v[d]     = X[q0 + 16 (jl + 64 d)],
//       v[8 + d] = X[q1 + 16 (jl + 64 d)]                 (w = 0),
//       v[8 + d] = X[8192 - (q0 + 16 (jl + 64 (7 - d)))]  (w > 0: sub-array 1
//                  lane-reversed, so v[15 - d] is the mirror bin of v[d]).
//     bin_of() gives the bin of any position.  A real-FFT split / merge pairs
//     bin k with 8192 - k: in the same thread for w > 0, in the same wave for w = 0.
// Forward: radix-16 over r in registers, the stage twiddle W_8192^(q t), a
// workgroup exchange through the 64 KiB buffer in two rounds (round s moves
// every wave's sub-array s: 8 points per thread out, 8 in, so no thread holds
// more than 16 points), then per sub-array a radix-8 in registers and two
// wave-private LDS transposes (8 KiB per wave) around two more radix-8
// passes.  The inverse runs the same steps backwards (conjugate twiddles).
// Twiddles: W[m] = exp(-2 pi i m / 16384) from the global table (L1/L2).
#pragma once
#include "fft8k.hpp"

namespace ldg {
namespace h8k {

constexpr int T = 512;                 // threads
constexpr int EX = 4096;               // exchange buffer, double2 (64 KiB)

__host__ __device__ __forceinline__ constexpr int q_of(int w, int s) { return s == 0 ? w : (w == 0 ? 8 : 16 - w); }

// the bin held at spectral-layout position (wave w, sub-array s, lane l, register d)
__host__ __device__ __forceinline__ constexpr int bin_of(int w, int s, int l, int d) {
  const int jl = (l >> 3) + 8 * (l & 7);
  return s == 0 ? w + 16 * (jl + 64 * d)
                : (w == 0 ? 8 + 16 * (jl + 64 * d) : 8192 - (w + 16 * (jl + 64 * (7 - d))));
}
// index of a per-position table (a wave's load of one register: 64 consecutive entries)
__host__ __device__ __forceinline__ constexpr int pos_of(int w, int s, int l, int d) {
  return ((w * 2 + s) * 8 + d) * 64 + l;
}

// wave-private transpose position: element e (0..7) of lane L, conflict-free for
// ds_read_b128 by lane (16-lane groups) and for the writes of both transposes
// base[idx] through a 32-bit unsigned byte offset: with a uniform base the access is
// global_load / store v_off, s[base] (one address VGPR instead of a 64-bit pair)
template <class T>
__device__ __forceinline__ T& at(T* base, unsigned idx) {
  return *reinterpret_cast<T*>(reinterpret_cast<char*>(base) + idx * (unsigned)sizeof(T));
}
template <class T>
__device__ __forceinline__ const T& at(const T* base, unsigned idx) {
  return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + idx * (unsigned)sizeof(T));
}

__device__ __forceinline__ int tpos(int L, int e) { return 8 * L + (e ^ ((L >> 1) & 7)); }

// Materialise a value here: the compiler may otherwise sink its arithmetic past
// the exchange's barriers to where the value is used, keeping its inputs (and
// everything in between) alive -- spills.
__device__ __forceinline__ void pin(double2& z) { asm volatile("" : "+v"(z.x), "+v"(z.y)); }
__device__ __forceinline__ void pin16(double2* v) {
#pragma unroll
  for (int i = 0; i < 16; i++) pin(v[i]);
}

__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

// T1 (lane bits 3-5 <-> element) or T2 (lane bits 0-2 <-> element) of 8 points
// through the wave's 8 KiB scratch sc.  Involutions.  lw / lr: the logical lane
// the physical lane writes as / reads as (63 - l on the lane-reversed side).
template <int BITS>   // 3: T1, 0: T2
__device__ __forceinline__ void wtranspose(double2* v, double2* sc, int lw, int lr) {
  const int keep = lw & ~(7 << BITS), mine = (lw >> BITS) & 7;
#pragma unroll
  for (int e = 0; e < 8; e++) sc[tpos(keep | (e << BITS), mine)] = v[e];
  wsync();
#pragma unroll
  for (int e = 0; e < 8; e++) v[e] = sc[tpos(lr, e)];
  wsync();
}

// the stage twiddles W_8192^(q t), q = 1..15, applied to y[q] (conjugate: INV)
template <bool INV>
__device__ __forceinline__ void tw16(double2* y, const double2* __restrict__ tw, int t) {
  double2 g1 = at(tw, 2 * t), g2 = at(tw, 4 * t), g4 = at(tw, 8 * t), g8 = at(tw, 16 * t);
  if (INV) { g1 = conj2(g1); g2 = conj2(g2); g4 = conj2(g4); g8 = conj2(g8); }
  const double2 g3 = cmul(g2, g1);
  y[1] = cmul(y[1], g1);
  y[2] = cmul(y[2], g2);
  y[3] = cmul(y[3], g3);
  y[4] = cmul(y[4], g4);
  y[5] = cmul(y[5], cmul(g4, g1));
  y[6] = cmul(y[6], cmul(g4, g2));
  y[7] = cmul(y[7], cmul(g4, g3));
  y[8] = cmul(y[8], g8);
  y[9] = cmul(y[9], cmul(g8, g1));
  y[10] = cmul(y[10], cmul(g8, g2));
  y[11] = cmul(y[11], cmul(g8, g3));
  const double2 g12 = cmul(g8, g4);
  y[12] = cmul(y[12], g12);
  y[13] = cmul(y[13], cmul(g12, g1));
  y[14] = cmul(y[14], cmul(g12, g2));
  y[15] = cmul(y[15], cmul(g12, g3));
}

// radix-16 DIF over v[0..15] in place, outputs in natural q order
template <bool INV>
__device__ __forceinline__ void dft16(double2* v) {
  double2 u[8], w[8];
#pragma unroll
  for (int r = 0; r < 8; r++) {
    u[r] = cadd(v[r], v[r + 8]);
    w[r] = w16<INV>(csub(v[r], v[r + 8]), r);
  }
  dft8<INV>(u);
  dft8<INV>(w);
#pragma unroll
  for (int k = 0; k < 8; k++) { v[2 * k] = u[k]; v[2 * k + 1] = w[k]; }
}

// its transpose (inverse-direction DIT radix-16: q order in, r order out)
template <bool INV>
__device__ __forceinline__ void dft16_t(double2* v) {
  double2 u[8], w[8];
#pragma unroll
  for (int k = 0; k < 8; k++) { u[k] = v[2 * k]; w[k] = v[2 * k + 1]; }
  dft8<INV>(u);
  dft8<INV>(w);
#pragma unroll
  for (int r = 0; r < 8; r++) {
    const double2 z = w16<INV>(w[r], r);
    v[r] = cadd(u[r], z);
    v[r + 8] = csub(u[r], z);
  }
}

// the 512-point sub-transform of sub-array s after the exchange: lane l holds
// Y[l + 64 r'] in v[r'] -> X[k1 + 8 (c + 8 d)] in v[d] at lane c + 8 k1 (at
// lane 63 - (c + 8 k1) when rev: the lane-reversed sub-array)
template <bool INV>
__device__ __forceinline__ void sub512_fwd(double2* v, double2* sc, const double2* __restrict__ tw, int l, bool rev) {
  asm volatile("" : "+v"(l));          // per-call addresses (not hoisted across the kernel's transforms)
  dft8<INV>(v);
  twiddle_row_w<8, INV>(v, at(tw, 32 * l));
  wtranspose<3>(v, sc, l, l);          // lane (a, k1), elements b
  dft8<INV>(v);
  twiddle_row_w<8, INV>(v, at(tw, 256 * (l & 7)));
  wtranspose<0>(v, sc, l, rev ? 63 - l : l);   // lane (c, k1), elements a
  dft8<INV>(v);
}

// inverse direction of sub512_fwd (its transpose)
template <bool INV>
__device__ __forceinline__ void sub512_inv(double2* v, double2* sc, const double2* __restrict__ tw, int l, bool rev) {
  asm volatile("" : "+v"(l));
  dft8<INV>(v);
  wtranspose<0>(v, sc, rev ? 63 - l : l, l);   // lane (a, k1), elements c
  twiddle_row_w<8, INV>(v, at(tw, 256 * (l & 7)));
  dft8<INV>(v);
  wtranspose<3>(v, sc, l, l);          // lane (a, b), elements k1
  twiddle_row_w<8, INV>(v, at(tw, 32 * l));
  dft8<INV>(v);
}

// Forward-direction transform (INV: conjugate kernel), natural layout in,
// spectral layout out.  ex: the workgroup's 64 KiB LDS buffer.  Begins with a
// workgroup barrier (ex may still be read by the previous phase).  Each wave
// ends owning its 8 KiB at ex + 512 w (its exchange slot, which no other wave
// reads any more): wave-private use needs no further barrier.
template <bool INV>
__device__ __forceinline__ void fwd(double2* v, double2* ex, const double2* __restrict__ tw, int t) {
  pin16(v);                              // the transform's arithmetic stays inside it
  asm volatile("" : "+v"(t));
  dft16<INV>(v);
  tw16<INV>(v, tw, t);
#pragma unroll
  for (int q = 0; q < 16; q++) pin(v[q]);
  const int w = __builtin_amdgcn_readfirstlane(t >> 6), l = t & 63;
  double2* mine = ex + 512 * w;
  // round 0: sub-arrays q = 0..7 (slot q), round 1: q_of(j, 1) in slot j
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 8; j++) ex[512 * j + t] = v[j];
  double2 o[8];
#pragma unroll
  for (int j = 0; j < 8; j++) o[j] = v[q_of(j, 1)];
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 8; r++) v[r] = mine[l + 64 * r];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 8; j++) ex[512 * j + t] = o[j];
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 8; r++) v[8 + r] = mine[l + 64 * r];
  sub512_fwd<INV>(v, mine, tw, l, false);
#pragma unroll
  for (int r = 8; r < 16; r++) pin(v[r]);   // the second sub-transform starts after the first (registers)
  sub512_fwd<INV>(v + 8, mine, tw, l, w > 0);
  pin16(v);
}

// Inverse-direction transform, spectral layout in, natural layout out.  Begins
// with a workgroup barrier; ends after its last LDS reads (no trailing barrier:
// a caller writing ex next must barrier first).
template <bool INV>
__device__ __forceinline__ void inv(double2* v, double2* ex, const double2* __restrict__ tw, int t) {
  pin16(v);
  asm volatile("" : "+v"(t));
  const int w = __builtin_amdgcn_readfirstlane(t >> 6), l = t & 63;
  double2* mine = ex + 512 * w;
  __syncthreads();                       // ex free of the previous phase
  sub512_inv<INV>(v, mine, tw, l, false);
#pragma unroll
  for (int r = 8; r < 16; r++) pin(v[r]);
  sub512_inv<INV>(v + 8, mine, tw, l, w > 0);
#pragma unroll
  for (int r = 0; r < 8; r++) mine[l + 64 * r] = v[r];
  __syncthreads();
  double2 y[16];
#pragma unroll
  for (int j = 0; j < 8; j++) y[j] = ex[512 * j + t];
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 8; r++) mine[l + 64 * r] = v[8 + r];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 8; j++) y[q_of(j, 1)] = ex[512 * j + t];
#pragma unroll
  for (int q = 0; q < 16; q++) v[q] = y[q];
  asm volatile("" : "+v"(t));
  tw16<INV>(v, tw, t);
  dft16_t<INV>(v);
  pin16(v);
}

}  // namespace h8k
}  // namespace ldg
