// Workgroup-level FP64 FFT for gfx950, LDS-resident, Stockham autosort.
//
// Data lives in LDS as interleaved complex doubles (one 16-byte double2 per
// point, ds_read_b128 / ds_write_b128) under an XOR swizzle
//     slot(i) = i ^ ((i >> 3) & 7) ^ ((i >> 3) & 8)
// that permutes points inside aligned groups of 16 (bits 3-5 into bits 0-2,
// bit 6 into bit 3: the latter keeps fft8k.hpp's strided inner stages free of
// 2-way conflicts under ds_read_b128's 16-lane groups).  Unit-stride reads stay a
// permutation of 16 consecutive slots (64 banks, conflict-free for the
// 4 x 16-lane groups of ds_read_b128), and the stride-8 writes of the first
// Stockham pass land on 8 distinct 16-byte bank groups (conflict-free for the
// 8 x 8-lane groups of ds_write_b128).  An 8192-point transform therefore takes
// exactly 128 KiB of the 160 KiB LDS.
//
// Twiddles: one 16-byte load per radix-R butterfly from a global table
// W[m] = exp(-2*pi*i*m/16384) (L2 resident), the other R-2 powers by complex
// multiplication (depth <= 3 products, a few ulp).  An N-point transform uses
// table stride 16384/N.  All sizes and radices are compile-time.
#pragma once
#include <hip/hip_runtime.h>

namespace ldg {

constexpr int TW_N = 16384;

__device__ __forceinline__ constexpr int SW(int i) { return i ^ ((i >> 3) & 7) ^ ((i >> 3) & 8); }

// Swizzled complex buffer in LDS.
struct CBuf {
  double2* p;
  __device__ __forceinline__ double2& operator[](int i) const { return p[SW(i)]; }
  __device__ __forceinline__ CBuf operator+(int off) const { return CBuf{p + off}; }   // off: multiple of 8
};

__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
  return make_double2(__fma_rn(a.x, b.x, -a.y * b.y), __fma_rn(a.x, b.y, a.y * b.x));
}
__device__ __forceinline__ double2 cmulc(double2 a, double2 b) {   // a * conj(b)
  return make_double2(__fma_rn(a.x, b.x, a.y * b.y), __fma_rn(a.y, b.x, -a.x * b.y));
}
__device__ __forceinline__ double2 conj2(double2 a) { return make_double2(a.x, -a.y); }
// multiply by -i (forward) or +i (inverse)
template <bool INV> __device__ __forceinline__ double2 mul_mi(double2 a) {
  return INV ? make_double2(-a.y, a.x) : make_double2(a.y, -a.x);
}

template <bool INV> __device__ __forceinline__ void dft2(double2& a, double2& b) {
  double2 t = csub(a, b); a = cadd(a, b); b = t;
}

template <bool INV> __device__ __forceinline__ void dft4(double2* v) {
  double2 b0 = cadd(v[0], v[2]), b1 = csub(v[0], v[2]);
  double2 b2 = cadd(v[1], v[3]), b3 = mul_mi<INV>(csub(v[1], v[3]));
  v[0] = cadd(b0, b2); v[2] = csub(b0, b2);
  v[1] = cadd(b1, b3); v[3] = csub(b1, b3);
}

template <bool INV> __device__ __forceinline__ void dft8(double2* x) {
  constexpr double R2 = 0.70710678118654752440;
  double2 u[4], w[4];
#pragma unroll
  for (int n = 0; n < 4; n++) { u[n] = cadd(x[n], x[n + 4]); w[n] = csub(x[n], x[n + 4]); }
  // w[n] *= W8^n  (forward: exp(-i*pi*n/4))
  {
    double2 t = w[1];
    w[1] = INV ? make_double2(R2 * (t.x - t.y), R2 * (t.x + t.y)) : make_double2(R2 * (t.x + t.y), R2 * (t.y - t.x));
    w[2] = mul_mi<INV>(w[2]);
    t = w[3];
    w[3] = INV ? make_double2(-R2 * (t.x + t.y), R2 * (t.x - t.y)) : make_double2(R2 * (t.y - t.x), -R2 * (t.x + t.y));
  }
  dft4<INV>(u);
  dft4<INV>(w);
  x[0] = u[0]; x[1] = w[0]; x[2] = u[1]; x[3] = w[1];
  x[4] = u[2]; x[5] = w[2]; x[6] = u[3]; x[7] = w[3];
}

template <int R, bool INV> __device__ __forceinline__ void dftR(double2* v) {
  if constexpr (R == 8) dft8<INV>(v);
  else if constexpr (R == 4) dft4<INV>(v);
  else dft2<INV>(v[0], v[1]);
}

// v[r] *= w^r, r = 1..R-1, from w1 = W^st (conjugated for the inverse).
template <int R, bool INV>
__device__ __forceinline__ void twiddle_row_w(double2* v, double2 w1) {
  if (INV) w1 = conj2(w1);
  v[1] = cmul(v[1], w1);
  if constexpr (R >= 4) {
    const double2 w2 = cmul(w1, w1);
    const double2 w3 = cmul(w2, w1);
    v[2] = cmul(v[2], w2);
    v[3] = cmul(v[3], w3);
    if constexpr (R == 8) {
      const double2 w4 = cmul(w2, w2);
      v[4] = cmul(v[4], w4);
      v[5] = cmul(v[5], cmul(w4, w1));
      v[6] = cmul(v[6], cmul(w3, w3));
      v[7] = cmul(v[7], cmul(w4, w3));
    }
  }
}

template <int R, bool INV>
__device__ __forceinline__ void twiddle_row(double2* v, const double2* __restrict__ tw, int m) {
  twiddle_row_w<R, INV>(v, tw[m]);
}

// One Stockham pass of radix R over an N-point array using threads [0, T).
// Threads >= T only take part in the barrier.
template <int N, int T, int R, bool INV>
__device__ __forceinline__ void stockham_pass(CBuf x, int Ns, const double2* __restrict__ tw, int tid) {
  constexpr int NB = N / R;                       // butterflies in this pass
  constexpr int BPT = NB >= T ? NB / T : 1;       // butterflies per active thread
  constexpr int TA = NB >= T ? T : NB;            // active threads
  constexpr int TWS = TW_N / N;
  double2 v[BPT][R];
  // Launder tid per pass: the LDS addresses depend only on tid and constants,
  // and without this the compiler hoists every pass's addresses of every
  // transform in the kernel to its start (and spills them).
  asm volatile("" : "+v"(tid));
  const bool act = tid < TA;
  if (act) {
#pragma unroll
    for (int b = 0; b < BPT; b++) {
      const int j = tid + b * TA;
#pragma unroll
      for (int r = 0; r < R; r++) v[b][r] = x[j + r * NB];
      const int k = j & (Ns - 1);
      if (Ns > 1) twiddle_row<R, INV>(v[b], tw, (N / (Ns * R)) * k * TWS);
      dftR<R, INV>(v[b]);
    }
  }
  __syncthreads();
  asm volatile("" : "+v"(tid));
  if (act) {
#pragma unroll
    for (int b = 0; b < BPT; b++) {
      const int j = tid + b * TA;
      const int k = j & (Ns - 1);
      const int base = (j - k) * R + k;
#pragma unroll
      for (int r = 0; r < R; r++) x[base + r * Ns] = v[b][r];
    }
  }
  __syncthreads();
}

template <int N> struct Log2 { static constexpr int v = 1 + Log2<N / 2>::v; };
template <> struct Log2<1> { static constexpr int v = 0; };

// In-place N-point FFT (unnormalised), natural order in and out.  Begins with a
// barrier so callers may write the input right before calling; ends with one.
template <int N, int T, bool INV>
__device__ __forceinline__ void fft_lds(CBuf x, const double2* __restrict__ tw, int tid) {
  __syncthreads();
  constexpr int L = Log2<N>::v;
  int Ns = 1;
#pragma unroll
  for (int p = 0; p < L / 3; p++) { stockham_pass<N, T, 8, INV>(x, Ns, tw, tid); Ns *= 8; }
  if constexpr (L % 3 == 1) stockham_pass<N, T, 2, INV>(x, Ns, tw, tid);
  if constexpr (L % 3 == 2) stockham_pass<N, T, 4, INV>(x, Ns, tw, tid);
}

}  // namespace ldg
