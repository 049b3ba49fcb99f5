// Workgroup-level FP64 FFT for gfx950, LDS-resident, Stockham autosort.
//
// Data lives in two LDS arrays (re / im, structure-of-arrays) indexed through
// PAD(i) = i + i/8: one pad double every 8 keeps the stride-R writes of the
// early Stockham passes conflict-free for ds_write_b64 (bank = dword mod 32)
// while the unit-stride reads stay conflict-free.  An 8192-point complex FFT
// therefore needs 2 * 9216 * 8 B = 144 KiB of the 160 KiB LDS.
//
// Twiddles come from one global table W[m] = exp(-2*pi*i*m/16384), m < 16384
// (L2/Infinity-cache resident); an N-point transform uses stride 16384/N.
// All sizes and radices are compile-time, every pass is a full
// load -> barrier -> store -> barrier round over the workgroup.
#pragma once
#include <hip/hip_runtime.h>

namespace ldg {

constexpr int TW_N = 16384;

__device__ __forceinline__ constexpr int PAD(int i) { return i + (i >> 3); }

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

__device__ __forceinline__ double2 twiddle(const double2* __restrict__ tw, int m, bool inv) {
  double2 w = tw[m];
  return inv ? conj2(w) : w;
}

// One Stockham pass of radix R over an N-point array using threads [0, T).
// Threads >= T only take part in the two barriers.
template <int N, int T, int R, bool INV>
__device__ __forceinline__ void stockham_pass(double* re, double* im, int Ns, const double2* __restrict__ tw, int tid) {
  constexpr int NB = N / R;                       // butterflies in this pass
  constexpr int BPT = NB >= T ? NB / T : 1;       // butterflies per active thread
  constexpr int TA = NB >= T ? T : NB;            // active threads
  constexpr int TWS = TW_N / N;
  double2 v[BPT][R];
  const bool act = tid < TA;
  if (act) {
#pragma unroll
    for (int b = 0; b < BPT; b++) {
      const int j = tid + b * TA;
#pragma unroll
      for (int r = 0; r < R; r++) { const int i = PAD(j + r * NB); v[b][r] = make_double2(re[i], im[i]); }
      const int k = j & (Ns - 1);
      if (Ns > 1) {
        const int st = (N / (Ns * R)) * k;
#pragma unroll
        for (int r = 1; r < R; r++) v[b][r] = cmul(v[b][r], twiddle(tw, r * st * TWS, INV));
      }
      dftR<R, INV>(v[b]);
    }
  }
  __syncthreads();
  if (act) {
#pragma unroll
    for (int b = 0; b < BPT; b++) {
      const int j = tid + b * TA;
      const int k = j & (Ns - 1);
      const int base = (j - k) * R + k;
#pragma unroll
      for (int r = 0; r < R; r++) { const int i = PAD(base + r * Ns); re[i] = v[b][r].x; im[i] = v[b][r].y; }
    }
  }
  __syncthreads();
}

template <int N> struct Log2 { static constexpr int v = 1 + Log2<N / 2>::v; };
template <> struct Log2<1> { static constexpr int v = 0; };

// In-place N-point FFT (unnormalised), natural order in and out.  Begins with a
// barrier so callers may write the input right before calling.
template <int N, int T, bool INV>
__device__ __forceinline__ void fft_lds(double* re, double* im, const double2* __restrict__ tw, int tid) {
  __syncthreads();
  constexpr int L = Log2<N>::v;
  int Ns = 1;
#pragma unroll
  for (int p = 0; p < L / 3; p++) { stockham_pass<N, T, 8, INV>(re, im, Ns, tw, tid); Ns *= 8; }
  if constexpr (L % 3 == 1) stockham_pass<N, T, 2, INV>(re, im, Ns, tw, tid);
  if constexpr (L % 3 == 2) stockham_pass<N, T, 4, INV>(re, im, Ns, tw, tid);
}

}  // namespace ldg
