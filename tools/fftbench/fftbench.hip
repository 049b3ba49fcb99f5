// Microbenchmark of the workgroup FFT (fft.hpp): R back-to-back 8192-point
// transforms per workgroup, one workgroup per CU slot, timed with HIP events.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off fftbench.hip -o fftbench && ./fftbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>
#include "../../ld-decode_amd/csrc/fft8k.hpp"
using namespace ldg;

constexpr int M = 8192, T = 1024;

template <int REPS, int KIND>
__global__ __launch_bounds__(1024) void k_fft(const double2* __restrict__ in, double2* __restrict__ out,
                                              const double2* __restrict__ tw) {
  __shared__ double2 s_x[M];
  __shared__ double2 s_a[2048];
  const CBuf X_{s_x};
  const int tid = threadIdx.x;
  const double2* src = in + (size_t)(blockIdx.x & 63) * M;
#pragma unroll
  for (int q = 0; q < 8; q++) X_[tid + T * q] = src[tid + T * q];
  if (tid == 0) s_a[0] = src[0];
  for (int r = 0; r < REPS; r++) {
    if (KIND == 0) {
      if (r & 1) fft_lds<M, T, true>(X_, tw, tid);
      else fft_lds<M, T, false>(X_, tw, tid);
    } else {
      if (r & 1) fft8k_dit<true>(s_x, tw, tid);
      else fft8k_dif<false>(s_x, tw, tid);
    }
  }
  double2* dst = out + (size_t)(blockIdx.x & 63) * M;
#pragma unroll
  for (int q = 0; q < 8; q++) dst[tid + T * q] = X_[tid + T * q];
}

int main(int argc, char** argv) {
  const int nblk = argc > 1 ? atoi(argv[1]) : 4096;
  std::vector<double2> tw(TW_N), in((size_t)64 * M);
  for (int m = 0; m < TW_N; m++) {
    long double a = -2.0L * 3.14159265358979323846264338327950288L * m / TW_N;
    tw[m] = make_double2((double)cosl(a), (double)sinl(a));
  }
  for (size_t i = 0; i < in.size(); i++) in[i] = make_double2(sin(0.001 * i), cos(0.0007 * i));
  double2 *d_tw, *d_in, *d_out;
  hipMalloc(&d_tw, TW_N * sizeof(double2));
  hipMalloc(&d_in, in.size() * sizeof(double2));
  hipMalloc(&d_out, in.size() * sizeof(double2));
  hipMemcpy(d_tw, tw.data(), TW_N * sizeof(double2), hipMemcpyHostToDevice);
  hipMemcpy(d_in, in.data(), in.size() * sizeof(double2), hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  std::vector<double2> out(in.size()), ref(in.size());
  auto run = [&](auto k1, auto k9, auto k2, const char* name) {
    float ms1 = 0, ms9 = 0;
    for (int it = 0; it < 3; it++) {
      hipEventRecord(e0);
      k1<<<nblk, 1024>>>(d_in, d_out, d_tw);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&ms1, e0, e1);
      hipEventRecord(e0);
      k9<<<nblk, 1024>>>(d_in, d_out, d_tw);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&ms9, e0, e1);
    }
    k2<<<64, 1024>>>(d_in, d_out, d_tw);
    hipMemcpy(out.data(), d_out, out.size() * sizeof(double2), hipMemcpyDeviceToHost);
    double err = 0;
    for (size_t i = 0; i < out.size(); i++)
      err = fmax(err, fmax(fabs(out[i].x / M - in[i].x), fabs(out[i].y / M - in[i].y)));
    const double per_fft_us = (ms9 - ms1) / 8.0 * 1e3 / nblk * 256;
    printf("%-10s blocks %d  1 fft %.3f ms  9 ffts %.3f ms  per-FFT %.2f CU-us  roundtrip err %.3g\n", name, nblk, ms1,
           ms9, per_fft_us, err);
  };
  run(k_fft<1, 0>, k_fft<9, 0>, k_fft<2, 0>, "stockham");
  run(k_fft<1, 1>, k_fft<9, 1>, k_fft<2, 1>, "fourstep");
  // forward spectra agree (digit-reversed positions)
  k_fft<1, 0><<<64, 1024>>>(d_in, d_out, d_tw);
  hipMemcpy(ref.data(), d_out, ref.size() * sizeof(double2), hipMemcpyDeviceToHost);
  k_fft<1, 1><<<64, 1024>>>(d_in, d_out, d_tw);
  hipMemcpy(out.data(), d_out, out.size() * sizeof(double2), hipMemcpyDeviceToHost);
  double e = 0, mx = 0;
  for (int b = 0; b < 64; b++)
    for (int k = 0; k < M; k++) {
      // k_fft writes X_[i] (swizzled read of natural index i) -> position i holds bin dr_nat(i)
      const double2 r = ref[(size_t)b * M + dr_nat(k)], o = out[(size_t)b * M + k];
      e = fmax(e, fmax(fabs(r.x - o.x), fabs(r.y - o.y)));
      mx = fmax(mx, fabs(r.x));
    }
  printf("forward spectra max |diff| %.3g (max |X| %.3g)\n", e, mx);
  return 0;
}
