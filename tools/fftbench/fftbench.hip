// Microbenchmark of the workgroup 8192-point FFTs: R back-to-back transforms per
// workgroup (alternating forward / inverse), timed with HIP events.
//   fourstep: fft8k.hpp, 1024 threads, data in 128 KiB of LDS (one workgroup per CU)
//   regs512:  fft8k_h.hpp, 512 threads, data in registers, 64 KiB of LDS (two per CU)
// Also checks both against a host FFT (forward spectra, inverse round trip).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -mllvm --amdgpu-sched-strategy=max-ilp \
//     fftbench.hip -o fftbench && ./fftbench [workgroups]
#include <hip/hip_runtime.h>
#include <cmath>
#include <complex>
#include <cstdio>
#include <vector>
#include "../../ld-decode_amd/csrc/fft8k_h.hpp"
using namespace ldg;

constexpr int M = 8192;

template <int REPS>
__global__ __launch_bounds__(1024) void k_fourstep(const double2* __restrict__ in, double2* __restrict__ out,
                                                   const double2* __restrict__ tw) {
  __shared__ double2 s_x[M];
  __shared__ double2 s_tw[TW_LDS_N];
  const int tid = threadIdx.x;
  s_tw[tw_lds_pos(tid)] = tw[2 * tid];
  const TwLds twl{s_tw};
  const double2* src = in + (size_t)(blockIdx.x & 63) * M;
  const CBuf X_{s_x};
#pragma unroll
  for (int q = 0; q < 8; q++) X_[tid + 1024 * q] = src[tid + 1024 * q];
#pragma clang loop unroll(disable)
  for (int r = 0; r < REPS / 2; r++) {
    fft8k_dif<false>(s_x, tw, twl, tid);
    fft8k_dit<true>(s_x, tw, twl, tid);
  }
  if (REPS & 1) fft8k_dif<false>(s_x, tw, twl, tid);
  double2* dst = out + (size_t)(blockIdx.x & 63) * M;
#pragma unroll
  for (int q = 0; q < 8; q++) dst[tid + 1024 * q] = X_[tid + 1024 * q];
}

template <int REPS>
__global__ __launch_bounds__(512, 4) void k_regs512(const double2* __restrict__ in, double2* __restrict__ out,
                                                    const double2* __restrict__ tw) {
  __shared__ double2 ex[h8k::EX];
  int t = threadIdx.x;
  const double2* src = in + (size_t)(blockIdx.x & 63) * M;
  double2 v[16];
#pragma unroll
  for (int r = 0; r < 16; r++) v[r] = src[t + 512 * r];
#pragma clang loop unroll(disable)
  for (int r = 0; r < REPS / 2; r++) {
    h8k::fwd<false>(v, ex, tw, t);
    h8k::inv<true>(v, ex, tw, t);
  }
  if (REPS & 1) h8k::fwd<false>(v, ex, tw, t);
  asm volatile("" : "+v"(t));
  double2* dst = out + (size_t)(blockIdx.x & 63) * M;
  if (REPS & 1) {
    // spectral layout -> natural bin order
    const int w = t >> 6, l = t & 63;
#pragma unroll
    for (int s = 0; s < 2; s++)
#pragma unroll
      for (int d = 0; d < 8; d++) dst[h8k::bin_of(w, s, l, d)] = v[8 * s + d];
  } else {
#pragma unroll
    for (int r = 0; r < 16; r++) dst[t + 512 * r] = v[r];
  }
}

static void host_fft(std::vector<std::complex<long double>>& a) {
  const int n = (int)a.size();
  for (int i = 1, j = 0; i < n; i++) {
    int bit = n >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j ^= bit;
    if (i < j) std::swap(a[i], a[j]);
  }
  for (int len = 2; len <= n; len <<= 1) {
    const long double ang = -2.0L * 3.14159265358979323846264338327950288L / len;
    for (int i = 0; i < n; i += len)
      for (int k = 0; k < len / 2; k++) {
        const std::complex<long double> w(cosl(ang * k), sinl(ang * k));
        const auto u = a[i + k], v = a[i + k + len / 2] * w;
        a[i + k] = u + v;
        a[i + k + len / 2] = u - v;
      }
  }
}

int main(int argc, char** argv) {
  const int nblk = argc > 1 ? atoi(argv[1]) : 6144;
  std::vector<double2> tw(TW_N), in((size_t)64 * M);
  for (int m = 0; m < TW_N; m++) {
    long double a = -2.0L * 3.14159265358979323846264338327950288L * m / TW_N;
    tw[m] = make_double2((double)cosl(a), (double)sinl(a));
  }
  for (size_t i = 0; i < in.size(); i++) in[i] = make_double2(sin(0.001 * i) + 0.3 * cos(0.37 * i * i), cos(0.0007 * i));
  double2 *d_tw, *d_in, *d_out;
  (void)hipMalloc(&d_tw, TW_N * sizeof(double2));
  (void)hipMalloc(&d_in, in.size() * sizeof(double2));
  (void)hipMalloc(&d_out, in.size() * sizeof(double2));
  (void)hipMemcpy(d_tw, tw.data(), TW_N * sizeof(double2), hipMemcpyHostToDevice);
  (void)hipMemcpy(d_in, in.data(), in.size() * sizeof(double2), hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  // host reference spectra of the first 4 inputs
  std::vector<std::vector<std::complex<long double>>> ref(4);
  double mx = 0;
  for (int b = 0; b < 4; b++) {
    ref[b].resize(M);
    for (int i = 0; i < M; i++) ref[b][i] = {in[(size_t)b * M + i].x, in[(size_t)b * M + i].y};
    host_fft(ref[b]);
    for (auto& z : ref[b]) mx = fmax(mx, (double)std::abs(z));
  }
  std::vector<double2> out(in.size());
  auto check = [&](auto k1, auto k2, int threads, const char* name, bool dr) {
    k1<<<64, threads>>>(d_in, d_out, d_tw);
    (void)hipMemcpy(out.data(), d_out, out.size() * sizeof(double2), hipMemcpyDeviceToHost);
    double e = 0;
    for (int b = 0; b < 4; b++)
      for (int k = 0; k < M; k++) {
        const double2 o = out[(size_t)b * M + (dr ? dr_pos(k) : k)];
        e = fmax(e, (double)std::abs(std::complex<long double>(o.x, o.y) - ref[b][k]));
      }
    k2<<<64, threads>>>(d_in, d_out, d_tw);
    (void)hipMemcpy(out.data(), d_out, out.size() * sizeof(double2), hipMemcpyDeviceToHost);
    double er = 0;
    for (size_t i = 0; i < out.size(); i++)
      er = fmax(er, fmax(fabs(out[i].x / M - in[i].x), fabs(out[i].y / M - in[i].y)));
    printf("%-10s forward max|err| %.3g (rel %.3g), round trip %.3g\n", name, e, e / mx, er);
  };
  auto time = [&](auto k1, auto k9, int threads, const char* name) {
    float ms1 = 1e9, ms9 = 1e9;
    for (int it = 0; it < 5; it++) {
      float a = 0, b = 0;
      (void)hipEventRecord(e0);
      k1<<<nblk, threads>>>(d_in, d_out, d_tw);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      (void)hipEventElapsedTime(&a, e0, e1);
      (void)hipEventRecord(e0);
      k9<<<nblk, threads>>>(d_in, d_out, d_tw);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      (void)hipEventElapsedTime(&b, e0, e1);
      ms1 = fminf(ms1, a);
      ms9 = fminf(ms9, b);
    }
    const double per_fft_us = (ms9 - ms1) / 8.0 * 1e3 / nblk * 256;
    printf("%-10s blocks %d  1 fft %.3f ms  9 ffts %.3f ms  per-FFT %.2f CU-us (%.1f us per block-pair of transforms)\n",
           name, nblk, ms1, ms9, per_fft_us, per_fft_us);
  };
  check(k_fourstep<1>, k_fourstep<2>, 1024, "fourstep", true);
  check(k_regs512<1>, k_regs512<2>, 512, "regs512", false);
  time(k_fourstep<1>, k_fourstep<9>, 1024, "fourstep");
  time(k_regs512<1>, k_regs512<9>, 512, "regs512");
  return 0;
}
