// Latency microbenchmark: a serial FP64 recurrence y = u - a*y on one lane
// (the comb's FilterIQ chain), with / without per-step LDS stores, alone and
// beside busy waves.  hipcc --offload-arch=gfx950 -O3 lat.hip -o lat
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ void chain(const double* __restrict__ in, double* __restrict__ out, unsigned long long* cyc, int nbusy) {
  __shared__ double s_u[1024];
  __shared__ double s_d[2048];
  const int tid = threadIdx.x;
  for (int i = tid; i < 1024; i += blockDim.x) s_u[i] = in[i];
  __syncthreads();
  if (tid == 0) {
    unsigned long long t0 = __builtin_readcyclecounter();
    double y = 0.0;
    const double a = -0.5465122036406802;
#pragma unroll 1
    for (int kb = 0; kb < 1024; kb += 16) {
      double us[16];
#pragma unroll
      for (int j = 0; j < 16; j++) us[j] = s_u[kb + j];
#pragma unroll
      for (int j = 0; j < 16; j++) {
        y = us[j] - a * y;
        if (MODE == 1) { s_d[2 * (kb + j)] = y; s_d[2 * (kb + j) + 1] = y; }
      }
    }
    unsigned long long t1 = __builtin_readcyclecounter();
    cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x] = y + s_d[5];
  } else if (tid >= 64 && tid < 64 + 64 * nbusy) {
    double z = in[tid];
    for (int i = 0; i < 20000; i++) z = z * 1.0000001 + 1e-9;
    out[1000 + tid] = z;
  }
}

int main() {
  double *in, *out;
  unsigned long long* cyc;
  hipMalloc(&in, 8192 * 8);
  hipMalloc(&out, 8192 * 8);
  hipMalloc(&cyc, 1024 * 8);
  hipMemset(in, 0, 8192 * 8);
  unsigned long long h[4];
  for (int mode = 0; mode < 2; mode++)
    for (int busy = 0; busy <= 3; busy += 3) {
      for (int rep = 0; rep < 2; rep++) {
        if (mode == 0) chain<0><<<1, 256>>>(in, out, cyc, busy);
        else chain<1><<<1, 256>>>(in, out, cyc, busy);
        hipDeviceSynchronize();
      }
      hipMemcpy(h, cyc, 8, hipMemcpyDeviceToHost);
      printf("mode %d (lds stores %s) busy waves %d: %.1f cycles per step\n", mode, mode ? "yes" : "no", busy,
             h[0] / 1024.0);
    }
  return 0;
}
