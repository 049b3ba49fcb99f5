// demod_05 without its full-rate channel.
//
// The reference's 0.5 MHz channel is demod_05 = roll(ifft(D * FVideo05), -32)
// with FVideo05 = FVideo * F05 and F05 the freqz of a 65-tap FIR
// (lddecode_core.py:199-202, 302-303).  The sampled FIR response makes the
// block's inverse transform a circular convolution of the block's video
// (ifft(D * FVideo), the demod channel) with the 65 taps h, so at a kept block
// position p (in [1024, 1024 + copylen))
//     demod_05[p] = sum_j h[j] * video[p + 32 - j],   j = 0..64,
// a window [p - 32, p + 32] of the SAME block.  Inside the kept range those
// video samples are the demod channel itself; the 32 positions before it
// ([992, 1024)) and the 32 after it (1024 + copylen .., mod 16384) are not
// kept, so the demod stores them per block ("halo", 64 doubles per block:
// 0.4% of the channel) instead of the whole 8 B/sample demod_05 channel, and
// the consumers (refine_linelocs_hsync's windows, the PAL pilot windows, the
// debug expander) rebuild the few demod_05 samples they read.  The FIR form
// differs from the FFT form by rounding only (~1e-15 relative).
#pragma once
#include "common.hpp"

namespace ldg {

constexpr int F05_TAPS = 65;
constexpr int D05_HALO = 64;                 // doubles per block: head [0, 32), tail [32, 64)

// copylen of block b of a read with n_out outputs (lddecode_core.py:402-405: the
// last block keeps n_out - off when off + 15360 passes n_out)
__device__ __forceinline__ int block_copylen(int b, int64_t n_out) {
  const int64_t off = (int64_t)b * BLOCKSTEP;
  return (off + (BLOCKLEN - BLOCKCUT) > n_out) ? (int)(n_out - off) : BLOCKSTEP;
}

// demod_05 of one read, evaluated from the demod channel and the block halos.
struct D05Src {
  const double* dm;      // demod channel of the slot (index = read output)
  const double* halo;    // [MAX_BLOCKS_PER_READ][D05_HALO] of the slot
  const double* h;       // the 65 taps
  int64_t n_out;
  int nb;                // blocks of the read
  int64_t o;             // index offset (D05Src + k)
  __device__ D05Src(const double* demod, const double* halos, int slot, const double* taps, int64_t n, int nblocks)
      : dm(demod), halo(halos + (int64_t)slot * MAX_BLOCKS_PER_READ * D05_HALO), h(taps), n_out(n), nb(nblocks),
        o(0) {}
  __device__ D05Src operator+(int64_t k) const {
    D05Src r = *this;
    r.o += k;
    return r;
  }
  __device__ __forceinline__ int block_of(int64_t n) const {
    const int b = (int)(n / BLOCKSTEP);
    return b < nb - 1 ? b : nb - 1;
  }
  // video at kept-relative position i of block b (i in [-32, copylen + 32))
  __device__ __forceinline__ double vid(int b, int64_t off, int cl, int i) const {
    if (i >= 0 && i < cl) return dm[off + i];
    return halo[(int64_t)b * D05_HALO + (i < 0 ? 32 + i : 32 + (i - cl))];
  }
  __device__ double operator[](int64_t k) const {
    const int64_t n = k + o;
    const int b = block_of(n);
    const int64_t off = (int64_t)b * BLOCKSTEP;
    const int cl = block_copylen(b, n_out);
    const int p = (int)(n - off);
    double s = 0.0;
#pragma unroll 5
    for (int j = 0; j < F05_TAPS; j++) s = __fma_rn(h[j], vid(b, off, cl, p + 32 - j), s);
    return s;
  }
};

// demod_05 outputs [lo, hi) of one read staged in LDS by one wave: the demod
// samples [lo - 32, hi + 32) are loaded once (coalesced) into s_vid, each output
// is the FIR over s_vid, or over the halo where its window leaves its block.
// Every lane of the wave calls this; the outputs land in s_out[k - lo].
__device__ inline void d05_fill(const D05Src& src, double* s_vid, double* s_out, int64_t lo, int64_t hi, int lane) {
  const int64_t vlo = lo - 32;
  for (int64_t k = vlo + lane; k < hi + 32; k += 64)
    s_vid[k - vlo] = (k >= 0 && k < src.n_out) ? src.dm[k] : 0.0;
  __syncthreads();
  // D05_ILP outputs per lane at once (n, n + 64, ...): independent FMA chains, each
  // in the taps' ascending order as in D05Src (the same doubles)
  constexpr int D05_ILP = 4;
  for (int64_t n0 = lo + lane; n0 < hi; n0 += 64 * D05_ILP) {
    bool fast = true;
#pragma unroll
    for (int u = 0; u < D05_ILP; u++) {
      const int64_t n = n0 + 64 * u;
      if (n >= hi) break;
      const int b = src.block_of(n);
      const int p = (int)(n - (int64_t)b * BLOCKSTEP);
      fast = fast && p >= 32 && p + 32 < block_copylen(b, src.n_out);
    }
    if (fast && n0 + 64 * (D05_ILP - 1) < hi) {
      const double* w = s_vid + (n0 - vlo) + 32;
      double s[D05_ILP] = {};
#pragma unroll 5
      for (int j = 0; j < F05_TAPS; j++) {
        const double hj = src.h[j];
#pragma unroll
        for (int u = 0; u < D05_ILP; u++) s[u] = __fma_rn(hj, w[64 * u - j], s[u]);
      }
#pragma unroll
      for (int u = 0; u < D05_ILP; u++) s_out[n0 + 64 * u - lo] = s[u];
      continue;
    }
    for (int64_t n = n0; n < hi && n < n0 + 64 * D05_ILP; n += 64) {
      const int b = src.block_of(n);
      const int64_t off = (int64_t)b * BLOCKSTEP;
      const int cl = block_copylen(b, src.n_out);
      const int p = (int)(n - off);
      double s = 0.0;
      if (p >= 32 && p + 32 < cl) {
        const double* w = s_vid + (n - vlo) + 32;
#pragma unroll 5
        for (int j = 0; j < F05_TAPS; j++) s = __fma_rn(src.h[j], w[-j], s);
      } else {
#pragma unroll 5
        for (int j = 0; j < F05_TAPS; j++) s = __fma_rn(src.h[j], src.vid(b, off, cl, p + 32 - j), s);
      }
      s_out[n - lo] = s;
    }
  }
  __syncthreads();
}

// an LDS-staged demod_05 window read by absolute output index (D05Win + k as for a pointer)
struct D05Win {
  const double* w;
  int64_t base;
  __device__ double operator[](int64_t k) const { return w[k - base]; }
  __device__ D05Win operator+(int64_t k) const { return {w, base - k}; }
};

}  // namespace ldg

// Debug / test path (ldg_debug_read what = 1): rebuild one read's demod_05 into its
// full-rate video channel slot.  grid: ceil(n_out / 256) workgroups of 256 threads.
extern "C" __global__ __launch_bounds__(256) void ldg_k_d05_expand(double* __restrict__ video, int64_t vread_stride,
                                                                  int64_t vchan_stride,
                                                                  const double* __restrict__ d05halo,
                                                                  const double* __restrict__ f05, int slot,
                                                                  int64_t n_out, int n_blocks) {
  using namespace ldg;
  const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (n >= n_out) return;
  double* rd = video + (int64_t)slot * vread_stride;
  const D05Src src(rd + (int64_t)CH_DEMOD * vchan_stride, d05halo, slot, f05, n_out, n_blocks);
  rd[(int64_t)CH_05 * vchan_stride + n] = src[n];
}
