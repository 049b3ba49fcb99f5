// Compact sync and burst channels.
//
// The demod computes demod_sync and demod_burst as periodic recurrences over
// 16-sample chunks (iir.hpp).  Instead of storing every sample (8 B each, two of
// the four channels' HBM stores), it stores per chunk the state that enters it:
//   sync : y[16g - 1] (double) and the detector bits of the chunk plus the bit
//          before it (uint32: bits 0-15, bit 16);
//   burst: (y[16g - 1], y[16g - 2], x[16g - 1], x[16g - 2]) (double4), x = demod.
// Chunk g of a read covers outputs [16 g, 16 g + 16): overlap-save blocks keep
// 15328 = 16 * 958 outputs from block position 1024 = 16 * 64, so chunks never
// straddle blocks and the read's chunk grid is every block's.  A field kernel
// that needs sync / burst at output n reruns the chunk's recurrence from its
// state with the demod's own steps (iir.hpp sync_step / sos_step), so the value
// is bit-identical to the one the demod computed.  The sync tiles (common.hpp)
// are still written by the demod from the full channel.
#pragma once
#include "common.hpp"
#include "iir.hpp"

namespace ldg {

constexpr int64_t CHUNKS_PER_SLOT = MAX_NOUT / IIR_CHUNK + 2;

// demod_sync of one read at output n.
struct SyncSrc {
  const double* st;      // [CHUNKS_PER_SLOT] of this slot
  const uint32_t* bits;  // [CHUNKS_PER_SLOT]
  double b0, p;
  __device__ SyncSrc(const double* sst, const uint32_t* sbits, int slot, const SysConst& C)
      : st(sst + (int64_t)slot * CHUNKS_PER_SLOT), bits(sbits + (int64_t)slot * CHUNKS_PER_SLOT),
        b0(C.sy_b0), p(C.sy_p) {}
  __device__ double operator[](int64_t n) const {
    const int64_t g = n >> 4;
    const int i = (int)(n & 15);
    double y = st[g];
    const uint32_t w = bits[g];
    uint32_t prev = (w >> 16) & 1u;
    for (int k = 0; k <= i; k++) {
      const uint32_t x = (w >> k) & 1u;
      y = sync_step(y, x, prev, b0, p);
      prev = x;
    }
    return y;
  }
};

// demod_burst of one read from the demod channel and the chunk states.
struct BurstSrc {
  const double4* st;     // [CHUNKS_PER_SLOT] of this slot
  const double* dm;      // demod channel of this slot
  double b0, b1, b2, a1, a2;
  __device__ BurstSrc(const double4* bst, const double* demod, int slot, const SysConst& C)
      : st(bst + (int64_t)slot * CHUNKS_PER_SLOT), dm(demod), b0(C.bu_b0), b1(C.bu_b1), b2(C.bu_b2),
        a1(C.bu_a1), a2(C.bu_a2) {}
  // outputs [n0, n1] of chunk g (16 g <= n0 <= n1 < 16 g + 16) into dst[n - n0]
  __device__ void chunk(int64_t g, int64_t n0, int64_t n1, double* dst) const {
    const double4 s = st[g];
    double s0 = s.x, s1 = s.y, xa = s.z, xb = s.w;
    const double* x = dm + 16 * g;
    double xv[IIR_CHUNK];
#pragma unroll
    for (int k = 0; k < IIR_CHUNK; k++) xv[k] = (16 * g + k <= n1) ? x[k] : 0.0;
#pragma unroll
    for (int k = 0; k < IIR_CHUNK; k++) {
      if (16 * g + k > n1) break;
      const double v = sos_step(xv[k], xa, xb, s0, s1, b0, b1, b2, a1, a2);
      s1 = s0;
      s0 = v;
      xb = xa;
      xa = xv[k];
      if (16 * g + k >= n0) dst[16 * g + k - n0] = v;
    }
  }
  __device__ double operator[](int64_t n) const {
    double v;
    chunk(n >> 4, n, n, &v);
    return v;
  }
  // outputs [n0, n1] into dst[n - n0], the chunks shared out over nt threads
  __device__ void window(int64_t n0, int64_t n1, double* dst, int tid, int nt) const {
    for (int64_t g = (n0 >> 4) + tid; g <= (n1 >> 4); g += nt) {
      const int64_t a = (16 * g > n0) ? 16 * g : n0, b = (16 * g + 15 < n1) ? 16 * g + 15 : n1;
      chunk(g, a, b, dst + (a - n0));
    }
  }
};

}  // namespace ldg

// Debug / test path (ldg_debug_read): expand one read's compact sync (what 2) or
// burst (what 3) channel into its full-rate video channel slot.  grid: chunks / 64
// workgroups of 64 threads, one chunk per thread.
extern "C" __global__ __launch_bounds__(64) void ldg_k_chan_expand(
    const double* __restrict__ sst, const uint32_t* __restrict__ sbits, const double4* __restrict__ bst,
    double* __restrict__ video, int64_t vread_stride, int64_t vchan_stride, ldg::SysConst C, int slot, int what,
    int64_t n_out) {
  using namespace ldg;
  const int64_t g = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (16 * g >= n_out) return;
  const int64_t n1 = (16 * g + 15 < n_out) ? 16 * g + 15 : n_out - 1;
  double* rd = video + (int64_t)slot * vread_stride;
  if (what == CH_SYNC) {
    const SyncSrc s(sst, sbits, slot, C);
    for (int64_t n = 16 * g; n <= n1; n++) rd[(int64_t)CH_SYNC * vchan_stride + n] = s[n];
  } else {
    const BurstSrc b(bst, rd + (int64_t)CH_DEMOD * vchan_stride, slot, C);
    b.chunk(g, 16 * g, n1, rd + (int64_t)CH_BURST * vchan_stride + 16 * g);
  }
}
