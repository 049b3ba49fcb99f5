// Synthetic LaserDisc RF capture generator on the GPU (benchmark / test tooling,
// not part of the reference interface).  Same signal model as ldgpu/synth.py:
// composite NTSC baseband (sync, equalising/broad pulses, burst, colour bars,
// ramp, Philips VBI code) -> 63-tap band-limit FIR -> the reference's Femp
// pre-emphasis IIR (lddecode_core.py:190-192) -> FM at ire0 + hz_ire*IRE ->
// + two FM audio carriers + Gaussian noise -> u8 / s16 / .r30 / .lds.
//
// Chunked: each 4096-sample chunk recomputes a 1024-sample IIR warm-up
// (pole 0.926: 0.926^1024 ~ 1e-34) and a 62-sample FIR halo, so chunks are
// independent; the FM phase is stitched with a host prefix sum of per-chunk
// phase totals (pass 1), then pass 2 regenerates and writes the RF.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "common.hpp"

namespace {

constexpr int SY_CH = 4096;
constexpr int SY_WARM = 1024;
constexpr int SY_FIR = 63;
constexpr int SY_T = 256;
constexpr int SY_N = SY_CH + SY_WARM;            // IIR outputs per chunk
constexpr int SY_X = SY_N + SY_FIR - 1;          // baseband inputs per chunk
constexpr double SY_FS = 40e6;

struct SynthConst {
  double spl, t0_lines, H, fsc, ire0, hz_ire, sync, burst_ire;
  double b0, b1, a1;              // emphasis IIR y = b0 x + b1 x[-1] - a1 y[-1]
  double audio_l, audio_r, noise, amp_scale;
  double fir[SY_FIR];
  int32_t lines, fmt, clv, pad;
  uint64_t seed;
};

__device__ __forceinline__ uint64_t splitmix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__device__ double ire_at(const SynthConst& S, const uint32_t* __restrict__ codes, int64_t ncodeframes, int64_t n) {
  const double H = S.H;
  const int L = S.lines;
  const double la = (double)n / S.spl + S.t0_lines;
  const double hlf = floor(la * 2);
  const int64_t hl = (int64_t)hlf;
  const int64_t frame = hl / (2 * L);
  const int h = (int)(hl - frame * 2 * L);
  const double phi = (la * 2 - hlf) * (H / 2);
  const int ln = h / 2;
  const double tau = (la - floor(la)) * H;
  const double tus = (double)n / SY_FS * 1e6 + S.t0_lines * H;
  const bool vi1 = h < 18, vi2 = h >= 525 && h < 543;
  const int hv = vi1 ? h : h - 525;
  const bool in_vi = vi1 || vi2;
  const bool eq = in_vi && (hv < 6 || hv >= 12);
  const bool broad = in_vi && hv >= 6 && hv < 12;
  const bool normal = !in_vi && h != 543;
  const bool vbi = (ln >= 9 && ln < 20) || (ln >= 272 && ln < 283);
  double ire = 0.0;
  if (eq && phi < 2.35) ire = S.sync;
  if (broad && phi < H / 2 - 4.7) ire = S.sync;
  if (normal && tau < 4.7) ire = S.sync;
  const double w = 2 * 3.141592653589793 * S.fsc * (tus * 1e-6);
  if (normal && tau >= 5.3 && tau < 5.3 + 9 / (S.fsc / 1e6)) ire += S.burst_ire * sin(w + 3.141592653589793);
  const double a0 = 9.4, a1 = H - 1.5;
  if (normal && !vbi && tau >= a0 && tau < a1) {
    const double x = (tau - a0) / (a1 - a0);
    const int lnf = ln % (L / 2 + 1);
    const bool lower = lnf > (L / 2) * 2 / 3;
    int bar = (int)(x * 8);
    if (bar > 7) bar = 7;
    const double yl[8] = {77.0, 69.0, 56.0, 48.0, 36.0, 28.0, 15.0, 7.5};
    const double camp[8] = {0.0, 31.0, 44.0, 41.0, 41.0, 44.0, 31.0, 0.0};
    const double cph[8] = {0.0, 167.0, 283.0, 241.0, 61.0, 103.0, 347.0, 0.0};
    if (lower) ire = 100.0 * x;
    else ire = yl[bar] + camp[bar] * sin(w + cph[bar] * (3.141592653589793 / 180.0));
  }
  const int cl0[3] = {16, 17, 18}, cl1[3] = {279, 280, 281};
  if (normal) {
    for (int j = 0; j < 3; j++) {
      if (ln == cl0[j] || ln == cl1[j]) {
        const double c = floor((tau - 10.0) / 2.0);
        if (c >= 0 && c < 24 && frame < ncodeframes) {
          const uint32_t code = codes[frame * 3 + j];
          const int ci = (int)c;
          const bool second = ((tau - 10.0) - 2.0 * c) >= 1.0;
          const int bit = (code >> (23 - ci)) & 1;
          const bool high = bit ? second : !second;
          ire = high ? 100.0 : 0.0;
        }
      }
    }
  }
  return ire;
}

// Emphasised instantaneous frequency (Hz) for the chunk's SY_N outputs (warm-up
// first) into y[]; x[] is scratch of SY_X.
__device__ void chunk_freq(const SynthConst& S, const uint32_t* codes, int64_t ncf, int64_t c0, double* x,
                           double* y, double* carry) {
  const int tid = threadIdx.x;
  const int64_t xs = c0 - SY_WARM - (SY_FIR - 1);
  for (int i = tid; i < SY_X; i += SY_T) {
    const int64_t n = xs + i;
    x[i] = n < 0 ? S.ire0 : S.ire0 + S.hz_ire * ire_at(S, codes, ncf, n);
  }
  __syncthreads();
  // 63-tap FIR (np.convolve 'valid' over [history, chunk])
  for (int i = tid; i < SY_N; i += SY_T) {
    double acc = 0.0;
    for (int k = 0; k < SY_FIR; k++) acc += S.fir[k] * x[i + SY_FIR - 1 - k];
    y[i] = acc;
  }
  __syncthreads();
  // first-order IIR as a blocked affine scan: u[i] = b0 x[i] + b1 x[i-1]; y[i] = u[i] - a1 y[i-1]
  constexpr int SEG = SY_N / SY_T;     // 20 samples per thread
  const int s0 = tid * SEG;
  double u[SEG];
  for (int k = 0; k < SEG; k++) {
    const int i = s0 + k;
    const double xm = i ? y[i - 1] : S.ire0;
    u[k] = S.b0 * y[i] + S.b1 * xm;
  }
  __syncthreads();
  const double a = -S.a1;
  double loc = 0.0, ak = 1.0;
  for (int k = 0; k < SEG; k++) { loc = a * loc + u[k]; ak *= a; }
  carry[tid] = loc;
  carry[SY_T + tid] = ak;
  __syncthreads();
  if (tid == 0) {
    double st = S.ire0;   // steady state for the constant carrier before the warm-up
    for (int t = 0; t < SY_T; t++) {
      const double e = carry[t], m = carry[SY_T + t];
      carry[2 * SY_T + t] = st;
      st = m * st + e;
    }
  }
  __syncthreads();
  double st = carry[2 * SY_T + tid];
  for (int k = 0; k < SEG; k++) { st = a * st + u[k]; y[s0 + k] = st; }
  __syncthreads();
}

}  // namespace

// Chunk index = blk0 + blockIdx.x: a launch's work-items stay below 2^32 (the
// dispatch packet's grid size), so long captures (1 h = 35M chunks) take several launches.
extern "C" __global__ __launch_bounds__(256) void ldg_k_synth_pass1(SynthConst S, const uint32_t* __restrict__ codes,
                                                                    int64_t ncf, double* __restrict__ totals, int64_t blk0) {
  __shared__ double x[SY_X], y[SY_N], carry[3 * SY_T];
  const int64_t blk = blk0 + blockIdx.x;
  const int64_t c0 = blk * SY_CH;
  chunk_freq(S, codes, ncf, c0, x, y, carry);
  // total phase advance over the chunk's SY_CH samples (fixed order, reused in pass 2)
  if (threadIdx.x == 0) {
    double tot = 0.0;
    for (int i = 0; i < SY_CH; i++) tot += (2 * 3.141592653589793 / SY_FS) * y[SY_WARM + i];
    totals[blk] = tot;
  }
}

extern "C" __global__ __launch_bounds__(256) void ldg_k_synth_pass2(SynthConst S, const uint32_t* __restrict__ codes,
                                                                    int64_t ncf, const double* __restrict__ phase0,
                                                                    int64_t nsamples, uint8_t* __restrict__ out, int64_t blk0) {
  __shared__ double x[SY_X], y[SY_N], carry[3 * SY_T];
  const int64_t blk = blk0 + blockIdx.x;
  const int64_t c0 = blk * SY_CH;
  chunk_freq(S, codes, ncf, c0, x, y, carry);
  const int tid = threadIdx.x;
  // inclusive prefix of phase increments within the chunk (16 per thread + thread scan)
  constexpr int PER = SY_CH / SY_T;
  double loc[PER];
  double s = 0.0;
  for (int k = 0; k < PER; k++) { s += (2 * 3.141592653589793 / SY_FS) * y[SY_WARM + tid * PER + k]; loc[k] = s; }
  carry[tid] = s;
  __syncthreads();
  if (tid == 0) {
    double acc = phase0[blk];
    for (int t = 0; t < SY_T; t++) { const double v = carry[t]; carry[t] = acc; acc += v; }
  }
  __syncthreads();
  const double base = carry[tid];
  for (int k = 0; k < PER; k++) {
    const int64_t n = c0 + tid * PER + k;
    if (n >= nsamples) break;
    const double ph = base + loc[k];
    double rf = cos(ph);
    const double t = (double)n / SY_FS;
    const double fl = fmod((double)n * (S.audio_l / SY_FS), 1.0);
    const double fr = fmod((double)n * (S.audio_r / SY_FS), 1.0);
    rf += 0.1 * cos(2 * 3.141592653589793 * fl + (50000.0 / 1000.0) * sin(2 * 3.141592653589793 * 1000.0 * t));
    rf += 0.1 * cos(2 * 3.141592653589793 * fr + (50000.0 / 400.0) * sin(2 * 3.141592653589793 * 400.0 * t));
    if (S.noise > 0) {
      const uint64_t r1 = splitmix(S.seed ^ (uint64_t)n * 2ull), r2 = splitmix(S.seed ^ ((uint64_t)n * 2ull + 1));
      const double u1 = ((r1 >> 11) + 1.0) * (1.0 / 9007199254740993.0);
      const double u2 = (r2 >> 11) * (1.0 / 9007199254740992.0);
      rf += S.noise * sqrt(-2.0 * log(u1)) * cos(2 * 3.141592653589793 * u2);
    }
    // quantise (ldgpu/synth.py SynthRF.quantise)
    if (S.fmt == 0) {
      double q = rint(128 + 100 * rf / 1.3);
      out[n] = (uint8_t)fmin(fmax(q, 0.0), 255.0);
    } else if (S.fmt == 1) {
      double q = rint(rf * 20000);
      reinterpret_cast<int16_t*>(out)[n] = (int16_t)fmin(fmax(q, -32768.0), 32767.0);
    } else {
      // 10-bit: staged as uint16 here, packed by ldg_k_synth_pack10
      double q = rint(512 + 400 * rf / 1.3);
      reinterpret_cast<uint16_t*>(out)[n] = (uint16_t)fmin(fmax(q, 0.0), 1023.0);
    }
  }
}

// Pack staged 10-bit samples: fmt 2 = .r30 (3 per LE uint32), 3 = .lds (4 per 5 bytes).
extern "C" __global__ void ldg_k_synth_pack10(const uint16_t* __restrict__ s, int64_t ngroups, int fmt,
                                              uint8_t* __restrict__ out, int64_t g0) {
  const int64_t g = g0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ngroups) return;
  if (fmt == 2) {
    const uint32_t w = (s[3 * g] & 0x3ffu) | ((uint32_t)(s[3 * g + 1] & 0x3ffu) << 10) |
                       ((uint32_t)(s[3 * g + 2] & 0x3ffu) << 20);
    reinterpret_cast<uint32_t*>(out)[g] = w;
  } else {
    const uint16_t a = s[4 * g], b = s[4 * g + 1], c = s[4 * g + 2], d = s[4 * g + 3];
    uint8_t* o = out + 5 * g;
    o[0] = (uint8_t)(a >> 2);
    o[1] = (uint8_t)(((a & 0x3) << 6) | (b >> 4));
    o[2] = (uint8_t)(((b & 0xf) << 4) | (c >> 6));
    o[3] = (uint8_t)(((c & 0x3f) << 2) | (d >> 8));
    o[4] = (uint8_t)(d & 0xff);
  }
}
