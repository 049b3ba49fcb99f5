// PAL Y/C decoder for 1135 x 625 .tbc frames -> rgb48 1057 x 576 (row F2).
//
// BUILD-DEFINED: the reference has no PAL comb for this geometry; this is
// attic2/comb-pal.cxx's dim = 2 path adapted to it (the adaptation and its
// stage map are in oracle/combpal.cpp, the CPU checker of these kernels).
// Parity with the reference is unpinned; parity with that checker is +-1 LSB.
//
// Three kernels, like the NTSC comb (comb.hip):
//   ldg_k_pal_split  one workgroup per (frame, line 24..624): raw lines l-4,
//                    l, l+4 -> Split1D (+-2 px) / Split2D (+-4 lines) ->
//                    SplitIQ's signed chroma cv[h] (the held U / V source);
//   ldg_k_pal_angle  one workgroup per frame: each line's burst angle (sum of
//                    the held U / V over the burst window, after AdjustY's
//                    2-px shift on lines >= 44), the frame's V-switch phase
//                    vote, and the burst-level EMA (constant level 8 in the
//                    reference: a chain that sits at its fixed point);
//   ldg_k_pal_out    one workgroup per (frame, output row): AdjustY, Y-NR
//                    (taps within the line for x >= 78), rotation of U / V
//                    to a 135-degree burst (one sincos per row), the V-switch flip, YUV -> RGB.
#include <hip/hip_runtime.h>
#include "common.hpp"

namespace ldg {
namespace pal {

constexpr int IN_X = 1135, IN_Y = 625;
constexpr int FIRST_LINE = 44, OUT_H = 576, OUT_X0 = 78, OUT_W = IN_X - 78;
constexpr int SPLIT_L0 = 24, CV_ROWS = IN_Y - SPLIT_L0;   // lines 24..624
constexpr int CV_STRIDE = 1136;
constexpr int ABL_LINES = (IN_Y - 2) - FIRST_LINE;        // EMA updates per frame (lines 44..622)
constexpr int BURST_H0 = 100, BURST_H1 = 132;
constexpr double IRESCALE = 376.32, IREBASE = 0.0;
constexpr double BLACK_IRE = 0.0, BRIGHTNESS = 240.0;
constexpr double NR_Y = 1.0 * IRESCALE;

// SplitIQ's held U (i) / V (q) at pixel p (0 outside [4, IN_X - 4)) from cv
__device__ __forceinline__ double held_i(const double* __restrict__ cv, int p) {
  if (p < 4 || p >= IN_X - 4) return 0.0;
  const int he = p & ~1;
  return ((he & 3) == 0) ? cv[he] : -cv[he];
}
__device__ __forceinline__ double held_q(const double* __restrict__ cv, int p) {
  if (p < 4 || p >= IN_X - 4) return 0.0;
  const int ho = (p & 1) ? p : p - 1;
  if (ho < 5) return 0.0;
  return ((ho & 3) == 1) ? -cv[ho] : cv[ho];
}

}  // namespace pal
}  // namespace ldg

using namespace ldg;

// grid: n * CV_ROWS workgroups of 256 threads; cv: [n][CV_ROWS][CV_STRIDE].
extern "C" __global__ __launch_bounds__(256) void ldg_k_pal_split(const uint16_t* __restrict__ frames,
                                                                  double* __restrict__ cvbuf) {
  __shared__ uint16_t s_raw[3][pal::IN_X + 3];             // raw lines l-4, l, l+4
  __shared__ double s_c[3][pal::IN_X];                     // their Split1D clp0
  const int tid = threadIdx.x;
  const int f = blockIdx.x / pal::CV_ROWS;
  const int l = pal::SPLIT_L0 + blockIdx.x % pal::CV_ROWS;
  const uint16_t* fr = frames + (size_t)f * pal::IN_X * pal::IN_Y;
  for (int t = tid; t < 3 * pal::IN_X; t += 256) {
    const int k = t / pal::IN_X, h = t % pal::IN_X;
    const int r = l - 4 + 4 * k;
    s_raw[k][h] = (r >= 0 && r < pal::IN_Y) ? fr[(size_t)r * pal::IN_X + h] : (uint16_t)0;
  }
  __syncthreads();
  for (int h = tid; h < pal::IN_X; h += 256) {
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const int r = l - 4 + 4 * k;
      double c = 0.0;
      if (r >= pal::SPLIT_L0 && r < pal::IN_Y && h >= 4 && h < pal::IN_X - 4) {
        const int avg = ((int)s_raw[k][h + 2] + (int)s_raw[k][h - 2]) / 2;
        c = (double)(avg - (int)s_raw[k][h]);
      }
      s_c[k][h] = c;
    }
  }
  __syncthreads();
  const bool invertphase = (s_raw[1][0] == 16384);
  double* cvrow = cvbuf + ((size_t)f * pal::CV_ROWS + (l - pal::SPLIT_L0)) * pal::CV_STRIDE;
  for (int h = tid; h < pal::CV_STRIDE; h += 256) {
    double cv = 0.0;
    if (h >= 4 && h < pal::IN_X - 4) {
      double cavg = 0;
      cavg += 0.0 * 0.0;
      if (l >= 4 && l <= pal::IN_Y - 4 && h >= 18) {
        cavg += comb::clp1_lds(s_c[0], s_c[1], s_c[2], h, 45 * pal::IRESCALE) * 1.0;
        cavg += s_c[1][h] * 0.0;
      } else {
        cavg += 0.0 * 0.0;
        cavg += s_c[1][h] * 1.0;
      }
      cavg /= 2;
      if (!invertphase) cavg = -cavg;
      cv = cavg;
    }
    cvrow[h] = cv;
  }
}

// grid: n workgroups of 256 threads, one per frame.  angle: [n][IN_Y] degrees;
// phase: [n]; abl: [n][ABL_LINES] (the EMA value line 44 + j uses).  The EMA is
// carried across calls: it enters from state_in[0] (-1 = not initialised) and
// the last frame's workgroup leaves it in state_out[0] (a different double: the
// other workgroups read state_in meanwhile).  Its input is the constant burst
// level 8, so the chain reaches a fixed point (ema(a) == a, at once from "not
// initialised": 8 * .99 + 8 * .01 == 8) and every workgroup runs it from
// state_in only until then, exactly as the sequential chain would.
extern "C" __global__ __launch_bounds__(256) void ldg_k_pal_angle(const double* __restrict__ cvbuf, int n,
                                                                  double* __restrict__ angle,
                                                                  int32_t* __restrict__ phase,
                                                                  const double* __restrict__ state_in,
                                                                  double* __restrict__ state_out,
                                                                  double* __restrict__ abl) {
  prio_latency();
  __shared__ double s_ang[pal::IN_Y];
  __shared__ int s_cnt, s_fix;
  __shared__ double s_a;
  const int tid = threadIdx.x;
  const int f = blockIdx.x;
  for (int l = tid; l < pal::IN_Y; l += 256) {
    double i = 0, q = 0;
    if (l >= pal::SPLIT_L0) {
      const double* cv = cvbuf + ((size_t)f * pal::CV_ROWS + (l - pal::SPLIT_L0)) * pal::CV_STRIDE;
      const int sh = (l >= pal::FIRST_LINE) ? 2 : 0;    // AdjustY's p[h] = p[h + 2]
      for (int h = pal::BURST_H0; h < pal::BURST_H1; h++) {
        i += pal::held_i(cv, h + sh);
        q += pal::held_q(cv, h + sh);
      }
    }
    double rv = 0.0;
    if (l >= 10) {
      rv = atan2(q, i) * (180 / 3.141592653589793);
      if (rv < 0) rv += 360;
    }
    s_ang[l] = rv;
    angle[(size_t)f * pal::IN_Y + l] = rv;
  }
  if (tid == 0) {
    s_cnt = 0;
    // burstlev = 8 (> 5) on every line: a -> (a < 0 ? 8 : a) * .99 + 8 * .01
    const double bl = 8;
    double a = state_in[0];
    const int64_t skip = (int64_t)f * pal::ABL_LINES;   // the EMA steps of the earlier frames
    for (int64_t j = 0; j < skip; j++) {
      const double an = ((a < 0) ? bl : a) * .99 + bl * .01;
      if (an == a) break;
      a = an;
    }
    double* out = abl + (size_t)f * pal::ABL_LINES;
    int j = 0;
    for (; j < pal::ABL_LINES; j++) {
      const double an = ((a < 0) ? bl : a) * .99 + bl * .01;
      if (an == a) break;
      a = an;
      out[j] = a;
    }
    s_fix = j;
    s_a = a;
    if (f == n - 1) state_out[0] = a;
  }
  __syncthreads();
  {
    double* out = abl + (size_t)f * pal::ABL_LINES;
    const double a = s_a;
    for (int j = s_fix + tid; j < pal::ABL_LINES; j += 256) out[j] = a;
  }
  int c = 0;
  for (int l = 20 + 4 * tid; l < pal::IN_Y - 4; l += 4 * 256) c += fabs(s_ang[l + 1] - s_ang[l]) < 20;
  if (c) atomicAdd(&s_cnt, c);
  __syncthreads();
  if (tid == 0) {
    const int tot = (pal::IN_Y - 4 - 20 + 3) / 4;
    phase[f] = s_cnt > (tot / 2) ? 1 : 0;
  }
}

// grid: n * OUT_H workgroups of 256 threads.
extern "C" __global__ __launch_bounds__(256) void ldg_k_pal_out(const uint16_t* __restrict__ frames,
                                                                const double* __restrict__ cvbuf,
                                                                const double* __restrict__ angle,
                                                                const int32_t* __restrict__ phase,
                                                                const double* __restrict__ abl,
                                                                uint16_t* __restrict__ rgb) {
  __shared__ uint16_t s_line[pal::IN_X + 1];
  __shared__ double s_y[pal::IN_X + 1];                    // AdjustY's Y; [IN_X]: the next line's p[0]
  const int tid = threadIdx.x;
  const int f = blockIdx.x / pal::OUT_H;
  const int row = blockIdx.x % pal::OUT_H;
  const int l = row + pal::FIRST_LINE;
  const uint16_t* line = frames + (size_t)f * pal::IN_X * pal::IN_Y + (size_t)l * pal::IN_X;
  for (int h = tid; h < pal::IN_X; h += 256) s_line[h] = line[h];
  __syncthreads();
  const bool invertphase = (s_line[0] == 16384);
  const double* cv = cvbuf + ((size_t)f * pal::CV_ROWS + (l - pal::SPLIT_L0)) * pal::CV_STRIDE;
  // AdjustY at h in [2, IN_X): y = p[h + 2].y + comp (p past the line's end: 0)
  for (int h = tid; h <= pal::IN_X; h += 256) {
    double v = 0.0;
    if (h >= 2 && h < pal::IN_X) {
      const int p = h + 2;
      const double yy = (p >= 4 && p < pal::IN_X - 4) ? (double)s_line[p] : 0.0;
      const double ii = pal::held_i(cv, p), qq = pal::held_q(cv, p);
      double comp = 0;
      switch (h & 3) {
        case 0: comp = ii; break;
        case 1: comp = -qq; break;
        case 2: comp = -ii; break;
        default: comp = qq; break;
      }
      if (invertphase) comp = -comp;
      v = yy + comp;
    }
    s_y[h] = v;
  }
  __syncthreads();
  const double aburst = abl[(size_t)f * pal::ABL_LINES + (l - pal::FIRST_LINE)];
  const double angleadj = 135 - angle[(size_t)f * pal::IN_Y + l];
  double sa, ca;
  sincos(((angleadj + 0) / 180.0) * 3.141592653589793, &sa, &ca);
  const bool ph = phase[f] != 0;
  const double m = pal::BRIGHTNESS * 255 / 100;
  uint16_t* out = rgb + ((size_t)f * pal::OUT_H + row) * pal::OUT_W * 3;
  for (int x = tid; x < pal::OUT_W; x += 256) {
    const int h = x + pal::OUT_X0;
    double yv = s_y[h];
    if (h < pal::IN_X - 12) {
      double y0 = 0;
#pragma unroll
      for (int o = 0; o < 25; o++) y0 += (comb::g_nr.b[o] / 1.0) * s_y[h + 12 - o];
      double a = y0;
      if (fabs(a) > pal::NR_Y) a = (a > 0) ? pal::NR_Y : -pal::NR_Y;
      yv -= a;
    }
    // the reference's polar form, mag * cis(atan2(q, i) + adj), as a rotation by the
    // row's angle (the same vector; rounding within the checker's +-1 LSB)
    const double i1 = pal::held_i(cv, h + 2), q1 = pal::held_q(cv, h + 2);
    double iv = i1 * ca - q1 * sa;
    double qv = i1 * sa + q1 * ca;
    iv *= (10 / aburst);
    qv *= (10 / aburst);
    const double i0 = iv, q0 = qv;
    bool flip = ((l & 3) == 1) || ((l & 3) == 2);
    if (ph) flip = !flip;
    if (flip) {
      iv = -q0;
      qv = -i0;
    }
    const double yc = comb::clampd(yv, 0, 65535);
    const uint16_t level = (uint16_t)yc;
    double y = (level == 0) ? -100.0 : -43.122874 + ((double)(level - pal::IREBASE) / pal::IRESCALE);
    y = (y - pal::BLACK_IRE) * (100 / (100 - pal::BLACK_IRE));
    const double u = +(iv) / pal::IRESCALE;
    const double v = +(qv) / pal::IRESCALE;
    double r = y + (1.13983 * v);
    double g = y - (0.58060 * v) - (u * 0.39465);
    double b = y + (u * 2.032);
    r = comb::clampd(r * m, 0, 65535);
    g = comb::clampd(g * m, 0, 65535);
    b = comb::clampd(b * m, 0, 65535);
    out[x * 3 + 0] = (uint16_t)r;
    out[x * 3 + 1] = (uint16_t)g;
    out[x * 3 + 2] = (uint16_t)b;
  }
}
