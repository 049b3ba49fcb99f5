// 2D NTSC comb filter: .tbc frames (910 x 525 uint16, 4fsc) -> rgb48 744 x 480.
//
// Restates comb-ntsc.cxx's default path (dim = 2, HQ colour LPF, nr_y = 1 IRE,
// nr_c = 0, no pulldown): Comb::Process :834-892 -> Split1D :246-288, Split2D
// :294-367, SplitIQ :414-483, AdjustY :735-763, FilterIQ :212-243, DoYNR
// :523-553, ToRGB :555-598 (RGB::conv :124-147), PostProcess :894-938.
//
// Every output row depends only on its own line and the lines two above and
// below it (the 2D stencil).  That holds with one exception: the burst-level
// EMA `aburstlev` is a recurrence over all lines of all frames in order, so a
// one-wave kernel runs that chain first.  DoYNR's FIR history crosses lines
// and frames in the reference, but for output pixels (x >= 78) all 25 taps
// fall inside the same line (h - 12 >= 66 >= 40), so the history never
// reaches an output pixel.  One workgroup per (frame, output row) runs
// SplitIQ -> AdjustY -> FilterIQ (two sequential 1-pole chains, as in the
// reference) -> Y-NR -> YIQ->RGB with the row in LDS.
#include <hip/hip_runtime.h>
#include "common.hpp"

namespace ldg {
namespace comb {

constexpr int IN_X = 910, IN_Y = 525;
constexpr int OUT_W = 744, OUT_H = 480, OUT_X0 = 78, FIRST_LINE = 38;
constexpr int CHAIN_LINES = IN_Y - FIRST_LINE;            // 487 lines feed aburstlev per frame
constexpr double IRESCALE = 358.4, IREBASE = 1024.0;
constexpr double BLACK_IRE = 7.5, BRIGHTNESS = 236.0;
constexpr double NR_Y = 1.0 * IRESCALE;
constexpr double P_2DRANGE = 45 * IRESCALE;
constexpr double LPI_B0 = 2.267438981796600e-01, LPI_B1 = 2.267438981796600e-01;
constexpr double LPI_A1 = -5.465122036406802e-01;

struct NRTaps { double b[25]; };
__constant__ NRTaps g_nr = {{
    1.141291975113614e-04, -1.857019211291029e-03, -4.499636864042073e-03, -5.577680979937061e-03,
    -4.423694440267179e-04, 1.309163063177155e-02,  2.861211356202848e-02,  3.029931283148555e-02,
    1.098965697652802e-03,  -6.398130386469833e-02, -1.492080690537196e-01, -2.223459379380252e-01,
    7.479077367478024e-01,  -2.223459379380252e-01, -1.492080690537196e-01, -6.398130386469833e-02,
    1.098965697652803e-03,  3.029931283148557e-02,  2.861211356202848e-02,  1.309163063177156e-02,
    -4.423694440267185e-04, -5.577680979937061e-03, -4.499636864042074e-03, -1.857019211291030e-03,
    1.141291975113614e-04}};

__device__ __forceinline__ double clampd(double v, double lo, double hi) { return v < lo ? lo : (v > hi ? hi : v); }

// Split1D's tc1 of row r (0 outside lines 44..524 / pixels 4..839): integer average.
__device__ __forceinline__ double clp0(const uint16_t* __restrict__ fr, int r, int h) {
  if (r < 44 || r >= IN_Y || h < 4 || h >= 840) return 0.0;
  const uint16_t* line = fr + r * IN_X;
  const int avg = ((int)line[h + 2] + (int)line[h - 2]) / 2;
  return (double)(avg - (int)line[h]);
}

// clp1 with the three clp0 rows staged in LDS (p = l-2, c = l, n = l+2).
__device__ __forceinline__ double clp1_lds(const double* p1, const double* c1, const double* n1, int h) {
  const double c0 = c1[h], cm = c1[h - 1];
  const double p0 = p1[h], pm = p1[h - 1];
  const double n0 = n1[h], nm = n1[h - 1];
  double kp = fabs(fabs(c0) - fabs(p0));
  kp += fabs(fabs(cm) - fabs(pm));
  kp -= (fabs(c0) + fabs(cm)) * .10;
  double kn = fabs(fabs(c0) - fabs(n0));
  kn += fabs(fabs(cm) - fabs(nm));
  kn -= (fabs(c0) + fabs(nm)) * .10;
  kp /= 2;
  kn /= 2;
  kp = clampd(1 - (kp / P_2DRANGE), 0, 1);
  kn = clampd(1 - (kn / P_2DRANGE), 0, 1);
  double sc = 1.0;
  if (kn != 0 || kp != 0) {
    if (kn > (3 * kp)) kp = 0;
    else if (kp > (3 * kn)) kn = 0;
    sc = (2.0 / (kn + kp));
    if (sc < 1.0) sc = 1.0;
  } else if ((fabs(fabs(p0) - fabs(n0)) - fabs((n0 + p0) * .2)) <= 0) {
    kn = kp = 1;
  }
  double tc1 = ((c0 - p0) * kp * sc);
  tc1 += ((c0 - n0) * kn * sc);
  tc1 /= (2 * 2);
  return tc1;
}

// u16_to_ire of a double passed as uint16_t (truncation to int32, low 16 bits)
__device__ __forceinline__ double u16_to_ire_of(double v) {
  const uint16_t level = (uint16_t)(int32_t)v;
  if (level == 0) return -100;
  return -40 + ((double)level - IREBASE) / IRESCALE;
}

// FilterIQ's 1-pole colorlpi chain over one of I (even h) / Q (odd h): every h
// writes the latest output two pixels back, so the feed at h fills h-2 and
// h-1.  Inputs are prefetched 16 at a time so only the recurrence is serial.
template <bool Q>
__device__ __forceinline__ void iq_chain(const double* __restrict__ src, double* __restrict__ dst) {
  double x0 = 0, x1 = 0, y1 = 0;
  if (Q) dst[2] = 0.0;                     // h = 4 writes the not-yet-fed Q output
  constexpr int H0 = Q ? 5 : 4;
  for (int hb = H0; hb < 840; hb += 32) {
    double xs[16];
#pragma unroll
    for (int k = 0; k < 16; k++) { const int h = hb + 2 * k; xs[k] = (h < 840) ? src[h] : 0.0; }
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const int h = hb + 2 * k;
      if (h < 840) {
        x1 = x0;
        x0 = xs[k];
        double y0 = 0;
        y0 += (LPI_B0 / 1.0) * x0;
        y0 += (LPI_B1 / 1.0) * x1;
        y0 -= (LPI_A1 / 1.0) * y1;
        y1 = y0;
        dst[h - 2] = y0;
        if (h + 1 < 840) dst[h - 1] = y0;
      }
    }
  }
}

}  // namespace comb
}  // namespace ldg

using namespace ldg::comb;

// aburstlev chain (ToRGB :560-566) over lines 38..524 of n frames in order.
// state[0]: aburstlev carried across calls (-1 = not initialised).
// abl[f * CHAIN_LINES + (l - 38)]: the value ToRGB uses for line l of frame f.
// The recurrence is exact and sequential: 256 threads stage the burst levels
// of a chunk in LDS, thread 0 runs the chain over them (the loads are off the
// dependency path, so it runs at the FP64 mul+add latency), all threads write
// the results back.  grid: 1 workgroup of 256 threads.
constexpr int BURST_CHUNK = 4096;
extern "C" __global__ __launch_bounds__(256) void ldg_k_comb_burst(const uint16_t* __restrict__ frames, int n,
                                                                   double* __restrict__ state,
                                                                   double* __restrict__ abl) {
  __shared__ double s_b[BURST_CHUNK];
  __shared__ double s_a[BURST_CHUNK];
  const int tid = threadIdx.x;
  double a = state[0];
  const int total = n * CHAIN_LINES;
  for (int c0 = 0; c0 < total; c0 += BURST_CHUNK) {
    const int cnt = (total - c0) < BURST_CHUNK ? (total - c0) : BURST_CHUNK;
    for (int k = tid; k < cnt; k += 256) {
      const int j = c0 + k;
      const int f = j / CHAIN_LINES, l = FIRST_LINE + j % CHAIN_LINES;
      s_b[k] = frames[(size_t)f * IN_X * IN_Y + (size_t)l * IN_X + 1] / IRESCALE;
    }
    __syncthreads();
    if (tid == 0) {
      int k = 0;
      for (; k < cnt && a < 0; k++) {       // until the first qualifying line sets it
        const double bk = s_b[k];
        if (bk > 3) {
          a = bk;
          a = (a * .99) + (bk * .01);
        }
        s_a[k] = a;
      }
      // a > 0 from here on (burst levels > 3): only the EMA is on the serial path
#pragma unroll 8
      for (; k < cnt; k++) {
        const double bk = s_b[k];
        const double e = (a * .99) + (bk * .01);
        a = (bk > 3) ? e : a;
        s_a[k] = a;
      }
    }
    __syncthreads();
    for (int k = tid; k < cnt; k += 256) abl[c0 + k] = s_a[k];
    __syncthreads();
  }
  if (tid == 0) state[0] = a;
}

// One output row: grid n * 480 workgroups of 256 threads; row r = line r + 38.
extern "C" __global__ __launch_bounds__(256) void ldg_k_comb_rows(const uint16_t* __restrict__ frames,
                                                                  const double* __restrict__ abl,
                                                                  uint16_t* __restrict__ rgb) {
  __shared__ double s_c[3][IN_X];                        // Split1D clp0 of rows l-2, l, l+2
  __shared__ double s_y[IN_X], s_i[IN_X], s_q[IN_X];    // cbuf after SplitIQ / AdjustY
  __shared__ double s_cv[IN_X];                          // signed chroma per pixel (before the hold)
  double* const s_fi = s_c[0];                           // FilterIQ output (clp0 rows are dead by then)
  double* const s_fq = s_c[1];
  const int tid = threadIdx.x;
  const int f = blockIdx.x / OUT_H;
  const int row = blockIdx.x % OUT_H;
  const int l = row + FIRST_LINE;
  const uint16_t* fr = frames + (size_t)f * IN_X * IN_Y;
  const uint16_t* line = fr + (size_t)l * IN_X;
  const bool invertphase = (line[0] == 16384);

  for (int h = tid; h < IN_X; h += 256) {
#pragma unroll
    for (int k = 0; k < 3; k++) s_c[k][h] = clp0(fr, l - 2 + 2 * k, h);
  }
  __syncthreads();
  // ---- SplitIQ: chroma samples (Split2D / Split1D weights), then the held I / Q
  for (int h = tid; h < IN_X; h += 256) {
    double cv = 0.0;
    if (h >= 4 && h < 840) {
      double cavg = 0;
      cavg += 0.0 * 0.0;                                 // clpbuffer[2] * combk[2]
      if (l < 524 && h >= 18) {
        cavg += clp1_lds(s_c[0], s_c[1], s_c[2], h) * 1.0;
        cavg += s_c[1][h] * 0.0;
      } else {
        cavg += 0.0 * 0.0;
        cavg += s_c[1][h] * 1.0;
      }
      cavg /= 2;
      if (!invertphase) cavg = -cavg;
      cv = cavg;
    }
    s_cv[h] = cv;
  }
  __syncthreads();
  for (int h = tid; h < IN_X; h += 256) {
    double y = 0, si = 0, sq = 0;
    if (h >= 4 && h < 840) {
      y = line[h];
      const int he = h & ~1;                 // latest even h' <= h (phase 0 / 2)
      si = ((he & 3) == 0) ? s_cv[he] : -s_cv[he];
      const int ho = (h & 1) ? h : h - 1;    // latest odd h' <= h (phase 1 / 3), none before 5
      if (ho >= 5) sq = ((ho & 3) == 1) ? -s_cv[ho] : s_cv[ho];
    }
    s_y[h] = y; s_i[h] = si; s_q[h] = sq;
  }
  __syncthreads();
  // ---- AdjustY: p[h] = p[h + 2] with y += +-I / +-Q (h in [2, 842))
  double ay[4], ai[4], aq[4];
#pragma unroll
  for (int e = 0; e < 4; e++) {
    const int h = tid + 256 * e;
    if (h >= IN_X) continue;
    if (h >= 2 && h < 842) {
      const double yy = s_y[h + 2], ii = s_i[h + 2], qq = s_q[h + 2];
      double comp = 0;
      switch (h & 3) {
        case 0: comp = ii; break;
        case 1: comp = -qq; break;
        case 2: comp = -ii; break;
        default: comp = qq; break;
      }
      if (invertphase) comp = -comp;
      ay[e] = yy + comp; ai[e] = ii; aq[e] = qq;
    } else {
      ay[e] = s_y[h]; ai[e] = s_i[h]; aq[e] = s_q[h];
    }
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < 4; e++) {
    const int h = tid + 256 * e;
    if (h < IN_X) { s_y[h] = ay[e]; s_i[h] = ai[e]; s_q[h] = aq[e]; s_fi[h] = ai[e]; s_fq[h] = aq[e]; }
  }
  __syncthreads();
  // ---- FilterIQ (lines >= 44): a fresh colorlpi IIR for I (fed at even h) and
  //      for Q (odd h); every h writes the latest output two pixels back, so
  //      each feed at h fills positions h-2 and h-1.  Thread 0: I, thread 64: Q.
  if (l >= 44) {
    if (tid == 0) iq_chain<false>(s_i, s_fi);
    if (tid == 64) iq_chain<true>(s_q, s_fq);
  }
  __syncthreads();
  // ---- DoYNR (taps inside this line for x >= 78) + ToRGB
  const double aburst = abl[(size_t)f * CHAIN_LINES + (l - FIRST_LINE)];
  const double m = BRIGHTNESS * 256 / 100;
  uint16_t* out = rgb + ((size_t)f * OUT_H + row) * OUT_W * 3;
  for (int x = tid; x < OUT_W; x += 256) {
    const int h = x + OUT_X0;
    double y0 = 0;
#pragma unroll
    for (int o = 0; o < 25; o++) y0 += (g_nr.b[o] / 1.0) * s_y[h + 12 - o];
    double a = y0;
    if (fabs(a) > NR_Y) a = (a > 0) ? NR_Y : -NR_Y;
    const double yv = s_y[h] - a;
    double iv = s_fi[h], qv = s_fq[h];
    iv *= (10 / aburst);
    qv *= (10 / aburst);
    double y = u16_to_ire_of(yv);
    y = (y - BLACK_IRE) * (100 / (100 - BLACK_IRE));
    const double q = +(iv) / IRESCALE;
    const double i = +(qv) / IRESCALE;
    double r = y + (.956 * i) + (.621 * q);
    double g = y - (.272 * i) - (.647 * q);
    double b = y - (1.106 * i) + (1.703 * q);
    r = clampd(r * m, 0, 65535);
    g = clampd(g * m, 0, 65535);
    b = clampd(b * m, 0, 65535);
    out[x * 3 + 0] = (uint16_t)r;
    out[x * 3 + 1] = (uint16_t)g;
    out[x * 3 + 2] = (uint16_t)b;
  }
}
