// Dense optical flow for the NTSC comb's 3D mode with flow (comb-ntsc -d 3
// without -F; comb-ntsc.cxx:600-662 OpticalFlow3D, Process :851-858): the
// Farneback flow between the luma fields of consecutive frames, and the 3D
// weight combk[2] the comb derives from its magnitude.
//
// BUILD-DEFINED, PARITY UNPINNED.  The reference calls OpenCV's
// calcOpticalFlowFarneback(new field, previous field, flow, 0.5, 4, 60, 3, 7,
// 1.5, OPTFLOW_USE_INITIAL_FLOW from its third call); OpenCV is absent here.
// These kernels follow oracle/farneback.py, a restatement of that function's
// CPU path (optflowgf.cpp: the pyramid loop, FarnebackPolyExp,
// FarnebackUpdateMatrices, FarnebackUpdateFlow_Blur; GaussianBlur with
// BORDER_REFLECT_101, resize INTER_LINEAR / INTER_AREA), step for step, in
// FP64 (OpenCV: float32 images, double accumulators).
//
// Layout: two fields side by side, field-major: an image is [2][h][w] doubles
// (5 or 2 channels interleaved per pixel where noted).  Level 0 is 252 x 840
// (rows 23 + field + 2 y, columns 70..909 of the comb's luma), levels 1 and 2
// are 126 x 420 and 63 x 210 (OpenCV stops at the 32-pixel minimum: two
// pyramid levels below the image, not four).  Everything is elementwise or a
// short stencil except the 61-tap box sums of UpdateFlow_Blur, which run as
// sequential running sums (one lane per column, then one per row), as OpenCV
// computes them.
#include <hip/hip_runtime.h>
#include "common.hpp"

namespace ldg {
namespace flow {

constexpr int NLEV = 3;                               // (FR, FC, FY0, FX0: common.hpp)
constexpr int POLY_N = 7;
constexpr int WIN = 60, WM = WIN / 2;                   // winsize 60: running sums over [-30, 30]
constexpr int ITERS = 3;
constexpr int BORDER = 5;

struct PolyK {
  double g[2 * POLY_N + 1], xg[2 * POLY_N + 1], xxg[2 * POLY_N + 1];   // indices -n..n at [k + n]
  double ig11, ig03, ig33, ig55;
};
struct BlurK {
  double k[9];
  int ks;
};

__device__ __forceinline__ int reflect101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = (i < 0) ? -i : 2 * n - 2 - i;
  return i;
}
__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

}  // namespace flow
}  // namespace ldg

using namespace ldg::flow;

// ---- the comb luma the flow sees: OpticalFlow3D's fieldbuf (comb-ntsc.cxx:617-624)
// from the NEW frame's tbuf after AdjustY and DoYNR (DoCNR only moves I / Q).  Rows
// below 36 are 0 (SplitIQ leaves them), rows 36 .. firstline-1 the raw samples at
// h 4..839 (SplitIQ's Y; AdjustY starts at firstline), rows from firstline AdjustY's
// Y minus DoYNR's clipped high pass (its taps stay inside the row for h >= 70).
// Rows past 524 (the reference reads past its buffer there) are 0.  The value goes
// to uint16_t as C converts a double: toward zero, the low 16 bits.
// cv: the frame's 2D signed chroma rows (comb_split), row l at (l - firstline).
// grid: 2 * FR workgroups of 256 threads.
extern "C" __global__ __launch_bounds__(256) void ldg_k_flow_luma(const uint16_t* __restrict__ fr,
                                                                  const double* __restrict__ cvbuf, int firstline,
                                                                  double nr_y, uint16_t* __restrict__ ybuf) {
  using namespace ldg::comb;
  __shared__ double s_y[IN_X + 4];
  const int tid = threadIdx.x;
  const int f = blockIdx.x / FR, r = blockIdx.x % FR;
  const int L = FY0 + f + 2 * r;
  uint16_t* out = ybuf + ((size_t)f * FR + r) * FC;
  if (L >= IN_Y) {
    for (int x = tid; x < FC; x += 256) out[x] = 0;
    return;
  }
  const uint16_t* line = fr + (size_t)L * IN_X;
  const double* cv = cvbuf + (size_t)(L - firstline) * CV_STRIDE;
  const bool inv = line[0] == 16384;
  for (int h = tid; h < IN_X + 4; h += 256) {
    double v = 0.0;
    if (h < IN_X) {
      if (L >= 36 && L < firstline) {
        v = (h >= 4 && h < 840) ? (double)line[h] : 0.0;
      } else if (L >= firstline && h >= 2 && h < 842) {
        const int p = h + 2;
        const double yy = (L >= 36 && p >= 4 && p < 840) ? (double)line[p] : 0.0;
        const double ii = held_i(cv, p), qq = held_q(cv, p);
        double comp = 0;
        switch (h & 3) {
          case 0: comp = ii; break;
          case 1: comp = -qq; break;
          case 2: comp = -ii; break;
          default: comp = qq; break;
        }
        if (inv) comp = -comp;
        v = yy + comp;
      }
    }
    s_y[h] = v;
  }
  __syncthreads();
  for (int x = tid; x < FC; x += 256) {
    const int h = x + FX0;
    double y = s_y[h];
    if (L >= firstline && nr_y > 0 && h >= 40 && h + 12 <= 843) {
      double y0 = 0;
#pragma unroll
      for (int o = 0; o < 25; o++) y0 += (g_nr.b[o] / 1.0) * s_y[h + 12 - o];
      double a = y0;
      if (fabs(a) > nr_y) a = (a > 0) ? nr_y : -nr_y;
      y = s_y[h] - a;
    }
    out[x] = (uint16_t)(int32_t)y;
  }
}

// ---- GaussianBlur (BORDER_REFLECT_101), rows then columns, full resolution.
// src16: the uint16 fields (or null: src64).  grid: 2 * FR workgroups of 256.
extern "C" __global__ __launch_bounds__(256) void ldg_k_flow_blur_rows(const uint16_t* __restrict__ src16,
                                                                       double* __restrict__ dst, BlurK K) {
  const int b = blockIdx.x;                 // field * FR + row
  const int R = K.ks / 2;
  const uint16_t* s = src16 + (size_t)b * FC;
  for (int x = threadIdx.x; x < FC; x += 256) {
    double acc = 0.0;
    for (int j = 0; j < K.ks; j++) acc += K.k[j] * (double)s[reflect101(x + j - R, FC)];
    dst[(size_t)b * FC + x] = acc;
  }
}
extern "C" __global__ __launch_bounds__(256) void ldg_k_flow_blur_cols(const double* __restrict__ src,
                                                                       double* __restrict__ dst, BlurK K) {
  const int b = blockIdx.x;
  const int f = b / FR, y = b % FR;
  const int R = K.ks / 2;
  const double* s = src + (size_t)f * FR * FC;
  for (int x = threadIdx.x; x < FC; x += 256) {
    double acc = 0.0;
    for (int j = 0; j < K.ks; j++) acc += K.k[j] * s[(size_t)reflect101(y + j - R, FR) * FC + x];
    dst[(size_t)b * FC + x] = acc;
  }
}

// ---- resize(INTER_LINEAR) from FR x FC to h x w (per channel-less image).
// grid: (2 * h) workgroups of 256.
__device__ __forceinline__ void lin_axis(int d, int nd, int ns, int& i0, int& i1, double& a) {
  const double ratio = (double)ns / (double)nd;
  const double fpos = ((double)d + 0.5) * ratio - 0.5;
  int j = (int)floor(fpos);
  double t = fpos - (double)j;
  if (j < 0) { t = 0.0; j = 0; }
  i1 = j + 1 < ns ? j + 1 : ns - 1;
  if (j >= ns - 1) { t = 0.0; j = ns - 1; }
  i0 = j;
  a = t;
}
extern "C" __global__ __launch_bounds__(256) void ldg_k_flow_resize(const double* __restrict__ src, int sh, int sw,
                                                                    double* __restrict__ dst, int h, int w, int ch,
                                                                    double mul) {
  const int b = blockIdx.x;
  const int f = b / h, y = b % h;
  int y0, y1;
  double ay;
  lin_axis(y, h, sh, y0, y1, ay);
  const double* s = src + (size_t)f * sh * sw * ch;
  for (int i = threadIdx.x; i < w * ch; i += 256) {
    const int x = i / ch, c = i % ch;
    int x0, x1;
    double ax;
    lin_axis(x, w, sw, x0, x1, ax);
    const double top = s[((size_t)y0 * sw + x0) * ch + c] * (1 - ax) + s[((size_t)y0 * sw + x1) * ch + c] * ax;
    const double bot = s[((size_t)y1 * sw + x0) * ch + c] * (1 - ax) + s[((size_t)y1 * sw + x1) * ch + c] * ax;
    dst[(((size_t)f * h + y) * w) * ch + i] = (top * (1 - ay) + bot * ay) * mul;
  }
}

// ---- resize(INTER_AREA) by an integer factor (the block mean), times mul (2 channels).
extern "C" __global__ __launch_bounds__(256) void ldg_k_flow_area(const double* __restrict__ src, int sh, int sw,
                                                                  double* __restrict__ dst, int h, int w, double mul) {
  const int b = blockIdx.x;
  const int f = b / h, y = b % h;
  const int fy = sh / h, fx = sw / w;
  const double* s = src + (size_t)f * sh * sw * 2;
  for (int i = threadIdx.x; i < w * 2; i += 256) {
    const int x = i / 2, c = i % 2;
    double acc = 0.0;
    for (int yy = 0; yy < fy; yy++)
      for (int xx = 0; xx < fx; xx++) acc += s[((size_t)(y * fy + yy) * sw + (x * fx + xx)) * 2 + c];
    dst[(((size_t)f * h + y) * w) * 2 + i] = acc / (double)(fy * fx) * mul;
  }
}

// ---- FarnebackPolyExp: vertical part (3 sums per pixel), then horizontal (the 5
// coefficients [r_y, r_x, r_yy, r_xx, r_xy]); replicate borders.  grid: 2 * h x 256.
extern "C" __global__ __launch_bounds__(256) void ldg_k_flow_poly_v(const double* __restrict__ I, int h, int w,
                                                                    double* __restrict__ rows3, PolyK P) {
  const int b = blockIdx.x;
  const int f = b / h, y = b % h;
  const double* src = I + (size_t)f * h * w;
  constexpr int n = POLY_N;
  for (int x = threadIdx.x; x < w; x += 256) {
    double r0 = src[(size_t)y * w + x] * P.g[n], r1 = 0.0, r2 = 0.0;
    for (int k = 1; k <= n; k++) {
      const double up = src[(size_t)(y - k < 0 ? 0 : y - k) * w + x];
      const double dn = src[(size_t)(y + k > h - 1 ? h - 1 : y + k) * w + x];
      const double p = up + dn;
      r0 = r0 + P.g[n + k] * p;
      r1 = r1 + P.xg[n + k] * (dn - up);
      r2 = r2 + P.xxg[n + k] * p;
    }
    double* o = rows3 + (((size_t)f * h + y) * w + x) * 3;
    o[0] = r0;
    o[1] = r1;
    o[2] = r2;
  }
}
extern "C" __global__ __launch_bounds__(256) void ldg_k_flow_poly_h(const double* __restrict__ rows3, int h, int w,
                                                                    double* __restrict__ R, PolyK P) {
  const int b = blockIdx.x;
  const int f = b / h, y = b % h;
  const double* row = rows3 + ((size_t)f * h + y) * w * 3;
  constexpr int n = POLY_N;
  for (int x = threadIdx.x; x < w; x += 256) {
    const double* c0 = row + (size_t)x * 3;
    double b1 = c0[0] * P.g[n], b2 = 0.0, b3 = c0[1] * P.g[n], b4 = 0.0, b5 = c0[2] * P.g[n], b6 = 0.0;
    for (int k = 1; k <= n; k++) {
      const double* pr = row + (size_t)(x + k > w - 1 ? w - 1 : x + k) * 3;
      const double* mr = row + (size_t)(x - k < 0 ? 0 : x - k) * 3;
      const double g0 = P.g[n + k];
      const double tg = pr[0] + mr[0];
      b1 = b1 + tg * g0;
      b4 = b4 + tg * P.xxg[n + k];
      b2 = b2 + (pr[0] - mr[0]) * P.xg[n + k];
      b3 = b3 + (pr[1] + mr[1]) * g0;
      b6 = b6 + (pr[1] - mr[1]) * P.xg[n + k];
      b5 = b5 + (pr[2] + mr[2]) * g0;
    }
    double* o = R + (((size_t)f * h + y) * w + x) * 5;
    o[1] = b2 * P.ig11;
    o[0] = b3 * P.ig11;
    o[3] = b1 * P.ig03 + b4 * P.ig33;
    o[2] = b1 * P.ig03 + b5 * P.ig33;
    o[4] = b6 * P.ig55;
  }
}

// ---- FarnebackUpdateMatrices: (G11, G12, G22, h1, h2) per pixel.  grid: 2 * h x 256.
__device__ __forceinline__ double flow_border(int i) {
  constexpr double B[BORDER] = {0.14, 0.14, 0.4472, 0.4472, 0.4472};
  return B[i];
}
extern "C" __global__ __launch_bounds__(256) void ldg_k_flow_update(const double* __restrict__ R0,
                                                                    const double* __restrict__ R1,
                                                                    const double* __restrict__ flow, int h, int w,
                                                                    double* __restrict__ M) {
  const int b = blockIdx.x;
  const int f = b / h, y = b % h;
  const size_t base = (size_t)f * h * w;
  for (int x = threadIdx.x; x < w; x += 256) {
    const size_t p = base + (size_t)y * w + x;
    const double dx = flow[p * 2], dy = flow[p * 2 + 1];
    const double fx = (double)x + dx, fy = (double)y + dy;
    const double flx = floor(fx), fly = floor(fy);
    const double ax = fx - flx, ay = fy - fly;
    const double* r0 = R0 + p * 5;
    double r2, r3, r4, r5, r6;
    const bool inside = flx >= 0 && flx < (double)(w - 1) && fly >= 0 && fly < (double)(h - 1);
    if (inside) {
      const int x1 = (int)flx, y1 = (int)fly;
      const double a00 = (1 - ax) * (1 - ay), a01 = ax * (1 - ay), a10 = (1 - ax) * ay, a11 = ax * ay;
      const double* q00 = R1 + (base + (size_t)y1 * w + x1) * 5;
      const double* q01 = q00 + 5;
      const double* q10 = q00 + (size_t)w * 5;
      const double* q11 = q10 + 5;
      double s[5];
#pragma unroll
      for (int c = 0; c < 5; c++) s[c] = a00 * q00[c] + a01 * q01[c] + a10 * q10[c] + a11 * q11[c];
      r2 = s[0];
      r3 = s[1];
      r4 = (r0[2] + s[2]) * 0.5;
      r5 = (r0[3] + s[3]) * 0.5;
      r6 = (r0[4] + s[4]) * 0.25;
    } else {
      r2 = r3 = 0.0;
      r4 = r0[2];
      r5 = r0[3];
      r6 = r0[4] * 0.5;
    }
    r2 = (r0[0] - r2) * 0.5;
    r3 = (r0[1] - r3) * 0.5;
    r2 = r2 + r4 * dy + r6 * dx;
    r3 = r3 + r6 * dy + r5 * dx;
    double sc = 1.0;
    if (x < BORDER) sc *= flow_border(x);
    if (x >= w - BORDER) sc *= flow_border(w - 1 - x);
    if (y < BORDER) sc *= flow_border(y);
    if (y >= h - BORDER) sc *= flow_border(h - 1 - y);
    if (sc != 1.0) {
      r2 *= sc; r3 *= sc; r4 *= sc; r5 *= sc; r6 *= sc;
    }
    double* m = M + p * 5;
    m[0] = r4 * r4 + r6 * r6;
    m[1] = (r4 + r5) * r6;
    m[2] = r5 * r5 + r6 * r6;
    m[3] = r4 * r2 + r6 * r3;
    m[4] = r6 * r2 + r5 * r3;
  }
}

// ---- FarnebackUpdateFlow_Blur: the vertical running sums over rows [y - 30, y + 30]
// (replicated) per column and channel, then per row the horizontal ones and the 2 x 2
// solve.  grid vsum: ceil(2 * w * 5 / 256); hsum: ceil(2 * h / 64) x 64.
extern "C" __global__ __launch_bounds__(256) void ldg_k_flow_vsum(const double* __restrict__ M, int h, int w,
                                                                  double* __restrict__ V) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= 2 * w * 5) return;
  const int f = i / (w * 5), xc = i % (w * 5);
  const double* s = M + (size_t)f * h * w * 5 + xc;
  double* d = V + (size_t)f * h * w * 5 + xc;
  const size_t st = (size_t)w * 5;
  double v = s[0] * (WM + 2);
  for (int y = 1; y < WM; y++) v += s[(size_t)clampi(y, 0, h - 1) * st];
  for (int y = 0; y < h; y++) {
    v += s[(size_t)clampi(y + WM, 0, h - 1) * st] - s[(size_t)clampi(y - WM - 1, 0, h - 1) * st];
    d[(size_t)y * st] = v;
  }
}
extern "C" __global__ __launch_bounds__(64) void ldg_k_flow_hsum_solve(const double* __restrict__ V, int h, int w,
                                                                       double* __restrict__ flow) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= 2 * h) return;
  const int f = i / h, y = i % h;
  const double* row = V + ((size_t)f * h + y) * w * 5;
  double* fl = flow + ((size_t)f * h + y) * w * 2;
  double s[5];
#pragma unroll
  for (int c = 0; c < 5; c++) {
    s[c] = row[c] * (WM + 2);
    for (int x = 1; x < WM; x++) s[c] += row[(size_t)clampi(x, 0, w - 1) * 5 + c];
  }
  const double scale = 1.0 / ((double)WIN * WIN);
  for (int x = 0; x < w; x++) {
    const double* a = row + (size_t)clampi(x + WM, 0, w - 1) * 5;
    const double* b = row + (size_t)clampi(x - WM - 1, 0, w - 1) * 5;
#pragma unroll
    for (int c = 0; c < 5; c++) s[c] += a[c] - b[c];
    const double g11 = s[0] * scale, g12 = s[1] * scale, g22 = s[2] * scale, h1 = s[3] * scale, h2 = s[4] * scale;
    const double idet = 1.0 / (g11 * g22 - g12 * g12 + 1e-3);
    fl[(size_t)x * 2] = (g11 * h2 - g12 * h1) * idet;
    fl[(size_t)x * 2 + 1] = (g22 * h1 - g12 * h2) * idet;
  }
}

// ---- OpticalFlow3D's 3D weight (comb-ntsc.cxx:633-650) for the frame the flow
// belongs to: c = 1 - clamp((|(fy, 2 fx)| - core) / range, 0, 1), the smaller of the
// two fields', per field pixel (applied to frame rows 2 y and 2 y + 1, columns 70..909).
// grid: FR workgroups of 256.
extern "C" __global__ __launch_bounds__(256) void ldg_k_flow_combk(const double* __restrict__ flow, double core,
                                                                   double range, double* __restrict__ cmap) {
  const int y = blockIdx.x;
  for (int x = threadIdx.x; x < FC; x += 256) {
    double c2[2];
#pragma unroll
    for (int f = 0; f < 2; f++) {
      const double* p = flow + (((size_t)f * FR + y) * FC + x) * 2;
      const double fx2 = p[0] * 2;
      const double r = sqrt((p[1] * p[1]) + (fx2 * fx2));
      double t = (r - core) / range;
      t = t < 0 ? 0 : (t > 1 ? 1 : t);
      c2[f] = 1 - t;
    }
    cmap[(size_t)y * FC + x] = (c2[0] < c2[1]) ? c2[0] : c2[1];
  }
}
