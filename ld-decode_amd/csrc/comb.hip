// NTSC comb filter: .tbc frames (910 x 525 uint16, 4fsc) -> rgb48 744 x 480,
// 2D (the default) or 3D without optical flow (comb-ntsc -d 3 -F).
//
// Restates comb-ntsc.cxx's default path (dim = 2, HQ colour LPF, nr_y = 1 IRE,
// nr_c = 0, no pulldown): Comb::Process :834-892 -> Split1D :246-288, Split2D
// :294-367, SplitIQ :414-483, AdjustY :735-763, FilterIQ :212-243, DoYNR
// :523-553, ToRGB :555-598 (RGB::conv :124-147), PostProcess :894-938.
//
// Every output row depends only on its own line and the lines two above and
// below it (the 2D stencil), with two exceptions that are sequential
// recurrences: the burst-level EMA `aburstlev` over all lines of all frames
// (ldg_k_comb_burst: speculative chunks, exact), and FilterIQ's two 1-pole chains per line
// (418 feeds each).  DoYNR's FIR history crosses lines and frames in the
// reference, but for output pixels (x >= 78) all 25 taps fall inside the same
// line (h - 12 >= 66 >= 40), so the history never reaches an output pixel.
//
// 3D (-d 3 -F): Process with f = 1 (:837,851-866) combs frame k once frame
// k+1 has arrived; Split3D(opt_flow = false) :369-412 adds a temporal chroma
// estimate clp2 = (prev + next)/2 - cur (integer average) with weight combk2
// from the lp_3d-filtered |next - prev| of the line, and combk1 = 1 - combk2.
// Only ldg_k_comb_split changes (ldg_k_comb_split3): the frames are passed as
// a contiguous window, so frame k's neighbours are one frame before and after.
// Split3D reads _k[4] and _k[832..835] without writing them (uninitialised
// stack in the reference): build-defined 0 here and in the oracle.
//
// Three row kernels, so that no workgroup holds a CU's LDS while one lane
// runs a 418-step chain:
//   ldg_k_comb_split  one workgroup per (frame, row): raw rows l-2, l, l+2 in
//                     LDS -> Split1D / Split2D -> the signed chroma cv[h] of
//                     SplitIQ, written to HBM (910 doubles per row);
//   ldg_k_comb_iq     one LANE per FilterIQ chain (row, I or Q): reads the held
//                     I / Q feeds from cv, runs the recurrence in the
//                     reference's arithmetic order, writes the 418 outputs;
//   ldg_k_comb_out    one workgroup per (frame, row): AdjustY from the raw line
//                     and cv, the FilterIQ outputs, DoYNR, YIQ -> RGB.
// At comb-ntsc's defaults (the CLI's and the benchmark's comb) the three run as
// one row kernel, ldg_k_comb_fused: cv and the FilterIQ outputs stay in LDS and
// the chains run as verified warm-started chunks across lanes (below).
#include <hip/hip_runtime.h>
#include "common.hpp"

namespace ldg {
namespace comb {

constexpr int IN_X = 910, IN_Y = 525;
constexpr int OUT_W = 744, OUT_H = 480, OUT_X0 = 78, FIRST_LINE = 38;
constexpr int OUT_HMAX = IN_Y;                             // rows per output frame with -v
constexpr int ROWS_MAX = IN_Y - 20;                        // combed rows with -v (lines 20..524)
constexpr int CHAIN_LINES = IN_Y - FIRST_LINE;            // 487 lines feed aburstlev per frame (505 with -v)
constexpr int CHAIN_MAX = IN_Y - 20;
constexpr int CV_STRIDE = 912;                             // doubles per row of the cv buffer
constexpr int IQ_ROWS_MAX = ROWS_MAX - (44 - 20);          // rows per frame that run the FilterIQ chains
constexpr double IRESCALE = 358.4, IREBASE = 1024.0;
constexpr double P_2DRANGE = 45 * IRESCALE;
constexpr double LPI_B0 = 2.267438981796600e-01, LPI_B1 = 2.267438981796600e-01;
constexpr double LPI_A1 = -5.465122036406802e-01;
constexpr double LPQ_B0 = 1.169303716013410e-01, LPQ_B1 = 1.169303716013410e-01;   // f_colorlpq (-Q)
constexpr double LPQ_A1 = -7.661392567973181e-01;

// comb-ntsc's options (main's getopt, comb-ntsc.cxx:972-1091), as the kernels use them
struct CombOpt {
  int firstline;      // 38; 20 with -v (linesout == 525): AdjustY / DoYNR / DoCNR / ToRGB start there
  int nrows;          // combed rows: lines firstline .. firstline + nrows - 1 (480; 505 with -v)
  int out_rows;       // rows per output frame (linesout); rows >= nrows stay 0 (never written)
  int adaptive2d;     // Split2D's adaptive weights (-a turns them off)
  int bw;             // -B: SplitIQ zeroes I and Q
  int colorlpf;       // FilterIQ (-L turns it off)
  int lpq;            // -Q: Q through f_colorlpq instead of f_colorlpi
  int debug_row;      // -l: this output row is black (-1: none)
  double black_ire;   // -I
  double bright_m;    // -b: brightness * 256 / 100
  double nr_y, nr_c;  // -n / -N times irescale; <= 0: DoYNR / DoCNR skipped
  int of;             // ldg_comb_ntsc3d with optical flow (comb-ntsc -d 3 without -F; host only)
  int wide;           // -W: 910-wide rows from x 0 (PostProcess rout_x / roffset, comb-ntsc.cxx:898-899);
                      // nrows then covers every line DoYNR feeds (to 524) for its cross-line history
  __host__ __device__ int out_w() const { return wide ? IN_X : OUT_W; }
  __host__ __device__ int out_x0() const { return wide ? 0 : OUT_X0; }
  __host__ __device__ int iq_row0() const { return 44 - firstline; }               // first row with FilterIQ (line 44)
  __host__ __device__ int iq_rows() const { return nrows - iq_row0(); }
  __host__ __device__ int chain_lines() const { return IN_Y - firstline; }
};

// comb-ntsc's defaults as compile-time constants (comb-ntsc.cxx:15-75,1074-1091):
// the kernels are instantiated for CombOpt (ldg_comb_set_opts) and for this, the
// options every CLI / benchmark run without comb flags uses; with them folded the
// kernels keep fewer registers (comb_out 78 VGPRs instead of 95) and no option tests.
struct CombDefaults {
  static constexpr int firstline = FIRST_LINE, nrows = OUT_H, out_rows = OUT_H;
  static constexpr int adaptive2d = 1, bw = 0, colorlpf = 1, lpq = 0, debug_row = -1;
  static constexpr double black_ire = 7.5, bright_m = 236.0 * 256 / 100, nr_y = 1.0 * IRESCALE, nr_c = 0.0;
  static constexpr int wide = 0;
  __host__ __device__ static constexpr int out_w() { return OUT_W; }
  __host__ __device__ static constexpr int out_x0() { return OUT_X0; }
  __host__ __device__ static constexpr int iq_row0() { return 44 - firstline; }
  __host__ __device__ static constexpr int iq_rows() { return nrows - iq_row0(); }
  __host__ __device__ static constexpr int chain_lines() { return IN_Y - firstline; }
};

struct LP3DTaps { double b[17]; };   // lp_3d = fir1(16, 0.1), comb-ntsc.cxx:379
__constant__ LP3DTaps g_lp3d = {{0.005719569452904, 0.009426612841315, 0.019748592575455, 0.036822680065252,
                                 0.058983880135427, 0.082947830292278, 0.104489989820068, 0.119454688318951,
                                 0.124812312996699, 0.119454688318952, 0.104489989820068, 0.082947830292278,
                                 0.058983880135427, 0.036822680065252, 0.019748592575455, 0.009426612841315,
                                 0.005719569452904}};
struct NRCTaps { double b[17]; };  // deemp.h f_nrc (DoCNR)
__constant__ NRCTaps g_nrc = {{
    -3.148569668063267e-03, -4.941974513425438e-03, -9.929538598536455e-03, -1.787793973911701e-02,
    -2.783702315543740e-02, -3.829928032339736e-02, -4.750186865627083e-02, -5.380281552534787e-02,
    9.469899799540406e-01,  -5.380281552534787e-02, -4.750186865627083e-02, -3.829928032339737e-02,
    -2.783702315543740e-02, -1.787793973911701e-02, -9.929538598536455e-03, -4.941974513425442e-03,
    -3.148569668063267e-03}};
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

// clp1 with the three clp0 rows staged in LDS (p = l-2, c = l, n = l+2; the
// PAL decoder passes l-4 / l+4 and its own p_2drange = 45 * its irescale).
__device__ __forceinline__ double clp1_v(double c0, double cm, double p0, double pm, double n0, double nm,
                                         double p2drange = P_2DRANGE, bool adaptive = true);
__device__ __forceinline__ double clp1_lds(const double* p1, const double* c1, const double* n1, int h,
                                           double p2drange = P_2DRANGE, bool adaptive = true) {
  return clp1_v(c1[h], c1[h - 1], p1[h], p1[h - 1], n1[h], n1[h - 1], p2drange, adaptive);
}
// the same from the six clp0 values (line l at h / h-1, l-2, l+2)
__device__ __forceinline__ double clp1_v(double c0, double cm, double p0, double pm, double n0, double nm,
                                         double p2drange, bool adaptive) {
  double kp = fabs(fabs(c0) - fabs(p0));
  kp += fabs(fabs(cm) - fabs(pm));
  kp -= (fabs(c0) + fabs(cm)) * .10;
  double kn = fabs(fabs(c0) - fabs(n0));
  kn += fabs(fabs(cm) - fabs(nm));
  kn -= (fabs(c0) + fabs(nm)) * .10;
  kp /= 2;
  kn /= 2;
  kp = clampd(1 - (kp / p2drange), 0, 1);
  kn = clampd(1 - (kn / p2drange), 0, 1);
  if (!adaptive) kn = kp = 1.0;                          // -a (comb-ntsc.cxx:333)
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

// SplitIQ's held I / Q at pixel p (0 outside [4, 840)) from the signed chroma cv.
__device__ __forceinline__ double held_i(const double* __restrict__ cv, int p) {
  if (p < 4 || p >= 840) return 0.0;
  const int he = p & ~1;                 // latest even h' <= p (phase 0 / 2)
  return ((he & 3) == 0) ? cv[he] : -cv[he];
}
__device__ __forceinline__ double held_q(const double* __restrict__ cv, int p) {
  if (p < 4 || p >= 840) return 0.0;
  const int ho = (p & 1) ? p : p - 1;    // latest odd h' <= p (phase 1 / 3), none before 5
  if (ho < 5) return 0.0;
  return ((ho & 3) == 1) ? -cv[ho] : cv[ho];
}

// FilterIQ's colorlpi chains: feeds h = H0 + 2k < 840 (H0 = 4 for I, 5 for Q),
// k < 418; the feed at h writes its output to pixels h-2 and h-1 (h-1 only
// while h+1 < 840; Q's pixel 2 is never fed and reads 0).
constexpr int IQ_NS = 418;

}  // namespace comb
}  // namespace ldg

using namespace ldg::comb;

// aburstlev chain (ToRGB :560-566) over lines 38..524 of n frames in order.
// state[0]: aburstlev carried across calls (-1 = not initialised).
// abl[f * CHAIN_LINES + (l - 38)]: the value ToRGB uses for line l of frame f.
//
// The recurrence is sequential in the reference and must stay bit-exact, but it
// forgets: two runs of it over the same levels from different states differ by
// 0.99^k after k qualifying lines, and once their difference is below an ulp
// they round to the same double and stay identical from then on.  So the lines
// of a piece are split into 256 chunks, one per thread; thread j starts `warm`
// lines before its chunk (from the piece's true state when that reaches back to
// the piece start, else from "not initialised") and runs the chain through its
// chunk.  Its state entering the chunk equals the state thread j-1 ends with iff
// the two runs have met, and then thread j's chunk is exactly the sequential
// chain's (by induction from chunk 0, which starts from the true state).  A chunk
// whose check fails is recomputed, with everything after it, sequentially by
// thread 0 from the verified state before it (the round-1 kernel's path).  With
// warm = 5120 a run from a guess within a few IRE meets the true one after
// ~3500 qualifying lines, so the serial path is a fallback; LDG_COMB_WARM small
// forces it (tests).  About warm + total/256 steps per thread instead of total
// steps on one lane: ~6k instead of ~30k for a 60-frame call.
// grid: 1 workgroup of 256 threads.
constexpr int BURST_PIECE = 40960;   // lines staged per pass (80 KiB of uint16 levels in LDS)
// raw / IRESCALE correctly rounded from a product and one FMA correction:
// checked equal to the division for every uint16 (tools/burst_div_check.c)
__device__ __forceinline__ double burst_level(uint16_t raw) {
  constexpr double INV = 1.0 / IRESCALE;
  const double x = (double)raw;
  const double q = x * INV;
  return __fma_rn(__fma_rn(-q, IRESCALE, x), INV, q);
}
__device__ __forceinline__ double burst_step(double a, uint16_t raw) {
  const double bk = burst_level(raw);                  // comb-ntsc.cxx:560
  const double base = (a < 0) ? bk : a;                // :563 (first qualifying line)
  const double e = (base * .99) + (bk * .01);          // :564
  return (bk > 3) ? e : a;
}
// The chain over s_u[k0, k1) from state a (abl[k] written when out != null).
// Once initialised (a > 0) a step is a = (a * m) + c with m = .99, c = bk * .01
// on a qualifying line and m = 1, c = 0 otherwise -- the same two roundings as
// the reference, and exactly a again on a skipped line -- so only a multiply and
// an add are on the dependency path; the levels of 16 lines are computed ahead.
__device__ __forceinline__ double burst_run(const uint16_t* s_u, int k0, int k1, double a, double* out) {
  int k = k0;
  for (; k < k1 && a < 0; k++) {
    a = burst_step(a, s_u[k]);
    if (out) out[k] = a;
  }
#pragma unroll 1
  for (; k + 16 <= k1; k += 16) {
    double m[16], c[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const double bk = burst_level(s_u[k + j]);
      const bool q = bk > 3;
      m[j] = q ? .99 : 1.0;
      c[j] = q ? bk * .01 : 0.0;
    }
#pragma unroll
    for (int j = 0; j < 16; j++) {
      a = (a * m[j]) + c[j];
      if (out) out[k + j] = a;
    }
  }
  for (; k < k1; k++) {
    a = burst_step(a, s_u[k]);
    if (out) out[k] = a;
  }
  return a;
}
extern "C" __global__ __launch_bounds__(256) void ldg_k_comb_burst(const uint16_t* __restrict__ frames, int n,
                                                                   double* __restrict__ state,
                                                                   double* __restrict__ abl, int warm,
                                                                   int firstline) {
  prio_latency();

  __shared__ uint16_t s_u[BURST_PIECE];
  __shared__ double s_in[256], s_out[256];
  __shared__ double s_fm[BURST_PIECE / 256], s_fc[BURST_PIECE / 256];   // the fix-up's per-line terms (one chunk)
  __shared__ int s_bad, s_stop;
  const int tid = threadIdx.x;
  double a_in = state[0];
  const int chain = IN_Y - firstline;
  const int total = n * chain;
  for (int p0 = 0; p0 < total; p0 += BURST_PIECE) {
    const int cnt = (total - p0) < BURST_PIECE ? (total - p0) : BURST_PIECE;
    // one uint16 per line, 1820 B apart: issue 16 loads per thread before their LDS
    // stores, so the staging costs a few memory latencies instead of one per line
    for (int k0 = 0; k0 < cnt; k0 += 16 * 256) {
      uint16_t v[16];
#pragma unroll
      for (int u = 0; u < 16; u++) {
        const int k = k0 + u * 256 + tid;
        const int j = p0 + k;
        const int f = j / chain, l = firstline + j % chain;
        v[u] = (k < cnt) ? frames[(size_t)f * IN_X * IN_Y + (size_t)l * IN_X + 1] : (uint16_t)0;
      }
#pragma unroll
      for (int u = 0; u < 16; u++) {
        const int k = k0 + u * 256 + tid;
        if (k < cnt) s_u[k] = v[u];
      }
    }
    if (tid == 0) s_bad = cnt;
    __syncthreads();
    const int L = (cnt + 255) / 256;
    const int c0 = tid * L, c1 = (c0 + L) < cnt ? c0 + L : cnt;
    if (c0 < cnt) {
      const int w = (c0 - warm) > 0 ? c0 - warm : 0;
      double a = burst_run(s_u, w, c0, (w == 0) ? a_in : -1.0, nullptr);
      s_in[tid] = a;
      a = burst_run(s_u, c0, c1, a, abl + p0);
      s_out[tid] = a;
    }
    __syncthreads();
    if (tid > 0 && c0 < cnt && __double_as_longlong(s_in[tid]) != __double_as_longlong(s_out[tid - 1]))
      atomicMin(&s_bad, c0);
    __syncthreads();
    const int bad = s_bad;
    const int last = (cnt - 1) / L;                     // the thread holding the piece's last line
    if (bad < cnt) {
      // The sequential chain from the verified state before the failed chunk, on wave 0:
      // each lane forms one line's multiplier / addend (the level arithmetic and its test
      // off the dependency path), lane 0 chains 64 lines at a time with only the multiply
      // and the add on the path (one thread doing it all ran ~120 cycles per line: the
      // per-line level test went through the scalar unit inside the chain).  It stops at
      // the first chunk end where the exact state equals that chunk's speculative end:
      // from there every chunk whose start check passed is exact, so it resumes only at
      // the next failed boundary.
      if (tid < 64) {
        int q = bad / L;                                 // the failed chunk
        double a = s_out[q - 1];                         // exact (the chunks before q are)
        while (q <= last) {
          bool met = false;
          for (; q <= last && !met; q++) {
            const int k0 = q * L, k1 = (k0 + L) < cnt ? k0 + L : cnt;
            for (int kk = k0 + tid; kk < k1; kk += 64) {
              const double bk = burst_level(s_u[kk]);
              const bool qual = bk > 3;
              s_fm[kk - k0] = qual ? .99 : 1.0;
              s_fc[kk - k0] = qual ? bk * .01 : 0.0;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            if (tid == 0) {
              const int nb = k1 - k0;
              int j = 0;
              for (; j < nb && a < 0; j++) {             // not yet initialised (the stream's first lines)
                a = burst_step(a, s_u[k0 + j]);
                abl[p0 + k0 + j] = a;
              }
#pragma unroll 1
              for (; j + 16 <= nb; j += 16) {
                double mm[16], cc[16];
#pragma unroll
                for (int u = 0; u < 16; u++) { mm[u] = s_fm[j + u]; cc[u] = s_fc[j + u]; }
#pragma unroll
                for (int u = 0; u < 16; u++) {
                  a = (a * mm[u]) + cc[u];
                  abl[p0 + k0 + j + u] = a;
                }
              }
              for (; j < nb; j++) {
                a = (a * s_fm[j]) + s_fc[j];
                abl[p0 + k0 + j] = a;
              }
              s_stop = __double_as_longlong(a) == __double_as_longlong(s_out[q]);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            met = s_stop != 0;
          }
          if (!met) {                                    // ran to the piece's end
            if (tid == 0) s_out[last] = a;
            break;
          }
          // the exact state after chunk q - 1 is its speculative end: chunks from q on are
          // exact up to the next failed start check
          int nxt = 256;
          for (int m = q + tid; m <= last; m += 64)
            if (__double_as_longlong(s_in[m]) != __double_as_longlong(s_out[m - 1])) { nxt = m; break; }
          for (int o = 32; o > 0; o >>= 1) nxt = min(nxt, __shfl_xor(nxt, o));
          if (nxt > last) break;                         // s_out[last] is exact already
          q = nxt;
          a = s_out[q - 1];
        }
      }
      __syncthreads();
    }
    a_in = s_out[last];
    __syncthreads();
  }
  if (tid == 0 && total > 0) state[0] = a_in;
}

// ---- ldg_k_comb_split: SplitIQ's signed chroma of one row.
// grid: n * O.nrows workgroups of 256 threads; row r = line r + firstline; cv: [n][nrows][CV_STRIDE].
// D3: frames[f] has its neighbours at frames[f -+ 1] (core / range: p_3dcore,
// p_3drange times irescale).  OF (with D3): the 3D mode with optical flow
// (Split3D(f, true), comb-ntsc.cxx:395-407): clp2 = next - cur and combk[2] from the
// flow's weight map kmap[f] (252 x 840 per frame: frame rows 2 y, 2 y + 1, columns
// 70..909; 0 elsewhere; flow.hip ldg_k_flow_combk).
template <bool D3, class OPT, bool OF = false>
__device__ __forceinline__ void comb_split_row(const uint16_t* __restrict__ frames, double* __restrict__ cvbuf,
                                               double core, double range, const OPT& O,
                                               const double* __restrict__ kmap = nullptr) {
  __shared__ uint16_t s_raw[3][IN_X + 2];                // raw lines l-2, l, l+2
  __shared__ double s_c[3][IN_X];                        // Split1D clp0 of those lines
  __shared__ uint16_t s_pn[D3 ? 2 : 1][IN_X + 2];        // 3D: line l of the previous / next frame
  __shared__ double s_x[D3 ? IN_X : 1];                  // 3D: lp_3d's input __k (0 where not fed)
  const int tid = threadIdx.x;
  const int f = blockIdx.x / O.nrows;
  const int row = blockIdx.x % O.nrows;
  const int l = row + O.firstline;
  double* cvrow = cvbuf + ((size_t)f * O.nrows + row) * CV_STRIDE;
  if (l < 36 || O.bw) {
    // SplitIQ covers lines 36..524 (the rest of cbuf is zero); -B zeroes I and Q
    for (int h = tid; h < CV_STRIDE; h += 256) cvrow[h] = 0.0;
    return;
  }
  const uint16_t* fr = frames + (size_t)f * IN_X * IN_Y;
  // lines are 1820 B apart: 4-byte loads are aligned; rows past 524 (l + 2 with -v) are
  // outside the frame and read as 0 (clpbuffer row 525 is the zeroed next plane)
  for (int t = tid; t < 3 * (IN_X / 2); t += 256) {
    const int k = t / (IN_X / 2), w = t % (IN_X / 2);
    const int r = l - 2 + 2 * k;
    const uint32_t v = (r < IN_Y) ? reinterpret_cast<const uint32_t*>(fr + (size_t)r * IN_X)[w] : 0u;
    s_raw[k][2 * w] = (uint16_t)(v & 0xffff);
    s_raw[k][2 * w + 1] = (uint16_t)(v >> 16);
  }
  if constexpr (D3) {
    for (int t = tid; t < 2 * (IN_X / 2); t += 256) {
      const int k = t / (IN_X / 2), w = t % (IN_X / 2);
      const uint16_t* nb = fr + (k ? 1 : -1) * (ptrdiff_t)IN_X * IN_Y;   // k 0: previous, 1: next frame
      const uint32_t v = reinterpret_cast<const uint32_t*>(nb + (size_t)l * IN_X)[w];
      s_pn[k][2 * w] = (uint16_t)(v & 0xffff);
      s_pn[k][2 * w + 1] = (uint16_t)(v >> 16);
    }
  }
  __syncthreads();
  if constexpr (D3 && !OF) {
    // __k = |F0 - F2| + |(F1 - F2) - (F1 - F0)| (ints), fed to lp_3d for h = 13..839
    for (int h = tid; h < IN_X; h += 256) {
      double k = 0.0;
      if (h > 12 && h < 840) {
        const int p = s_pn[0][h], c = s_raw[1][h], nx = s_pn[1][h];
        k = abs(nx - p);
        k += abs((c - p) - (c - nx));
      }
      s_x[h] = k;
    }
  }
  for (int h = tid; h < IN_X; h += 256) {
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const int r = l - 2 + 2 * k;
      double c = 0.0;
      if (r >= 44 && r < IN_Y && h >= 4 && h < 840) {
        const int avg = ((int)s_raw[k][h + 2] + (int)s_raw[k][h - 2]) / 2;   // integer average (Split1D)
        c = (double)(avg - (int)s_raw[k][h]);
      }
      s_c[k][h] = c;
    }
  }
  __syncthreads();
  const bool invertphase = (s_raw[1][0] == 16384);
  const bool adaptive = O.adaptive2d != 0;
  for (int h = tid; h < CV_STRIDE; h += 256) {
    double cv = 0.0;
    if (h >= 4 && h < 840) {
      double cavg = 0;
      if constexpr (D3) {
        double k2, clp2;
        if constexpr (OF) {
          // the flow's weight (OpticalFlow3D writes frame rows 0..503, columns 70..909)
          k2 = (l < 2 * flow::FR && h >= flow::FX0) ? kmap[(size_t)f * flow::FR * flow::FC +
                                                           (size_t)(l >> 1) * flow::FC + (h - flow::FX0)] : 0.0;
          clp2 = (double)((int)s_pn[1][h] - (int)s_raw[1][h]);    // p3line (Frame[0], the next frame) - line
        } else {
          // _k[h] = lp_3d output of the feed at h + 8 (h = 5..831), the raw __k at
          // 836..839, 0 at 4 and 832..835 (never written in the reference)
          double kk = 0.0;
          if (h >= 5 && h <= 831) {
#pragma unroll
            for (int t = 0; t < 17; t++) kk += (g_lp3d.b[t] / 1.0) * s_x[h + 8 - t];
          } else if (h >= 836) {
            kk = s_x[h];
          }
          k2 = clampd(1 - ((kk - core) / range), 0, 1);
          clp2 = (double)((((int)s_pn[1][h] + (int)s_pn[0][h]) / 2) - (int)s_raw[1][h]);
        }
        const double k1 = (l <= 523) ? 1 - k2 : 0.0;     // Split3D :401-403 (Split2D left line 524 at 0)
        const double k0 = 1 - k2 - k1;
        const double clp1 = (l < 524 && h >= 18) ? clp1_lds(s_c[0], s_c[1], s_c[2], h, P_2DRANGE, adaptive) : 0.0;
        cavg += clp2 * k2;
        cavg += clp1 * k1;
        cavg += s_c[1][h] * k0;
      } else {
        cavg += 0.0 * 0.0;                               // clpbuffer[2] * combk[2]
        if (l < 524 && h >= 18) {
          cavg += clp1_lds(s_c[0], s_c[1], s_c[2], h, P_2DRANGE, adaptive) * 1.0;
          cavg += s_c[1][h] * 0.0;
        } else {
          cavg += 0.0 * 0.0;
          cavg += s_c[1][h] * 1.0;
        }
      }
      cavg /= 2;
      if (!invertphase) cavg = -cavg;
      cv = cavg;
    }
    cvrow[h] = cv;
  }
}

extern "C" __global__ __launch_bounds__(256) void ldg_k_comb_split(const uint16_t* __restrict__ frames,
                                                                   double* __restrict__ cvbuf) {
  comb_split_row<false>(frames, cvbuf, 0.0, 1.0, CombDefaults{});
}
extern "C" __global__ __launch_bounds__(256) void ldg_k_comb_split_opt(const uint16_t* __restrict__ frames,
                                                                       double* __restrict__ cvbuf, CombOpt O) {
  comb_split_row<false>(frames, cvbuf, 0.0, 1.0, O);
}

// 3D (-d 3 -F): frames[-1] and frames[n] must be valid (the window's neighbours).
extern "C" __global__ __launch_bounds__(256) void ldg_k_comb_split3(const uint16_t* __restrict__ frames,
                                                                    double* __restrict__ cvbuf, double core,
                                                                    double range, CombOpt O) {
  comb_split_row<true>(frames, cvbuf, core, range, O);
}
// 3D with optical flow (-d 3): frames[n] must be valid; kmap: one weight map per frame.
extern "C" __global__ __launch_bounds__(256) void ldg_k_comb_split3_of(const uint16_t* __restrict__ frames,
                                                                       double* __restrict__ cvbuf, CombOpt O,
                                                                       const double* __restrict__ kmap) {
  comb_split_row<true, CombOpt, true>(frames, cvbuf, 0.0, 1.0, O, kmap);
}

// ---- ldg_k_comb_iq: FilterIQ's two chains of every row with line >= 44, one
// lane each.  Feed h: x_h = AdjustY's I (Q) at h = the held value at h + 2;
// y = ((0 + b0 x_h) + b1 x_{h-2}) - a1 y_prev in the reference's order
// (Filter::feed, ld-decoder.h:180-186); Q through f_colorlpq with -Q.
// grid: ceil(n * iq_rows * 2 / 256) x 256.  iq: [n][iq_rows][2][IQ_NS] outputs.
template <class OPT>
__device__ __forceinline__ void comb_iq_lane(const double* __restrict__ cvbuf, int n, double* __restrict__ iq,
                                             const OPT& O) {
  prio_latency();

  const int rows = O.iq_rows();
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= n * rows * 2) return;
  const int q = c & 1, rr = (c >> 1) % rows, f = (c >> 1) / rows;
  const double* cv = cvbuf + ((size_t)f * O.nrows + O.iq_row0() + rr) * CV_STRIDE;
  double* out = iq + (((size_t)f * rows + rr) * 2 + q) * IQ_NS;
  const bool lq = q && O.lpq;
  const double B0 = lq ? LPQ_B0 : LPI_B0, B1 = lq ? LPQ_B1 : LPI_B1, A1 = lq ? LPQ_A1 : LPI_A1;
  // feed k reads the held value at p = H0 + 2k + 2: I (p = 6 + 2k, even) is
  // -cv[p] for even k and +cv[p] for odd k; Q (p = 7 + 2k, odd) is +cv[p] for
  // even k and -cv[p] for odd k; both are 0 at p >= 840 (k = 417).  Lanes c
  // and c + 1 (I and Q of one row) read the same pairs (cv[6 + 2k], cv[7 + 2k]).
  const double2* cv2 = reinterpret_cast<const double2*>(cv) + 3;
  double x1 = 0.0, y1 = 0.0;
  // the feeds of chunk kb + 16 are loaded while chunk kb's steps run (the chain is
  // then bound by its own FP64 latency, not by a load round trip per chunk)
  double nx[16];
#pragma unroll
  for (int j = 0; j < 16; j++) {
    const double2 v = cv2[j];
    nx[j] = q ? v.y : v.x;
  }
#pragma unroll 1
  for (int kb = 0; kb < IQ_NS; kb += 16) {
    double xs[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const int k = kb + j;
      xs[j] = (k >= IQ_NS - 1) ? 0.0 : (((k & 1) != q) ? nx[j] : -nx[j]);
    }
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const int k = kb + 16 + j;
      const double2 v = cv2[k < IQ_NS - 1 ? k : 0];
      nx[j] = q ? v.y : v.x;
    }
#pragma unroll
    for (int j = 0; j < 16; j += 2) {
      if (kb + j < IQ_NS) {
        double ya = 0;
        ya += (B0 / 1.0) * xs[j];
        ya += (B1 / 1.0) * x1;
        ya -= (A1 / 1.0) * y1;
        double yb = 0;
        yb += (B0 / 1.0) * xs[j + 1];
        yb += (B1 / 1.0) * xs[j];
        yb -= (A1 / 1.0) * ya;
        x1 = xs[j + 1];
        y1 = yb;
        *reinterpret_cast<double2*>(out + kb + j) = make_double2(ya, yb);
      }
    }
  }
}

extern "C" __global__ __launch_bounds__(256) void ldg_k_comb_iq(const double* __restrict__ cvbuf, int n,
                                                                double* __restrict__ iq) {
  comb_iq_lane(cvbuf, n, iq, CombDefaults{});
}
extern "C" __global__ __launch_bounds__(256) void ldg_k_comb_iq_opt(const double* __restrict__ cvbuf, int n,
                                                                    double* __restrict__ iq, CombOpt O) {
  comb_iq_lane(cvbuf, n, iq, O);
}

// ---- ldg_k_comb_out: AdjustY, the FilterIQ outputs, the VBI copy, DoYNR,
// DoCNR and ToRGB of one output row.  grid: n * O.out_rows workgroups of 256
// threads (rows >= O.nrows are the -v frame's never-written bottom rows: 0).
// For output pixels x >= 78 every FIR tap of DoYNR (h - 12 >= 66 >= 40) and
// DoCNR (h + 12 - 16 >= 74 >= 60) falls inside the row, so their cross-line
// histories never reach an output pixel.  With -W (x from 0) DoYNR's taps at
// x 40..51 reach the previous fed line's last 12 feeds (positions 832..843 of
// line l-1, or of line 524 of the previous frame -- of the previous call's last
// frame through hist_in, 0 for the stream's first frame); DoCNR's reach only
// positions 839..842 of the previous line, which are always 0 (FilterIQ writes
// I / Q up to 837, AdjustY's held values past 840 are 0).

// The Y DoYNR feeds at pixel p (40 <= p <= 843) of line L: AdjustY's (or the VBI
// copy's) value, from the raw lines and L's signed-chroma row cv (comb-ntsc.cxx
// :735-763, :870-877).
__device__ __forceinline__ double fed_y(const uint16_t* __restrict__ fr, const double* __restrict__ cv, int L, int p) {
  if (p >= 842) return 0.0;                              // untouched by AdjustY, never set by SplitIQ
  if (L < 24 && p >= 4 && p < 840) return (double)fr[(size_t)(L + 20) * IN_X + p];
  const uint16_t* line = fr + (size_t)L * IN_X;
  const int q = p + 2;
  const double yy = (L >= 36 && q >= 4 && q < 840) ? (double)line[q] : 0.0;
  const double ii = held_i(cv, q), qq = held_q(cv, q);
  double comp = 0;
  switch (p & 3) {
    case 0: comp = ii; break;
    case 1: comp = -qq; break;
    case 2: comp = -ii; break;
    default: comp = qq; break;
  }
  if (line[0] == 16384) comp = -comp;
  return yy + comp;
}

template <class OPT>
__device__ __forceinline__ void comb_out_row(const uint16_t* __restrict__ frames, const double* __restrict__ cvbuf,
                                             const double* __restrict__ iq, const double* __restrict__ abl,
                                             uint16_t* __restrict__ rgb, const OPT& O,
                                             const double* __restrict__ hist_in = nullptr,
                                             double* __restrict__ hist_out = nullptr, int n = 0) {
  __shared__ uint16_t s_line[IN_X + 2];
  __shared__ uint16_t s_vbi[IN_X + 2];                   // -v: raw line l + 20 (the VBI copy, rows 20..23)
  __shared__ double s_y[IN_X];                           // AdjustY's Y (+ the VBI copy)
  __shared__ double s_i[IN_X], s_q[IN_X];                // FilterIQ's I / Q (DoCNR's input)
  __shared__ double s_hist[12];                          // -W: the previous fed line's feeds 832..843
  const int tid = threadIdx.x;
  const int f = blockIdx.x / O.out_rows;
  const int row = blockIdx.x % O.out_rows;
  const int W = O.out_w(), X0 = O.out_x0();
  uint16_t* out = rgb + ((size_t)f * O.out_rows + row) * W * 3;
  if (row >= O.nrows) {
    for (int x = tid; x < W * 3; x += 256) out[x] = 0;
    return;
  }
  const int l = row + O.firstline;
  const uint16_t* fr = frames + (size_t)f * IN_X * IN_Y;
  const uint16_t* line = fr + (size_t)l * IN_X;
  const bool vbi = l < 24;                                 // tbuf rows 0..23 hold raw lines 20..43
  for (int w = tid; w < IN_X / 2; w += 256) {
    const uint32_t v = reinterpret_cast<const uint32_t*>(line)[w];
    s_line[2 * w] = (uint16_t)(v & 0xffff);
    s_line[2 * w + 1] = (uint16_t)(v >> 16);
    if (vbi) {
      const uint32_t u = reinterpret_cast<const uint32_t*>(fr + (size_t)(l + 20) * IN_X)[w];
      s_vbi[2 * w] = (uint16_t)(u & 0xffff);
      s_vbi[2 * w + 1] = (uint16_t)(u >> 16);
    }
  }
  if (O.wide) {
    // DoYNR's history: the previous fed line (l - 1, or line 524 of the previous
    // frame); the last row of the call's last frame hands its own feeds to the next call
    const size_t fsz = (size_t)IN_X * IN_Y;
    const int last = IN_Y - O.firstline - 1;             // the row of line 524 (nrows covers it with -W)
    if (tid < 12) {
      double v = 0.0;
      if (row > 0)
        v = fed_y(fr, cvbuf + ((size_t)f * O.nrows + row - 1) * CV_STRIDE, l - 1, 832 + tid);
      else if (f > 0)
        v = fed_y(fr - fsz, cvbuf + ((size_t)(f - 1) * O.nrows + last) * CV_STRIDE, IN_Y - 1, 832 + tid);
      else if (hist_in)
        v = hist_in[tid];
      s_hist[tid] = v;
    } else if (row == 0 && f == n - 1 && hist_out && tid >= 32 && tid < 44) {
      hist_out[tid - 32] = fed_y(fr, cvbuf + ((size_t)f * O.nrows + last) * CV_STRIDE, IN_Y - 1, 832 + tid - 32);
    }
  }
  __syncthreads();
  const bool invertphase = (s_line[0] == 16384);
  const bool ycb = l >= 36;                              // SplitIQ sets cbuf's Y on lines 36..524 only
  const double* cv = cvbuf + ((size_t)f * O.nrows + row) * CV_STRIDE;
  const bool fiq = O.colorlpf && l >= 44;
  const double* iqI = fiq ? iq + (((size_t)f * O.iq_rows() + (row - O.iq_row0())) * 2 + 0) * IQ_NS : nullptr;
  const double* iqQ = iqI ? iqI + IQ_NS : nullptr;
  // I / Q at pixel t after FilterIQ (lines >= 44: I from feed (t - 2) / 2 for t in
  // [2, 838), Q from feed (t - 3) / 2 for t in [3, 838)), otherwise AdjustY's I / Q
  // (the held values at t + 2: 0 past 837 and before 2)
  auto I_at = [&](int t) { return (iqI && t >= 2 && t < 838) ? iqI[(t - 2) >> 1] : held_i(cv, t + 2); };
  auto Q_at = [&](int t) { return (iqQ && t >= 3 && t < 838) ? iqQ[(t - 3) >> 1] : (iqQ && t == 2) ? 0.0 : held_q(cv, t + 2); };
  // ---- AdjustY: p[h] = p[h + 2] with y += +-I / +-Q (h in [2, 842)); only
  //      h in [66, 834) reaches an output pixel (DoYNR taps h-12..h+12), all of
  //      of [0, 910) with -W (0 where AdjustY and SplitIQ leave the row alone)
  const int ylo = O.wide ? 0 : 66, yhi = O.wide ? IN_X : 834;
  for (int h = ylo + tid; h < yhi; h += 256) {
    const int p = h + 2;
    const double yy = (ycb && p >= 4 && p < 840) ? (double)s_line[p] : 0.0;
    const double ii = held_i(cv, p), qq = held_q(cv, p);
    double comp = 0;
    switch (h & 3) {
      case 0: comp = ii; break;
      case 1: comp = -qq; break;
      case 2: comp = -ii; break;
      default: comp = qq; break;
    }
    if (invertphase) comp = -comp;
    double v = (vbi && h >= 4 && h < 840) ? (double)s_vbi[h] : yy + comp;
    if (h < 2 || h >= 842) v = 0.0;
    s_y[h] = v;
  }
  if (O.nr_c > 0) {
    const int clo = O.wide ? 56 : 74, chi = O.wide ? 843 : 834;
    for (int t = clo + tid; t < chi; t += 256) {
      s_i[t] = t < 60 ? 0.0 : I_at(t);                   // t < 60: the previous line's feeds 839..842 (0)
      s_q[t] = t < 60 ? 0.0 : Q_at(t);
    }
  }
  __syncthreads();
  // ---- DoYNR, DoCNR, ToRGB
  const double aburst = abl[(size_t)f * O.chain_lines() + (l - O.firstline)];
  const double m = O.bright_m;
  const bool black = row == O.debug_row;
  const double kc = 10 / aburst, kb = 100 / (100 - O.black_ire);   // per-pixel factors of ToRGB, hoisted
  for (int x = tid; x < W; x += 256) {
    const int h = x + X0;
    double yv = s_y[h];
    // DoYNR on h in [40, 843); hplinef[h + 12] past the last feed (843) is 0
    if (O.nr_y > 0 && (!O.wide || (h >= 40 && h + 12 <= 843))) {
      double y0 = 0;
#pragma unroll
      for (int o = 0; o < 25; o++) {
        const int pp = h + 12 - o;
        const double xv = (O.wide && pp < 40) ? s_hist[pp - 28] : s_y[pp];
        y0 += (g_nr.b[o] / 1.0) * xv;
      }
      double a = y0;
      if (fabs(a) > O.nr_y) a = (a > 0) ? O.nr_y : -O.nr_y;
      yv = s_y[h] - a;
    }
    double iv, qv;
    if (O.nr_c > 0 && (!O.wide || (h >= 60 && h < 842))) {
      double ai = 0, aq = 0;
      if (!O.wide || h + 12 <= 842) {
#pragma unroll
        for (int o = 0; o < 17; o++) {
          ai += (g_nrc.b[o] / 1.0) * s_i[h + 12 - o];
          aq += (g_nrc.b[o] / 1.0) * s_q[h + 12 - o];
        }
      }
      if (fabs(ai) > O.nr_c) ai = (ai > 0) ? O.nr_c : -O.nr_c;
      if (fabs(aq) > O.nr_c) aq = (aq > 0) ? O.nr_c : -O.nr_c;
      iv = s_i[h] - ai;
      qv = s_q[h] - aq;
    } else {
      iv = I_at(h);
      qv = Q_at(h);
    }
    iv *= kc;
    qv *= kc;
    double y = u16_to_ire_of(yv);
    y = (y - O.black_ire) * kb;
    const double q = +(iv) / IRESCALE;
    const double i = +(qv) / IRESCALE;
    double r = y + (.956 * i) + (.621 * q);
    double g = y - (.272 * i) - (.647 * q);
    double b = y - (1.106 * i) + (1.703 * q);
    r = clampd(r * m, 0, 65535);
    g = clampd(g * m, 0, 65535);
    b = clampd(b * m, 0, 65535);
    if (black) r = g = b = 0;                            // -l: the debug line (comb-ntsc.cxx:586-589)
    out[x * 3 + 0] = (uint16_t)r;
    out[x * 3 + 1] = (uint16_t)g;
    out[x * 3 + 2] = (uint16_t)b;
  }
}

extern "C" __global__ __launch_bounds__(256) void ldg_k_comb_out(const uint16_t* __restrict__ frames,
                                                                 const double* __restrict__ cvbuf,
                                                                 const double* __restrict__ iq,
                                                                 const double* __restrict__ abl,
                                                                 uint16_t* __restrict__ rgb) {
  comb_out_row(frames, cvbuf, iq, abl, rgb, CombDefaults{});
}
extern "C" __global__ __launch_bounds__(256) void ldg_k_comb_out_opt(const uint16_t* __restrict__ frames,
                                                                     const double* __restrict__ cvbuf,
                                                                     const double* __restrict__ iq,
                                                                     const double* __restrict__ abl,
                                                                     uint16_t* __restrict__ rgb, CombOpt O,
                                                                     const double* __restrict__ hist_in,
                                                                     double* __restrict__ hist_out, int n) {
  comb_out_row(frames, cvbuf, iq, abl, rgb, O, hist_in, hist_out, n);
}

// ---- ldg_k_comb_fused: the default 2D path (CombDefaults) in one row kernel:
// comb_split's Split1D / Split2D, comb_iq's FilterIQ chains and comb_out's
// AdjustY / DoYNR / ToRGB, with cv and the FilterIQ outputs kept in LDS
// instead of round-tripping through HBM (910 + 836 doubles per row).
// FilterIQ runs on waves 0 (I) and 1 (Q), IQC feeds per lane.  Like the
// burst-level EMA, the 1-pole chain forgets (|A1| = 0.547: a state difference
// shrinks by 0.547^k and, once below an ulp, the two runs round alike and stay
// equal), so lane j starts IQW feeds before its chunk from y = 0 (exact where
// that reaches feed 0) and its chunk is the sequential chain's iff its state
// entering the chunk equals lane j - 1's final state; any failed check reruns
// the whole chain on one lane.  Every arithmetic step is comb_iq's, so the
// output is bit-identical to the three-kernel path.  iqw: the exact warm-up from an
// affine-scan seed (28 feeds; LDG_COMB_IQW=0 forces the fallback in the tests).
// grid: n * OUT_H workgroups of 256 threads.
constexpr int IQC = 7;
// One row of the default 2D comb with its raw lines l-2, l, l+2 already in s_raw
// (ldg_k_comb_fused, ldg_k_comb_rows).  Ends with every thread's stores issued;
// s_raw, s_cv and s_buf may be rewritten after a __syncthreads.
__device__ __forceinline__ void comb_row_default(const uint16_t (*s_raw)[IN_X + 2], double* s_cv, double* s_buf,
                                                 int f, int row, double aburst, uint16_t* __restrict__ rgb, int iqw) {
  using O = CombDefaults;
  double* s_y = s_buf;                                   // [0, 834)
  double (*s_iq)[IQ_NS] = reinterpret_cast<double (*)[IQ_NS]>(s_buf + 840);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int l = row + O::firstline;
  KSTAMP(0, 2);
  // Split1D's clp0 of the three lines, formed where Split2D reads it (no staging pass)
  auto clp0 = [&](int k, int h) -> double {
    const int r = l - 2 + 2 * k;
    if (r < 44 || h < 4 || h >= 840) return 0.0;
    const int avg = ((int)s_raw[k][h + 2] + (int)s_raw[k][h - 2]) / 2;   // integer average (Split1D)
    return (double)(avg - (int)s_raw[k][h]);
  };
  const bool invertphase = (s_raw[1][0] == 16384);
  // (unrolled: the pixels' dependent clp1 chains -- three divisions each -- interleave)
#pragma unroll
  for (int u = 0; u < (CV_STRIDE + 255) / 256; u++) {
    const int h = tid + 256 * u;
    if (h >= CV_STRIDE) continue;
    double cv = 0.0;
    if (h >= 4 && h < 840) {
      double cavg = 0;
      cavg += 0.0 * 0.0;                                 // clpbuffer[2] * combk[2]
      const double c1h = clp0(1, h);
      if (h >= 18) {
        cavg += clp1_v(c1h, clp0(1, h - 1), clp0(0, h), clp0(0, h - 1), clp0(2, h), clp0(2, h - 1), P_2DRANGE, true) * 1.0;
        cavg += c1h * 0.0;
      } else {
        cavg += 0.0 * 0.0;
        cavg += c1h * 1.0;
      }
      cavg /= 2;
      if (!invertphase) cavg = -cavg;
      cv = cavg;
    }
    s_cv[h] = cv;
  }
  __syncthreads();
  KSTAMP(0, 3);
  const bool fiq = l >= 44;
  // AdjustY over h in [66, 834) (the span DoYNR's taps reach from the output pixels):
  // waves 2-3 while waves 0-1 run the FilterIQ chains (all four without them)
  {
    const int t0 = fiq ? tid - 128 : tid, nt = fiq ? 128 : 256;
    if (t0 >= 0) {
      for (int h = 66 + t0; h < 834; h += nt) {
        const int p = h + 2;
        const double yy = (p >= 4 && p < 840) ? (double)s_raw[1][p] : 0.0;
        const double ii = held_i(s_cv, p), qq = held_q(s_cv, p);
        double comp = 0;
        switch (h & 3) {
          case 0: comp = ii; break;
          case 1: comp = -qq; break;
          case 2: comp = -ii; break;
          default: comp = qq; break;
        }
        if (invertphase) comp = -comp;
        s_y[h] = yy + comp;
      }
    }
  }
  if (fiq && wv < 2) {
    // FilterIQ chain q = wv (comb_iq_lane's arithmetic, feed k from cv[6 + 2k + q])
    const int q = wv;
    auto xin = [&](int k) -> double {
      if (k < 0 || k >= IQ_NS - 1) return 0.0;
      const double v = s_cv[6 + 2 * k + q];
      return ((k & 1) != q) ? v : -v;
    };
    auto step = [&](double x, double x1, double y) {
      double ya = 0;
      ya += (LPI_B0 / 1.0) * x;
      ya += (LPI_B1 / 1.0) * x1;
      ya -= (LPI_A1 / 1.0) * y;
      return ya;
    };
    const int k0 = lane * IQC, k1 = (k0 + IQC < IQ_NS) ? k0 + IQC : IQ_NS;
    // the chunk's feeds, read once
    double xs[IQC];
#pragma unroll
    for (int u = 0; u < IQC; u++) xs[u] = (k0 + u < k1) ? xin(k0 + u) : 0.0;
    // Seed: the chunk maps y -> A y + B composed across the lanes (an affine scan) give
    // every chunk start's state to within rounding; from the seed iqw feeds back (whole
    // chunks) the exact steps run up to the chunk, and by then the seed's error has
    // shrunk by 0.547^iqw (iqw 28: ~5e-8 of an ulp), so the states agree bit for bit --
    // which the neighbour check below still verifies.
    const int wch = (iqw + IQC - 1) / IQC;               // warm-up in whole chunks
    const int kw = (lane - wch > 0) ? (lane - wch) * IQC : 0;
    double y = 0.0;
    {
      const double alpha = -(LPI_A1 / 1.0);
      double A = 1.0, B = 0.0, xp = xin(k0 - 1);
#pragma unroll
      for (int u = 0; u < IQC; u++) {
        if (k0 + u < k1) {
          double c = 0;
          c += (LPI_B0 / 1.0) * xs[u];
          c += (LPI_B1 / 1.0) * xp;
          A = alpha * A;
          B = alpha * B + c;
          xp = xs[u];
        }
      }
      // inclusive Kogge-Stone over the lanes: (A, B) = mine after theirs
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const double At = __shfl_up(A, o), Bt = __shfl_up(B, o);
        if (lane >= o) {
          B = A * Bt + B;
          A = A * At;
        }
      }
      // the state entering lane j's chunk is lane j-1's inclusive B (y_{-1} = 0); the
      // warm-up starts at lane (j - wch)'s chunk, entered with lane (j - wch - 1)'s B
      const int src = lane - wch - 1;
      const double seed = __shfl(B, src < 0 ? 0 : src);
      if (kw > 0) y = seed;
    }
    double x1 = xin(kw - 1);
    if (k0 < IQ_NS) {
      // 8 feeds read ahead of their steps: only the multiply-subtract on y is on the chain
      int k = kw;
#pragma unroll 1
      for (; k + 8 <= k0; k += 8) {
        double xw[8];
#pragma unroll
        for (int u = 0; u < 8; u++) xw[u] = xin(k + u);
#pragma unroll
        for (int u = 0; u < 8; u++) {
          y = step(xw[u], x1, y);
          x1 = xw[u];
        }
      }
      for (; k < k0; k++) {
        const double x = xin(k);
        y = step(x, x1, y);
        x1 = x;
      }
    }
    const double y_in = y;
    if (k0 < IQ_NS) {
#pragma unroll
      for (int u = 0; u < IQC; u++) {
        if (k0 + u < k1) {
          y = step(xs[u], x1, y);
          x1 = xs[u];
          s_iq[q][k0 + u] = y;
        }
      }
    }
    const long long prev = __shfl_up(__double_as_longlong(y), 1);
    const bool bad = lane > 0 && k0 < IQ_NS && kw > 0 && prev != __double_as_longlong(y_in);
    if (__ballot(bad) && lane == 0) {
      double yy = 0.0, xx1 = 0.0;
      for (int k = 0; k < IQ_NS; k++) {
        const double x = xin(k);
        yy = step(x, xx1, yy);
        xx1 = x;
        s_iq[q][k] = yy;
      }
    }
  }
  __syncthreads();
  KSTAMP(0, 4);
  // ---- DoYNR, ToRGB
  const double m = O::bright_m;
  const double kc = 10 / aburst, kb = 100 / (100 - O::black_ire);
  uint16_t* out = rgb + ((size_t)f * O::out_rows + row) * OUT_W * 3;
#pragma unroll
  for (int u = 0; u < (OUT_W + 255) / 256; u++) {
    const int x = tid + 256 * u;
    if (x >= OUT_W) continue;
    const int h = x + OUT_X0;
    double y0 = 0;
#pragma unroll
    for (int o = 0; o < 25; o++) y0 += (g_nr.b[o] / 1.0) * s_y[h + 12 - o];
    double a = y0;
    if (fabs(a) > O::nr_y) a = (a > 0) ? O::nr_y : -O::nr_y;
    const double yv = s_y[h] - a;
    double iv = (fiq && h >= 2 && h < 838) ? s_iq[0][(h - 2) >> 1] : held_i(s_cv, h + 2);
    double qv = (fiq && h >= 3 && h < 838) ? s_iq[1][(h - 3) >> 1] : (fiq && h == 2) ? 0.0 : held_q(s_cv, h + 2);
    iv *= kc;
    qv *= kc;
    double yi = u16_to_ire_of(yv);
    yi = (yi - O::black_ire) * kb;
    const double qq = +(iv) / IRESCALE;
    const double ii = +(qv) / IRESCALE;
    double r = yi + (.956 * ii) + (.621 * qq);
    double g = yi - (.272 * ii) - (.647 * qq);
    double b = yi - (1.106 * ii) + (1.703 * qq);
    r = clampd(r * m, 0, 65535);
    g = clampd(g * m, 0, 65535);
    b = clampd(b * m, 0, 65535);
    out[x * 3 + 0] = (uint16_t)r;
    out[x * 3 + 1] = (uint16_t)g;
    out[x * 3 + 2] = (uint16_t)b;
  }
  KSTAMP(0, 5);
}

extern "C" __global__ __launch_bounds__(256) void ldg_k_comb_fused(const uint16_t* __restrict__ frames,
                                                                   const double* __restrict__ abl,
                                                                   uint16_t* __restrict__ rgb, int iqw) {
  using O = CombDefaults;
  static_assert(O::firstline >= 36 && O::firstline + O::nrows <= IN_Y - 2 && !O::wide && O::nr_c <= 0 &&
                    O::colorlpf && !O::lpq && !O::bw,
                "the fused kernel covers comb-ntsc's default options only");
  static_assert(64 * IQC >= IQ_NS, "one chunk per lane");
  __shared__ uint16_t s_raw[3][IN_X + 2];                // raw lines l-2, l, l+2
  __shared__ double s_cv[CV_STRIDE];                     // SplitIQ's signed chroma
  // AdjustY's Y (h < 834) and the FilterIQ outputs (26.3 KiB of LDS in all: 6 workgroups per CU)
  __shared__ double s_buf[840 + 2 * IQ_NS];
  KSTAMP(0, 0);
  const int tid = threadIdx.x;
  const int f = blockIdx.x / O::nrows;
  const int row = blockIdx.x % O::nrows;
  const int l = row + O::firstline;
  const uint16_t* fr = frames + (size_t)f * IN_X * IN_Y;
  for (int t = tid; t < 3 * (IN_X / 2); t += 256) {
    const int k = t / (IN_X / 2), w = t % (IN_X / 2);
    const int r = l - 2 + 2 * k;
    const uint32_t v = reinterpret_cast<const uint32_t*>(fr + (size_t)r * IN_X)[w];
    s_raw[k][2 * w] = (uint16_t)(v & 0xffff);
    s_raw[k][2 * w + 1] = (uint16_t)(v >> 16);
  }
  __syncthreads();
  KSTAMP(0, 1);
  comb_row_default(s_raw, s_cv, s_buf, f, row, abl[(size_t)f * O::chain_lines() + (l - O::firstline)], rgb, iqw);
}

// ldg_k_comb_rows: the same rows from a persistent grid of G workgroups, row
// r = blockIdx.x + G i.  A row workgroup spends most of its life waiting on its
// three raw-line loads, and any resident comb wave keeps a demod workgroup off
// its CU; here the next row's lines (and its burst level) are loaded into
// registers while the current row is computed, so each CU the comb holds is
// busy computing.  grid: G x 256 (G <= rows).
constexpr int COMB_PRE = (3 * (IN_X / 2) + 255) / 256;   // raw 32-bit words per thread per row
extern "C" __global__ __launch_bounds__(256) void ldg_k_comb_rows(const uint16_t* __restrict__ frames,
                                                                  const double* __restrict__ abl,
                                                                  uint16_t* __restrict__ rgb, int iqw, int total) {
  using O = CombDefaults;
  __shared__ uint16_t s_raw[3][IN_X + 2];
  __shared__ double s_cv[CV_STRIDE];
  __shared__ double s_buf[840 + 2 * IQ_NS];
  const int tid = threadIdx.x;
  const int G = gridDim.x;
  uint32_t pre[COMB_PRE];
  double ab_pre = 0.0;
  auto fetch = [&](int r) {
    const int f = r / O::nrows, row = r % O::nrows, l = row + O::firstline;
    const uint16_t* fr = frames + (size_t)f * IN_X * IN_Y;
#pragma unroll
    for (int q = 0; q < COMB_PRE; q++) {
      const int t = tid + 256 * q;
      if (t < 3 * (IN_X / 2)) {
        const int k = t / (IN_X / 2), w = t % (IN_X / 2);
        pre[q] = reinterpret_cast<const uint32_t*>(fr + (size_t)(l - 2 + 2 * k) * IN_X)[w];
      }
    }
    ab_pre = abl[(size_t)f * O::chain_lines() + row];
  };
  int r = blockIdx.x;
  if (r < total) fetch(r);
  for (; r < total; r += G) {
#pragma unroll
    for (int q = 0; q < COMB_PRE; q++) {
      const int t = tid + 256 * q;
      if (t < 3 * (IN_X / 2)) {
        const int k = t / (IN_X / 2), w = t % (IN_X / 2);
        s_raw[k][2 * w] = (uint16_t)(pre[q] & 0xffff);
        s_raw[k][2 * w + 1] = (uint16_t)(pre[q] >> 16);
      }
    }
    const double aburst = ab_pre;
    __syncthreads();
    if (r + G < total) fetch(r + G);                     // in flight while this row is computed
    comb_row_default(s_raw, s_cv, s_buf, r / O::nrows, r % O::nrows, aburst, rgb, iqw);
    __syncthreads();                                     // s_raw / s_cv / s_buf free for the next row
  }
}
