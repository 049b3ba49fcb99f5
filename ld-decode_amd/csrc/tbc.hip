// Time-base correction: per-line spline resampling to 4fsc, NTSC colour-burst
// line refinement, final IRE -> uint16 .tbc lines, 48 kHz audio, frame assembly.
//
// Restates Field.downscale + lddutils.scale (lddecode_core.py:789-812,
// lddutils.py:83-97), FieldNTSC.refine_linelocs_burst / apply_offsets /
// downscale(final) (lddecode_core.py:1054-1162), FieldPAL.downscale(final)
// (:1023-1035), downscale_audio (:431-484) and Framer.formatoutput (:1238-1252).
//
// Spline: scipy splrep(s=0) on unit-spaced points is the not-a-knot cubic
// interpolant, solved in second-derivative form by one workgroup per line
// (spline_block): the line's samples in LDS, the tridiagonal solve as chunked
// affine scans.  The final pass solves the whole line on 256 threads; the
// burst pass (40 outputs per line) solves only the rows within KTR=40 samples
// of its outputs (exact to rho^40 ~ 1e-23 relative) on one wave.
#include <hip/hip_runtime.h>
#include "common.hpp"
#include "field_rec.hpp"
#include "pyops.hpp"
#include "chan.hpp"

using namespace ldg;

namespace {

constexpr int SPL_MAXN = 2816;                 // whole-line LDS solve up to this many points (NTSC ~2545, PAL ~2563)
// Longer lines (line locations around a damaged vsync can be 3000+ samples apart) are
// solved in windows (KTR margin) like the burst pass: any length up to SPL_HARDN.
constexpr int64_t SPL_HARDN = 1 << 24;
constexpr int LINE_GROUPS = (MAX_LINES + 63) / 64;

struct CTab { double v[17]; };
constexpr CTab make_ctab() {
  CTab t{};
  double c = 0.25;
  for (int i = 0; i < 17; i++) { t.v[i] = c; c = 1.0 / (4.0 - c); }
  return t;
}
__constant__ CTab g_ctab = make_ctab();        // Thomas c'_t for diag 4 / off-diag 1 (fixed point from t=14)
constexpr double kCtInf = make_ctab().v[16];    // c'_t for t >= 16
// Spline evaluation M/6 terms as products with 1/6 (the reference's splev is
// FITPACK's B-spline evaluation, so no formula reproduces its rounding; the
// .tbc values agree within the +-1 LSB bar either way)
constexpr double kSixth = 1.0 / 6.0;
__device__ __forceinline__ double ctab(int64_t t) { return g_ctab.v[t < 16 ? t : 16]; }

// Truncation margin of a windowed spline solve (the burst pass needs 40 of a
// line's outputs): the interior system (1,4,1) couples M_j to its neighbours
// with decay rho = 2 - sqrt(3) per sample, so cutting the system KTR rows
// beyond the needed range perturbs the result by < rho^KTR ~ 1.5e-23
// (relative) -- below double rounding.
constexpr int KTR = 40;
constexpr int64_t SCR_PER_SLOT = (int64_t)MAX_LINES * 64 + 3 * MAX_LINES;   // PAL pilot offsets (PILOT_MAX = 64) per slot

// Not-a-knot cubic spline through y[j] = buf[ib + j], j = 0..n (lddutils.scale:
// splrep(s=0) on unit spacing), evaluated at x_o = o*step + x0 (numpy
// linspace(begin-ib, end-ib, W+1) arithmetic).  Second-derivative form: the
// not-a-knot rows fold into M_1 = r_1/6 and M_{n-1} = r_{n-1}/6; rows 2..n-2
// are tridiagonal (1,4,1) with right-hand side r_j = 6 (y_{j+1} - 2 y_j + y_{j-1});
// M_0 = 2 M_1 - M_2, M_n = 2 M_{n-1} - M_{n-2}.
// spline_block: the interpolant on one workgroup of NT threads (NT = 64 * waves).
// Rows [lo, hi] around the requested outputs (the whole line for the final
// pass; KTR rows past the outputs otherwise, exactly as spline_window) are
// solved with the line's samples staged in LDS (one coalesced load) and the
// tridiagonal solve as chunked affine scans: thread i owns rows
// [i*CH, (i+1)*CH) (CH odd: conflict-free strided LDS access), composes its
// rows' maps, a workgroup Kogge-Stone scan gives each chunk its carry-in, and
// the thread re-runs its rows with the Thomas arithmetic (forward d_t = (r_t -
// d_{t-1}) c_t, backward M_t = d_t - c_t M_{t+1}) into ms.  Outputs
// o = o_lo + tid + NT q < o_hi: sink(o, value).  Returns -1 (uniform) where
// splrep would raise.
template <int NT, int CAP = SPL_MAXN + 1>
struct SplineLDS {
  static constexpr int cap = CAP;   // samples [base, top] of the solved window
  double ys[CAP];
  double ms[CAP];
  double ct[17];
  double ra[NT / 16], rb[NT / 16];
  double m1, mn1;
  double ye[6];                     // y[0..2], y[n-2..n] (the not-a-knot end rows)
};

// Composition of affine maps x -> A x + B over the workgroup's threads in order
// (SUFFIX: in reverse order); returns the carry-in of this thread's chunk, i.e.
// the composition of all earlier (later) chunks applied to 0.  Inside each row
// of 16 lanes a Kogge-Stone scan by DPP row shifts (no LDS round trip), the
// row totals through LDS, then each thread folds the rows before (after) its own.
template <int CTRL>
__device__ __forceinline__ double dpp_f64_or(double x, double ident) {
  const int lo = __builtin_amdgcn_update_dpp(__double2loint(ident), __double2loint(x), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(__double2hiint(ident), __double2hiint(x), CTRL, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}
template <bool SUFFIX, int CTRL>
__device__ __forceinline__ void affine_row_step(double& A, double& B) {
  const double pa = dpp_f64_or<CTRL>(A, 1.0), pb = dpp_f64_or<CTRL>(B, 0.0);
  B = A * pb + B;
  A = A * pa;
}
template <int NT, bool SUFFIX, class SL>
__device__ __forceinline__ double block_affine_carry(double A, double B, int tid, SL& S) {
  static_assert(NT / 16 <= 16, "row totals");
  constexpr int NR = NT / 16;
  const int row = tid >> 4, li = tid & 15;
  // inclusive within the row: prefix from lanes below (row_shr), suffix from above (row_shl)
  affine_row_step<SUFFIX, SUFFIX ? 0x101 : 0x111>(A, B);
  affine_row_step<SUFFIX, SUFFIX ? 0x102 : 0x112>(A, B);
  affine_row_step<SUFFIX, SUFFIX ? 0x104 : 0x114>(A, B);
  affine_row_step<SUFFIX, SUFFIX ? 0x108 : 0x118>(A, B);
  if (li == (SUFFIX ? 0 : 15)) { S.ra[row] = A; S.rb[row] = B; }
  // exclusive within the row: the neighbour's inclusive value (identity at the row end)
  const double exA = dpp_f64_or<SUFFIX ? 0x101 : 0x111>(A, 1.0);
  const double exB = dpp_f64_or<SUFFIX ? 0x101 : 0x111>(B, 0.0);
  __syncthreads();
  double rb = 0.0;
  if constexpr (NR <= 4) {
    if (SUFFIX) {
      for (int r = NR - 1; r > row; r--) rb = S.ra[r] * rb + S.rb[r];
    } else {
      for (int r = 0; r < row; r++) rb = S.ra[r] * rb + S.rb[r];
    }
  } else {
    // the row totals' carries by a Kogge-Stone on wave 0 (one dependent step per doubling
    // instead of one per earlier row), written back over S.rb
    if (tid < 64) {
      double a = 1.0, b = 0.0;
      if (tid < NR) { a = S.ra[tid]; b = S.rb[tid]; }
#pragma unroll
      for (int o = 1; o < NR; o <<= 1) {
        const double at = SUFFIX ? __shfl_down(a, o) : __shfl_up(a, o);
        const double bt = SUFFIX ? __shfl_down(b, o) : __shfl_up(b, o);
        if (SUFFIX ? (tid + o < NR) : (tid >= o)) {
          b = a * bt + b;
          a = a * at;
        }
      }
      // exclusive: the neighbouring row's inclusive value (0 at the end)
      const double ex = SUFFIX ? __shfl_down(b, 1) : __shfl_up(b, 1);
      if (tid < NR) S.rb[tid] = (SUFFIX ? (tid == NR - 1) : (tid == 0)) ? 0.0 : ex;
    }
    __syncthreads();
    rb = S.rb[row];
  }
  __syncthreads();
  return exA * rb + exB;
}

template <int NT, int STK = -1, bool PRELOADED = false, class Src, class SL, class Sink>
__device__ int spline_block(const Src& buf, int64_t len, double begin, double end, int W, int o_lo,
                            int o_hi, int tid, SL& S, Sink&& sink) {
  if constexpr (STK >= 0) KSTAMP(STK, 0);
  if (tid < 17) S.ct[tid] = g_ctab.v[tid];
  const int64_t ib = py_int(begin), ie = py_int(end);
  const int64_t n64 = ie - ib;
  if (ib < 0 || n64 < 6 || n64 >= SPL_HARDN || ib + n64 + 1 > len) return -1;
  const int n = (int)n64;
  const double x0 = begin - (double)ib;
  const double span = end - begin;
  const double step = ((span + x0) - x0) / (double)W;
  auto xo = [&](int o) { double x = (double)o * step; return x + x0; };
  auto ival = [&](double x) {
    int64_t j = (int64_t)floor(x);
    return (int)(j < 0 ? 0 : (j > n - 1 ? n - 1 : j));
  };
  const int jlo = ival(xo(o_lo)), jhi = ival(xo(o_hi - 1));
  const int lo = (jlo - KTR > 2) ? jlo - KTR : 2;
  const int hi = (jhi + 1 + KTR < n - 2) ? jhi + 1 + KTR : n - 2;
  const int base = (lo - 1 < jlo) ? lo - 1 : jlo;            // ys / ms hold j in [base, top]
  const int top = (hi + 1 > jhi + 1) ? hi + 1 : jhi + 1;
  if (top - base + 1 > SL::cap) return -2;                    // window larger than the LDS (callers size it)
  double* ys = S.ys - base;
  double* ms = S.ms - base;
  if constexpr (PRELOADED) {
    // the caller staged y[0..n] in S.ys (base == 0 for a whole-line solve)
    __syncthreads();
    if (tid == 0) {
      S.m1 = (6.0 * ((ys[2] - ys[1]) - (ys[1] - ys[0]))) / 6.0;
      S.mn1 = (6.0 * ((ys[n] - ys[n - 1]) - (ys[n - 1] - ys[n - 2]))) / 6.0;
    }
  } else {
    buf.window(ib + base, ib + top, ys + base, tid, NT);   // ys[j] = y[j], j in [base, top]
    if (tid < 6) S.ye[tid] = buf[ib + (tid < 3 ? tid : n - 5 + tid)];
  }
  __syncthreads();
  if constexpr (STK >= 0) KSTAMP(STK, 1);
  const double* ye = S.ye;
  const double M1 = PRELOADED ? S.m1 : (6.0 * ((ye[2] - ye[1]) - (ye[1] - ye[0]))) / 6.0;
  const double Mn1 = PRELOADED ? S.mn1 : (6.0 * ((ye[5] - ye[4]) - (ye[4] - ye[3]))) / 6.0;
  const double BL = (lo == 2) ? M1 : 0.0, BR = (hi == n - 2) ? Mn1 : 0.0;
  const int T = hi - lo + 1;                                  // rows j = lo + t
  int CH = (T + NT - 1) / NT;
  CH |= 1;
  const int t0 = tid * CH;
  const int nq = ((t0 + CH < T) ? t0 + CH : T) - t0;         // this thread's rows (may be <= 0)
  auto ct = [&](int t) { return S.ct[t < 16 ? t : 16]; };
  // the thread's right-hand sides and Thomas coefficients, all loaded up front
  // (CHMAX >= CH: the loops are unrolled and predicated, so the LDS reads issue together)
  constexpr int CHMAX = ((SL::cap + NT - 1) / NT) | 1;
  double rr[CHMAX], cc[CHMAX], dd[CHMAX];
#pragma unroll
  for (int q = 0; q < CHMAX; q++) {
    if (q < nq) {
      const int t = t0 + q, j = lo + t;
      double r = 6.0 * ((ys[j + 1] - ys[j]) - (ys[j] - ys[j - 1]));
      if (t == 0) r -= BL;
      if (t == T - 1) r -= BR;
      rr[q] = r;
      cc[q] = ct(t);
    }
  }
  // forward sweep: d -> -c d + c r
  double A = 1.0, B = 0.0;
#pragma unroll
  for (int q = 0; q < CHMAX; q++) {
    if (q < nq) {
      const double c = cc[q];
      A = -c * A;
      B = (rr[q] - B) * c;
    }
  }
  double dprev = block_affine_carry<NT, false>(A, B, tid, S);
  if constexpr (STK >= 0) KSTAMP(STK, 2);
#pragma unroll
  for (int q = 0; q < CHMAX; q++) {
    if (q < nq) {
      const double d = (rr[q] - dprev) * cc[q];
      dd[q] = d;
      dprev = d;
    }
  }
  // back substitution: M -> d - c M, top down
  A = 1.0; B = 0.0;
#pragma unroll
  for (int q = CHMAX - 1; q >= 0; q--) {
    if (q < nq) {
      const double c = cc[q];
      A = -c * A;
      B = dd[q] - c * B;
    }
  }
  if constexpr (STK >= 0) KSTAMP(STK, 3);
  double Mnext = block_affine_carry<NT, true>(A, B, tid, S);
  if constexpr (STK >= 0) KSTAMP(STK, 4);
#pragma unroll
  for (int q = CHMAX - 1; q >= 0; q--) {
    if (q < nq) {
      const double M = dd[q] - cc[q] * Mnext;
      ms[lo + t0 + q] = M;
      Mnext = M;
    }
  }
  __syncthreads();
  if (tid == 0) {
    if (lo == 2) { ms[1] = M1; if (base == 0) ms[0] = 2.0 * M1 - ms[2]; }
    if (hi == n - 2) { ms[n - 1] = Mn1; if (top == n) ms[n] = 2.0 * Mn1 - ms[n - 2]; }
  }
  __syncthreads();
  if constexpr (STK >= 0) KSTAMP(STK, 5);
  for (int o = o_lo + tid; o < o_hi; o += NT) {
    const double x = xo(o);
    const int k = ival(x);
    const double Mk = ms[k], Mk1 = ms[k + 1], yk = ys[k], yk1 = ys[k + 1];
    const double a = (double)(k + 1) - x, b = x - (double)k;
    const double m6 = Mk * kSixth, m16 = Mk1 * kSixth;
    const double v = m6 * a * a * a + m16 * b * b * b + (yk - m6) * a + (yk1 - m16) * b;
    sink(o, v);
  }
  if constexpr (STK >= 0) KSTAMP(STK, 6);
  return 0;
}

__device__ inline int calczc_s(const double* d, int len, int s, double target, int count, int st, double* res) {
  const bool rising = d[s * st] < target;
  const int hi = (s + count + 1 < len) ? s + count + 1 : len;
  int hit = -1;
  for (int k = s; k < hi; k++) {
    const double v = d[k * st];
    if (rising ? (v >= target) : (v <= target)) { hit = k - s; break; }
  }
  if (hit < 0) return 1;
  const int x = s + hit;
  if (x == 0) return 1;
  const double a = d[(x - 1) * st] - target, b = d[x * st] - target;
  *res = (double)(x - 1) + ((-a) / ((-a) + b));
  return 0;
}

}  // namespace

// ---------------------------------------------------------------------------
// Burst pass, per (read, line): resample demod_burst over [li[l], li[l+1]] to
// 4fsc pixels 20..59 (lineoffset 0, wow-scaled), then the per-line part of
// refine_linelocs_burst (lddecode_core.py:1069-1110).
// grid: (lines per read, n_reads) workgroups of 64 threads, one line each.
extern "C" __global__ __launch_bounds__(64) void ldg_k_burst_lines(
    const int32_t* __restrict__ smap, const double* __restrict__ video, int64_t vread_stride, int64_t vchan_stride, SysConst C,
    FieldRec* __restrict__ recs, double* __restrict__ lines, float* __restrict__ blevel, int pass,
    const double4* __restrict__ bst, const ReadDesc* __restrict__ reads) {
  prio_latency();

  // window rows for 40 outputs: <= 40 * SPL_MAXN / W + 2 * KTR + 4 < 384
  __shared__ SplineLDS<64, 384> S;
  __shared__ double s_ba[40], s_t[40], s_g[2][40];
  const int lane = threadIdx.x;
  const int slot = smap[blockIdx.y];
  const int l = blockIdx.x;
  FieldRec* R = recs + slot;
  double* LN = lines + (int64_t)slot * LINES_STRIDE;
  const double* li = LN + (pass == 0 ? LL2 : LL3) * MAX_LINES;
  // the record and the line's two locations in one memory round trip (clamped indices)
  const int status = R->status, nl = R->nlines, lc = R->linecount;
  const double b0 = li[l], b1 = li[l + 1 < MAX_LINES ? l + 1 : MAX_LINES - 1];
  asm volatile("" ::"v"(b0), "v"(b1), "v"(status), "v"(nl), "v"(lc));
  if (status != FS_PENDING) return;
  double* pv0 = LN + PAVG0 * MAX_LINES;
  double* pv1 = LN + PAVG1 * MAX_LINES;
  float* lvl = blevel + (int64_t)slot * MAX_LINES;
  if (l >= nl) return;
  if (l >= lc) {
    if (lane == 0) { pv0[l] = 0.0; pv1[l] = 0.0; lvl[l] = 0.0f; }
    return;
  }
  if (py_int(b1) + 1 >= reads[slot].vcut) {   // the window reaches past the read's video cut
    if (lane == 0) R->status = FS_VCUT;
    return;
  }
  // demod_burst from the demod channel and the demod's per-chunk states (chan.hpp)
  const BurstSrc bur(bst, video + (int64_t)slot * vread_stride + (int64_t)CH_DEMOD * vchan_stride, slot, C);
  const double wow = (b1 - b0) / (double)C.linelen;
  const int W = C.outlinelen;
  const int rc = spline_block<64, 4>(bur, R->n_out, b0, b1, W, 20, 60, lane, S,
                                  [&](int o, double v) { s_ba[o - 20] = v * wow; });
  if (rc < 0) {
    if (lane == 0) R->status = FS_TBC;   // benign race: every writer stores the same value
    return;
  }
  __syncthreads();
  // the burst statistics on the whole wave (numpy's pairwise sums via wave_pw_block)
  double* ba = s_ba;
  double* tt = s_t;
  const double hzs = 1700000 / 140.0;
  const double m = (0.0 + wave_pw_block(ba, 40, lane)) / 40.0;
  double v = 0.0, amx = 0.0;
  if (lane < 40) { v = ba[lane] - m; amx = fabs(v); }
  for (int o = 32; o > 0; o >>= 1) amx = fmax(amx, __shfl_xor(amx, o));   // fmax drops NaNs, as the loop did
  const double mx = fmax(0.0, amx);
  __syncthreads();
  if (lane < 40) ba[lane] = v;
  __syncthreads();
  const float lf = (float)mx;
  const double lv = (double)lf;               // numpy-1: float32 element promoted to float64
  // np.std(ba)
  const double m2 = (0.0 + wave_pw_block(ba, 40, lane)) / 40.0;
  if (lane < 40) { const double d = ba[lane] - m2; tt[lane] = d * d; }
  __syncthreads();
  const double sd = sqrt((0.0 + wave_pw_block(tt, 40, lane)) / 40.0);
  // the zero-crossing walk (lddecode_core.py:1089-1104): every start position's
  // crossing (calczc over <= 11 samples) on its own lane; the walk from 0 visits
  // the first qualifying position at or after the previous one's int(zc) + 1,
  // so it reduces to bit scans over the qualifying mask (v_readlane for the jumps)
  bool qual = false;
  double zc = 0.0;
  if (lane < 40 && fabs(ba[lane]) > lv * .6) qual = calczc_s(ba, 40, lane, 0.0, 10, 1, &zc) == 0;
  const bool pos = lane < 40 && ba[lane] > 0;
  double off = 0.0;
  if (qual) {
    off = zc - ((floor(zc / 4) * 4) - 1);
    if (off > 3.5) off -= 4;
  }
  const uint64_t Q = __ballot(qual), P = __ballot(qual && pos);
  const int jt = qual ? (int)zc + 1 : 0;
  uint64_t V = 0;
  for (int x = 0; x < 40;) {
    const uint64_t m = Q & (~0ull << x);
    if (!m) break;
    const int q = __ffsll((unsigned long long)m) - 1;
    V |= 1ull << q;
    x = __builtin_amdgcn_readlane(jt, q);
  }
  const uint64_t VT = V & P, VF = V & ~P;
  const int nT = __popcll(VT), nF = __popcll(VF);
  // each group's offsets in visiting (= position) order
  const uint64_t below = (1ull << lane) - 1;
  if ((VT >> lane) & 1) s_g[1][__popcll(VT & below)] = off;
  if ((VF >> lane) & 1) s_g[0][__popcll(VF & below)] = off;
  __syncthreads();
  if (lane != 0) return;
  double p0 = 0.0, p1 = 0.0;
  float out_level = lf;
  if (((lv / hzs) > 30) || (sd / hzs) < 3) {
    out_level = 0.0f;
  } else if (!(nF < 3 || nT < 3)) {
    // mean of each group's [1:-1] (np.array of the list, pairwise sum)
    const double mF = pw_sum(s_g[0] + 1, nF - 2) / (double)(nF - 2);
    const double mT = pw_sum(s_g[1] + 1, nT - 2) / (double)(nT - 2);
    if (l % 2) { p0 = 2 - mT; p1 = 2 - mF; }
    else { p0 = 2 - mF; p1 = 2 - mT; }
  }
  lvl[l] = out_level;
  pv0[l] = p0;
  pv1[l] = p1;
#ifdef LDG_STAMPS
  if (blockIdx.x < KST_BLOCKS) g_kst[4][blockIdx.x][7] = __builtin_readcyclecounter();
#endif
}

// Per-read part of refine_linelocs_burst (lddecode_core.py:1112-1133) and, on
// the second pass, apply_offsets (:1161-1162, 1184-1186).  grid: n_reads x 64.
extern "C" __global__ __launch_bounds__(64) void ldg_k_burst_field(const int32_t* __restrict__ smap,
                                                                   FieldRec* __restrict__ recs,
                                                                   double* __restrict__ lines,
                                                                   float* __restrict__ blevel, SysConst C,
                                                                   int pass) {
  prio_latency();

  __shared__ double s_c0[512], s_c1[512];
  __shared__ int s_hist[256];
  __shared__ double s_lo[MAX_LINES];
  __shared__ float s_lvl[MAX_LINES];
  __shared__ int s_g;
  const int lane = threadIdx.x;
  const int slot = smap[blockIdx.x];
  FieldRec* R = recs + slot;
  if (R->status != FS_PENDING) return;
  const int nl = R->nlines;
  double* LN = lines + (int64_t)slot * LINES_STRIDE;
  const double* li = LN + (pass == 0 ? LL2 : LL3) * MAX_LINES;
  double* lo = LN + (pass == 0 ? LL3 : LL4) * MAX_LINES;
  const double* pv0 = LN + PAVG0 * MAX_LINES;
  const double* pv1 = LN + PAVG1 * MAX_LINES;
  float* lvl = blevel + (int64_t)slot * MAX_LINES;
  KSTAMP(2, 0);
  // phaseaverages_cut: rows with a nonzero entry (NaN counts as nonzero), in
  // order -- a ballot compaction -- then np.median of each column (wave bitonic sort)
  int nc = 0;
  for (int l0 = 0; l0 < nl; l0 += 64) {
    const int l = l0 + lane;
    double a0 = 0.0, a1 = 0.0;
    bool p = false;
    if (l < nl) { a0 = pv0[l]; a1 = pv1[l]; p = (a0 != 0 || a1 != 0); }
    const uint64_t m = __ballot(p);
    if (p) {
      const int pos = nc + __popcll(m & ((1ull << lane) - 1));
      s_c0[pos] = a0;
      s_c1[pos] = a1;
    }
    nc += __popcll(m);
  }
  __syncthreads();
  bool nan0 = false, nan1 = false;
  for (int k = lane; k < nc; k += 64) { nan0 |= s_c0[k] != s_c0[k]; nan1 |= s_c1[k] != s_c1[k]; }
  nan0 = __any(nan0);
  nan1 = __any(nan1);
  KSTAMP(2, 1);
  // np.median of each column (NaN if the column has one), by radix select
  const double m0 = (nan0 || nc == 0) ? __builtin_nan("") : wave_median(s_c0, nc, lane, s_hist);
  const double m1 = (nan1 || nc == 0) ? __builtin_nan("") : wave_median(s_c1, nc, lane, s_hist);
  KSTAMP(2, 2);
  if (lane == 0) s_g = (fabs(m0) < fabs(m1)) ? 0 : 1;
  __syncthreads();
  const int g = s_g;
  const double* adj = g ? pv1 : pv0;
  const double K = C.freq / ((4.0 * 315.0) / 88.0);
  // the group's lines flip their level sign; a phase adjustment beyond 2 samples
  // zeroes the level, otherwise it moves the line (lddecode_core.py:1120-1127)
  for (int l = lane; l < nl; l += 64) {
    float lv = lvl[l];
    if ((l & 1) == g) lv = -lv;
    double v = li[l];
    const double a = adj[l];
    if (fabs(a) > 2) lv = 0.0f;
    else v -= a * K * 1;
    s_lo[l] = v;
    s_lvl[l] = lv;
  }
  __syncthreads();
  // lines with no burst take the mean of their neighbours, in line order (a
  // line's left neighbour may itself have just been replaced): lane 0 visits
  // only those lines, found by ballot
  for (int l0 = 2; l0 < nl - 1; l0 += 64) {
    const int l = l0 + lane;
    const uint64_t m = __ballot(l < nl - 1 && s_lvl[l] == 0.0f);
    if (lane == 0) {
      uint64_t mm = m;
      while (mm) {
        const int j = l0 + __ffsll((unsigned long long)mm) - 1;
        mm &= mm - 1;
        s_lo[j] = (s_lo[j - 1] + s_lo[j + 1]) / 2;
      }
    }
    __syncthreads();
  }
  const double shift = (90 + 1.5) * (3.141592653589793 / 180);
  const double c = (shift - 8) * K;
  double* lf = LN + LLF * MAX_LINES;
  for (int l = lane; l < nl; l += 64) {
    lo[l] = s_lo[l];
    lvl[l] = s_lvl[l];
    if (pass == 1) lf[l] = (s_lo[l] + 0) + c;
  }
  if (lane == 0) R->burst_group = g;
#ifdef LDG_STAMPS
  if (blockIdx.x < KST_BLOCKS) g_kst[2][blockIdx.x][3] = __builtin_readcyclecounter();
#endif
}

// Final resample of 'demod' (lineoffset 1 NTSC / 3 PAL, wow) to uint16 .tbc
// lines (lddecode_core.py:1135-1159 NTSC, :1023-1035 PAL): the whole-line
// not-a-knot spline of spline_block, with the samples read from the demod
// channel in HBM / L2 (each thread its own rows into registers, the
// evaluation's two knots per output straight from the channel) and only the
// second derivatives in LDS.  ~25 KiB of LDS per workgroup, so a final-pass
// workgroup fits beside a demod workgroup (128 KiB) on one CU.
// grid: (rows per read, n_reads) workgroups of FINAL_NT threads, one line each.
constexpr int FINAL_NT = 256;
constexpr int FINAL_CHMAX = ((SPL_MAXN + FINAL_NT - 1) / FINAL_NT) | 1;   // rows per thread, upper bound
struct FinalLDS {
  double ms[SPL_MAXN + 1];
  double ct[17];
  double ra[FINAL_NT / 16], rb[FINAL_NT / 16];
  double m1, mn1;
};
// the windowed solve of lines with n >= SPL_MAXN points (shares FinalLDS's memory)
constexpr int FINAL_WCAP = 1280;
using FinalWinLDS = SplineLDS<FINAL_NT, FINAL_WCAP>;
static_assert(sizeof(FinalWinLDS) <= sizeof(FinalLDS), "long-line window must fit the final pass's LDS");

// the demod channel as a spline_block source
struct ChanSrc {
  const double* p;
  __device__ double operator[](int64_t i) const { return p[i]; }
  __device__ void window(int64_t n0, int64_t n1, double* dst, int tid, int nt) const {
    for (int64_t i = n0 + tid; i <= n1; i += nt) dst[i - n0] = p[i];
  }
};

// .tbc pixel of one resampled value (lddecode_core.py:1139-1142 NTSC, :1030-1035 PAL)
__device__ __forceinline__ uint16_t tbc_pixel(double v, double wow, const SysConst& C) {
  const bool pal = C.system == 1;
  const double scale_ = pal ? (double)(0xd300 - 0x0100) / (100 - C.vsync_ire)
                            : (double)(0xc800 - 0x0400) / (100 - C.vsync_ire);
  const double base = pal ? 256.0 : 1024.0;
  double red = ((v * wow) - C.ire0) / C.hz_ire;           // the reference divides (:1139)
  red -= C.vsync_ire;
  double px = (red * scale_) + base;
  if (px != px) px = 0.0;
  px = fmin(fmax(px, 0.0), 65535.0) + 0.5;
  return (uint16_t)px;
}
#ifndef LDG_FINAL_WAVES
#define LDG_FINAL_WAVES 6
#endif
// (6 waves per SIMD: 78 VGPRs, six line workgroups per CU, 138 KiB of LDS)
// HOIST: the evaluation's two knot samples per output are loaded together with the
// solve's samples (one memory round trip per line instead of two, for more VGPRs)
template <bool HOIST>
__device__ __forceinline__ void final_lines_impl(
    const int32_t* __restrict__ smap, const double* __restrict__ video, int64_t vread_stride, int64_t vchan_stride,
    SysConst C, FieldRec* __restrict__ recs, const double* __restrict__ lines, const float* __restrict__ blevel,
    uint16_t* __restrict__ pic, int64_t pic_stride, const ReadDesc* __restrict__ reads) {
  prio_latency();
  __shared__ union {
    FinalLDS S;
    FinalWinLDS Wn;
  } U;
  FinalLDS& S = U.S;
  const int tid = threadIdx.x;
  const int slot = smap[blockIdx.y];
  const int row = blockIdx.x;
  FieldRec* R = recs + slot;
  const int loff = (C.system == 1) ? 3 : 1;
  const int l = row + loff;
  const double* lf = lines + (int64_t)slot * LINES_STRIDE + LLF * MAX_LINES;
  // the record and the line's two locations in one memory round trip (the locations
  // are read before the record says the row is live: indices clamped into the array)
  const int status = R->status, lc = R->linecount;
  const int64_t len = R->n_out;
  const double begin = lf[l < MAX_LINES ? l : MAX_LINES - 1], end = lf[l + 1 < MAX_LINES ? l + 1 : MAX_LINES - 1];
  asm volatile("" ::"v"(begin), "v"(end), "v"(status), "v"(lc));
  if (status != FS_PENDING) return;
  if (row >= lc) return;
  const double* dm = video + (int64_t)slot * vread_stride + (int64_t)CH_DEMOD * vchan_stride;
  const int W = C.outlinelen;
  uint16_t* out = pic + (int64_t)slot * pic_stride + (int64_t)row * W;
  // ---- geometry (spline_block): y[j] = dm[ib + j], j = 0..n
  const int64_t ib = py_int(begin), ie = py_int(end);
  const int64_t n64 = ie - ib;
  if (ib < 0 || n64 < 6 || n64 >= SPL_HARDN || ib + n64 + 1 > len) {
    if (tid == 0) R->status = FS_TBC;
    return;
  }
  if (ib + n64 + 1 >= reads[slot].vcut) {     // samples past the read's video cut: decode it in full
    if (tid == 0) R->status = FS_VCUT;
    return;
  }
  const bool pal = C.system == 1;
  if (n64 >= SPL_MAXN) {
    // a long line: windowed solves over chunks of outputs, each within FINAL_WCAP rows
    const double wow = (end - begin) / (double)C.linelen;
    const int64_t oc64 = ((int64_t)(FINAL_WCAP - 2 * KTR - 16) * W) / n64;
    const int oc = oc64 < 1 ? 1 : (int)oc64;
    for (int o0 = 0; o0 < W; o0 += oc) {
      const int o1 = o0 + oc < W ? o0 + oc : W;
      const int rc = spline_block<FINAL_NT>(ChanSrc{dm}, len, begin, end, W, o0, o1, tid, U.Wn,
                                            [&](int o, double v) { out[o] = tbc_pixel(v, wow, C); });
      if (rc < 0) {
        if (tid == 0) R->status = FS_TBC;
        return;
      }
      __syncthreads();
    }
    __syncthreads();
    if (!pal && tid < 2 && row >= 1 && row < lc - 1) {
      const float bl = blevel[(int64_t)slot * MAX_LINES + row];
      const double hzs = 1700000 / 140.0;
      if (tid == 0) out[0] = bl > 0 ? 16384 : 32768;
      const double clevel = (1 / 1.45) / hzs;
      if (tid == 1) out[1] = (uint16_t)(327.67 * clevel * fabs((double)bl));
    }
    return;
  }
  const int n = (int)n64;
  const double* y = dm + ib;
  KSTAMP(1, 0);
  if (tid < 17) S.ct[tid] = g_ctab.v[tid];
  if (tid == 0) {
    S.m1 = (6.0 * ((y[2] - y[1]) - (y[1] - y[0]))) / 6.0;
    S.mn1 = (6.0 * ((y[n] - y[n - 1]) - (y[n - 1] - y[n - 2]))) / 6.0;
  }
  // rows j = lo + t, t < T (lo = 2, hi = n - 2: the whole line)
  constexpr int lo = 2;
  const int T = n - 3;
  int CH = (T + FINAL_NT - 1) / FINAL_NT;
  CH |= 1;
  const int t0 = tid * CH;
  const int nq = ((t0 + CH < T) ? t0 + CH : T) - t0;
  // this thread's samples y[lo + t0 - 1 .. lo + t0 + nq], loads issued together
  double yv[FINAL_CHMAX + 2];
#pragma unroll
  for (int q = 0; q < FINAL_CHMAX + 2; q++) yv[q] = (q < nq + 2) ? y[lo + t0 - 1 + q] : 0.0;
  // ---- evaluation geometry: linspace(b - ib, (e - b) + (b - ib), W + 1)[:-1]
  const double x0 = begin - (double)ib;
  const double span = end - begin;
  const double step = ((span + x0) - x0) / (double)W;
  constexpr int NO = (MAX_OUTW + FINAL_NT - 1) / FINAL_NT;
  auto knot = [&](int e) {
    const int o = tid + FINAL_NT * e;
    double x = (double)o * step;
    x = x + x0;
    int64_t j = (int64_t)floor(x);
    return (int)(j < 0 ? 0 : (j > n - 1 ? n - 1 : j));
  };
  double yk[NO], yk1[NO];
  if constexpr (HOIST) {
#pragma unroll
    for (int e = 0; e < NO; e++) {
      const int o = tid + FINAL_NT * e, k = knot(e);
      yk[e] = (o < W) ? y[k] : 0.0;
      yk1[e] = (o < W) ? y[k + 1] : 0.0;
    }
  }
  __syncthreads();
  KSTAMP(1, 1);
  const double M1 = S.m1, Mn1 = S.mn1;
  const double BL = M1, BR = Mn1;
  auto ct = [&](int t) { return t < 16 ? S.ct[t] : kCtInf; };
  // (the Thomas coefficient c_t is re-read where used: it is constant past t = 16,
  // and holding it per row would cost 22 VGPRs -- a wave per SIMD of occupancy)
  double rr[FINAL_CHMAX], dd[FINAL_CHMAX];
#pragma unroll
  for (int q = 0; q < FINAL_CHMAX; q++) {
    if (q < nq) {
      const int t = t0 + q;
      double r = 6.0 * ((yv[q + 2] - yv[q + 1]) - (yv[q + 1] - yv[q]));
      if (t == 0) r -= BL;
      if (t == T - 1) r -= BR;
      rr[q] = r;
    }
  }
  auto cc = [&](int q) { return ct(t0 + q); };
  // forward sweep: d -> -c d + c r
  double A = 1.0, B = 0.0;
#pragma unroll
  for (int q = 0; q < FINAL_CHMAX; q++) {
    if (q < nq) {
      const double c = cc(q);
      A = -c * A;
      B = (rr[q] - B) * c;
    }
  }
  double dprev = block_affine_carry<FINAL_NT, false>(A, B, tid, S);
  KSTAMP(1, 2);
#pragma unroll
  for (int q = 0; q < FINAL_CHMAX; q++) {
    if (q < nq) {
      const double d = (rr[q] - dprev) * cc(q);
      dd[q] = d;
      dprev = d;
    }
  }
  // back substitution: M -> d - c M, top down
  A = 1.0; B = 0.0;
#pragma unroll
  for (int q = FINAL_CHMAX - 1; q >= 0; q--) {
    if (q < nq) {
      const double c = cc(q);
      A = -c * A;
      B = dd[q] - c * B;
    }
  }
  double Mnext = block_affine_carry<FINAL_NT, true>(A, B, tid, S);
  KSTAMP(1, 3);
  double* ms = S.ms;
#pragma unroll
  for (int q = FINAL_CHMAX - 1; q >= 0; q--) {
    if (q < nq) {
      const double M = dd[q] - cc(q) * Mnext;
      ms[lo + t0 + q] = M;
      Mnext = M;
    }
  }
  __syncthreads();
  if (tid == 0) {
    ms[1] = M1;
    ms[0] = 2.0 * M1 - ms[2];
    ms[n - 1] = Mn1;
    ms[n] = 2.0 * Mn1 - ms[n - 2];
  }
  __syncthreads();
  KSTAMP(1, 4);
  // ---- evaluation at W points
  const double wow = (end - begin) / (double)C.linelen;
  int kk[NO];
  double xs[NO];
#pragma unroll
  for (int e = 0; e < NO; e++) {
    const int o = tid + FINAL_NT * e;
    double x = (double)o * step;
    x = x + x0;
    const int k = knot(e);
    kk[e] = k;
    xs[e] = x;
    if constexpr (!HOIST) {
      yk[e] = (o < W) ? y[k] : 0.0;
      yk1[e] = (o < W) ? y[k + 1] : 0.0;
    }
  }
#pragma unroll
  for (int e = 0; e < NO; e++) {
    const int o = tid + FINAL_NT * e;
    if (o >= W) continue;
    const double x = xs[e];
    const int k = kk[e];
    const double Mk = ms[k], Mk1 = ms[k + 1];
    const double a = (double)(k + 1) - x, b = x - (double)k;
    const double m6 = Mk * kSixth, m16 = Mk1 * kSixth;
    const double v = m6 * a * a * a + m16 * b * b * b + (yk[e] - m6) * a + (yk1[e] - m16) * b;
    out[o] = tbc_pixel(v, wow, C);
  }
  KSTAMP(1, 5);
  // NTSC burst flag pixels (threads 0 / 1 wrote pixels 0 / 1 above)
  if (!pal && tid < 2 && row >= 1 && row < lc - 1) {
    const float bl = blevel[(int64_t)slot * MAX_LINES + row];
    const double hzs = 1700000 / 140.0;
    if (tid == 0) out[0] = bl > 0 ? 16384 : 32768;
    const double clevel = (1 / 1.45) / hzs;
    if (tid == 1) out[1] = (uint16_t)(327.67 * clevel * fabs((double)bl));
  }
}

extern "C" __global__ __launch_bounds__(FINAL_NT, LDG_FINAL_WAVES) void ldg_k_final_lines(
    const int32_t* __restrict__ smap, const double* __restrict__ video, int64_t vread_stride, int64_t vchan_stride,
    SysConst C, FieldRec* __restrict__ recs, const double* __restrict__ lines, const float* __restrict__ blevel,
    uint16_t* __restrict__ pic, int64_t pic_stride, const ReadDesc* __restrict__ reads) {
  final_lines_impl<false>(smap, video, vread_stride, vchan_stride, C, recs, lines, blevel, pic, pic_stride, reads);
}
extern "C" __global__ __launch_bounds__(FINAL_NT, 5) void ldg_k_final_lines_h(
    const int32_t* __restrict__ smap, const double* __restrict__ video, int64_t vread_stride, int64_t vchan_stride,
    SysConst C, FieldRec* __restrict__ recs, const double* __restrict__ lines, const float* __restrict__ blevel,
    uint16_t* __restrict__ pic, int64_t pic_stride, const ReadDesc* __restrict__ reads) {
  final_lines_impl<true>(smap, video, vread_stride, vchan_stride, C, recs, lines, blevel, pic, pic_stride, reads);
}

// Mark reads still pending after the whole chain as valid.
// ---------------------------------------------------------------------------
// downscale_audio (lddecode_core.py:431-484) for n fields.  grid: n x 256.
// Field i's inputs live at entry idx[i] of (recs, lines + entry * lines_stride,
// audio2 + entry * a2read_stride): the read slots (lines_stride LINES_STRIDE,
// final locations at LLF) or the field archive (lines_stride MAX_LINES).
extern "C" __global__ __launch_bounds__(256) void ldg_k_audio_ds(
    const int64_t* __restrict__ idx, const double* __restrict__ offsets, const FieldRec* __restrict__ recs,
    const double* __restrict__ lines, int64_t lines_stride, const double* __restrict__ audio2, int64_t a2read_stride,
    int64_t a2chan_stride, SysConst C, int16_t* __restrict__ pcm, int64_t pcm_stride, int32_t* __restrict__ counts,
    double* __restrict__ next_off, int32_t* __restrict__ err) {
  const int f = blockIdx.x;
  const int64_t slot = idx[f];
  const FieldRec* R = recs + slot;
  const int lc = R->linecount, nl = R->nlines;
  const double* lf = lines + slot * lines_stride;
  const double* aL = audio2 + slot * a2read_stride;
  const double* aR = aL + a2chan_stride;
  const int64_t na = R->n_out > 0 ? ((R->n_out - 1) / AUDIO_DIV1 + 1) / AUDIO_DIV2 : 0;
  const double frametime = (C.line_period * lc) / 1000000;
  const double gap = 1 / 48000.0;
  const double start = offsets[f];
  const double stop = frametime + gap;
  const int64_t len = (int64_t)ceil((stop - start) / gap);
  const double t1 = start + gap;
  const double dl = t1 - start;
  auto tick = [&](int64_t i) { return i == 0 ? start : (i == 1 ? t1 : start + (double)i * dl); };
  int16_t* out = pcm + (int64_t)f * pcm_stride;
  for (int64_t i = threadIdx.x; i < len - 1; i += blockDim.x) {
    const double t = tick(i);
    const double ln = ((t * 1000000) / C.line_period) + 1;
    const int64_t il = (int64_t)ln;
    if (il < 0 || il >= nl) { atomicOr(err + f, 1); continue; }
    const double cur = lf[il];
    const double nxt = (il + 1 < nl) ? lf[il + 1] : cur + C.linelen;
    double pos = cur;
    pos += (nxt - cur) * (ln - floor(ln));
    const double swow = ((nxt - cur) / C.linelen);
    const double loc = pos / 64;
    int64_t ai;
    if (!py_index((int64_t)loc, na, ai)) { atomicOr(err + f, 1); continue; }
    double left = aL[ai], right = aR[ai];
    left *= swow; right *= swow;
    left -= C.audio_lfreq; right -= C.audio_rfreq;
    double ol = rint(left * 32767 / 150000), orr = rint(right * 32767 / 150000);
    ol = fmin(fmax(ol, -32766.0), 32766.0);
    orr = fmin(fmax(orr, -32766.0), 32766.0);
    out[2 * i] = (int16_t)ol;
    out[2 * i + 1] = (int16_t)orr;
  }
  if (threadIdx.x == 0) {
    counts[f] = (int32_t)(len - 1);
    next_off[f] = tick(len - 1) - frametime;
  }
}

// Framer.formatoutput: grid (n_frames, ceil(frame_lines / FRAME_ROWS)) x 256, FRAME_ROWS
// rows per workgroup (one row per workgroup was ~16k tiny workgroups per call, each
// holding a CU for a load round trip), 32-bit copies when the line length is even.
constexpr int FRAME_ROWS = 8;
extern "C" __global__ __launch_bounds__(256) void ldg_k_frames(const int32_t* __restrict__ top,
                                                               const int32_t* __restrict__ bot,
                                                               const FieldRec* __restrict__ recs,
                                                               const uint16_t* __restrict__ pic, int64_t pic_stride,
                                                               SysConst C, uint16_t* __restrict__ out) {
  const int f = blockIdx.x;
  const int W = C.outlinelen;
  const int ts = top[f], bs = bot[f];
  const int lt = recs[ts].linecount, lb = recs[bs].linecount;
  const int lc = ((lt < lb) ? lt : lb) * 2;
  for (int i = 0; i < FRAME_ROWS; i++) {
    const int row = blockIdx.y * FRAME_ROWS + i;
    if (row >= C.frame_lines) break;
    uint16_t* dst = out + ((int64_t)f * C.frame_lines + row) * W;
    const uint16_t* src = nullptr;
    if (row < lc) src = pic + (int64_t)((row & 1) ? bs : ts) * pic_stride + (int64_t)(row >> 1) * W;
    else if (row == lc) src = pic + (int64_t)((lt >= lb) ? ts : bs) * pic_stride + (int64_t)(lc >> 1) * W;
    if ((W & 1) == 0 && (pic_stride & 1) == 0) {
      uint32_t* d32 = reinterpret_cast<uint32_t*>(dst);
      const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src);
      for (int x = threadIdx.x; x < W / 2; x += blockDim.x) d32[x] = src ? s32[x] : 0u;
    } else {
      for (int x = threadIdx.x; x < W; x += blockDim.x) dst[x] = src ? src[x] : 0;
    }
  }
}

// ---------------------------------------------------------------------------
// PAL pilot refine (FieldPAL.refine_linelocs_pilot, lddecode_core.py:962-1021).
// Per line (lane): zero crossings of the flipped (demod - demod_05) 4.7 us
// window before the line location; offsets to scratch.  Per read: median of
// all kept offsets -> target phase; per-line median adjustment.
namespace {
constexpr int PILOT_MAX = 64;
__device__ __forceinline__ double* pilot_base(double* scratch, int slot) {
  return scratch + (int64_t)slot * SCR_PER_SLOT;
}
}  // namespace

// grid: n_reads * MAX_LINES workgroups of 64 threads (one wave per line): the
// wave forms the flipped (demod - demod_05) of the window in LDS.  The
// reference's crossing walk (i -> int(zc + 1) + 1 after a crossing, i + 1
// otherwise) only ever starts calczc at qualifying positions, and calczc's
// result does not depend on the walk: every lane evaluates its own positions
// first, then the walk is a bit scan over the qualifying mask (one LDS read per
// crossing).  The per-line median of offsets[1:-1] is a rank sort across lanes.
extern "C" __global__ __launch_bounds__(64) void ldg_k_pilot_lines(const int32_t* __restrict__ smap,
                                                                   const double* __restrict__ video,
                                                                   int64_t vread_stride, int64_t vchan_stride,
                                                                   SysConst C, FieldRec* __restrict__ recs,
                                                                   double* __restrict__ lines,
                                                                   double* __restrict__ scratch,
                                                                   const ReadDesc* __restrict__ reads) {
  prio_latency();

  constexpr int PW = 256;                       // 4.7 us at 40 MSPS: 188 samples
  __shared__ double s_pil[PW];
  __shared__ double s_zc[PW];
  __shared__ double s_off[PILOT_MAX];
  __shared__ double s_srt[PILOT_MAX];
  const int lane = threadIdx.x;
  const int slot = smap[blockIdx.y];
  const int l = blockIdx.x;
  FieldRec* R = recs + slot;
  if (R->status != FS_PENDING) return;
  const int nl = R->nlines;
  if (l >= nl) return;
  const double* ll = lines + (int64_t)slot * LINES_STRIDE + LL2 * MAX_LINES;
  const double* dm = video + (int64_t)slot * vread_stride + (int64_t)CH_DEMOD * vchan_stride;
  const int64_t len = R->n_out;
  double* P = pilot_base(scratch, slot);
  double* offs = P + (int64_t)l * PILOT_MAX;
  double* meta = P + (int64_t)MAX_LINES * PILOT_MAX;    // [count, keep, median] per line
  int64_t a, b;
  py_slice(py_int(ll[l] - 4.7 * C.freq), py_int(ll[l]), len, a, b);
  const int pn = (int)(b > a ? b - a : 0);
  const int pm = pn < PW ? pn : PW;             // pn <= PW at the reference's sample rates
  if (pn > 0 && b - 1 >= reads[slot].vcut) {    // past the read's video cut: decode it in full
    if (lane == 0) R->status = FS_VCUT;
    return;
  }
  const double* d05 = video + (int64_t)slot * vread_stride + (int64_t)CH_05 * vchan_stride;
  for (int q = lane; q < pm; q += 64) s_pil[q] = dm[b - 1 - q] - d05[b - 1 - q];   // np.flip
  __syncthreads();
  uint64_t qm[PW / 64];
#pragma unroll
  for (int j = 0; j < PW / 64; j++) {
    const int i = lane + 64 * j;
    bool q = false;
    if (i < pm && inrange(s_pil[i], -300000, -100000)) {
      double zc;
      if (calczc(s_pil, pm, (double)i, 0.0, 10, &zc) == 0) {
        s_zc[i] = zc;
        q = true;
      }
    }
    qm[j] = __ballot(q);
  }
  __syncthreads();
  double adjfreq = C.freq;
  if (l > 1) adjfreq /= (ll[l] - ll[l - 1]) / (double)C.linelen;
  int cnt = 0, i = 0;
  double myoff = 0.0;                           // offsets[l][lane]
  while (i < pm) {
    int nxt = -1;
#pragma unroll
    for (int j = 0; j < PW / 64; j++) {
      uint64_t m = qm[j];
      if ((i >> 6) > j) m = 0;
      else if ((i >> 6) == j) m &= ~0ull << (i & 63);
      if (nxt < 0 && m) nxt = 64 * j + __ffsll((unsigned long long)m) - 1;
    }
    if (nxt < 0) break;
    const double zc = s_zc[nxt];
    const double zcp = zc / (adjfreq / 3.75);
    if (lane == cnt) myoff = zcp - floor(zcp);
    cnt++;
    i = (int)(zc + 1) + 1;
  }
  if (i < pn) i = pn;                           // the walk runs on to the window's end
  if (cnt > PILOT_MAX) cnt = PILOT_MAX;
  // offsets[l][1:-1] for l >= 2 (len(offsets dict) >= 3); kept in alloffsets if i >= 11
  int keep = 0, k = 0;
  double med = 0.0;
  if (l >= 2) {
    k = cnt >= 2 ? cnt - 2 : 0;
    keep = (i >= 11) ? 1 : 0;
    const bool mine = lane >= 1 && lane <= k;
    if (mine) {
      s_off[lane - 1] = myoff;
      offs[lane - 1] = myoff;
    }
    __syncthreads();
    if (mine) {                                 // stable rank = np.sort position
      int r = 0;
      for (int t = 0; t < k; t++) {
        const double v = s_off[t];
        r += (v < myoff) || (v == myoff && t < lane - 1);
      }
      s_srt[r] = myoff;
    }
    __syncthreads();
    if (k > 0) med = sorted_median(s_srt, k);
  }
  if (lane == 0) {
    meta[3 * l + 0] = k;
    meta[3 * l + 1] = keep;
    meta[3 * l + 2] = med;
  }
}

namespace {
// k-th smallest dkey of a[0..n) (0 <= k < n, no NaNs), whole 256-thread block:
// radix select, 8 bits per pass, the digit chosen by wave 0.
__device__ uint64_t block_kth_key(const double* a, int n, int k, int tid, int* hist, int* sel, uint64_t* key) {
  const int lane = tid & 63;
  uint64_t prefix = 0, mask = 0;
  for (int shift = 56; shift >= 0; shift -= 8) {
    hist[tid] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += 256) {
      const uint64_t u = dkey(a[i]);
      if ((u & mask) == prefix) atomicAdd(&hist[(u >> shift) & 255], 1);
    }
    __syncthreads();
    if (tid < 64) {
      int c[4], tot = 0;
#pragma unroll
      for (int e = 0; e < 4; e++) { c[e] = hist[4 * lane + e]; tot += c[e]; }
      int incl = tot;
      for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o);
        if (lane >= o) incl += v;
      }
      const int excl = incl - tot;
      if (k >= excl && k < incl) {
        int run = excl, digit = -1;
#pragma unroll
        for (int e = 0; e < 4; e++) {
          if (digit < 0 && k < run + c[e]) { digit = 4 * lane + e; sel[0] = digit; sel[1] = run; sel[2] = c[e]; }
          run += c[e];
        }
      }
    }
    __syncthreads();
    const int digit = sel[0], below = sel[1], cnt = sel[2];
    k -= below;
    prefix |= (uint64_t)digit << shift;
    mask |= (uint64_t)255 << shift;
    if (cnt == 1 && shift > 0) {
      // one key left with this prefix: it is the k-th
      for (int i = tid; i < n; i += 256) {
        const uint64_t u = dkey(a[i]);
        if ((u & mask) == prefix) *key = u;
      }
      __syncthreads();
      const uint64_t r = *key;
      __syncthreads();
      return r;
    }
    __syncthreads();
  }
  return prefix;
}
}  // namespace

// grid: n reads x 256 threads.  alloffsets (the kept lines' offsets, line order)
// gathered by a block scan of the per-line counts, np.median by radix select,
// then every line's adjustment in parallel.
extern "C" __global__ __launch_bounds__(256) void ldg_k_pilot_field(const int32_t* __restrict__ smap,
                                                                    FieldRec* __restrict__ recs,
                                                                    double* __restrict__ lines, SysConst C,
                                                                    double* __restrict__ scratch) {
  prio_latency();

  constexpr int NALL = 8192;
  static_assert(MAX_LINES <= 512, "two lines per thread");
  __shared__ double s_all[NALL];
  __shared__ int s_wsum[4];
  __shared__ int s_hist[256];
  __shared__ int s_sel[3];
  __shared__ uint64_t s_key;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int slot = smap[blockIdx.x];
  FieldRec* R = recs + slot;
  if (R->status != FS_PENDING) return;
  const int nl = R->nlines;
  double* P = pilot_base(scratch, slot);
  const double* meta = P + (int64_t)MAX_LINES * PILOT_MAX;
  const int l0 = 2 * tid, l1 = 2 * tid + 1;
  const int c0 = (l0 < nl && meta[3 * l0 + 1] != 0) ? (int)meta[3 * l0 + 0] : 0;
  const int c1 = (l1 < nl && meta[3 * l1 + 1] != 0) ? (int)meta[3 * l1 + 0] : 0;
  const int tot = c0 + c1;
  int incl = tot;
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(incl, o);
    if (lane >= o) incl += v;
  }
  if (lane == 63) s_wsum[w] = incl;
  __syncthreads();
  int off = incl - tot;
  for (int q = 0; q < w; q++) off += s_wsum[q];
  const int total = s_wsum[0] + s_wsum[1] + s_wsum[2] + s_wsum[3];
  for (int q = 0; q < c0; q++)
    if (off + q < NALL) s_all[off + q] = P[(int64_t)l0 * PILOT_MAX + q];
  off += c0;
  for (int q = 0; q < c1; q++)
    if (off + q < NALL) s_all[off + q] = P[(int64_t)l1 * PILOT_MAX + q];
  __syncthreads();
  const int n = total < NALL ? total : NALL;
  double med = __builtin_nan("");               // np.median([]) is nan
  if (n > 0) {
    med = dkey_val(block_kth_key(s_all, n, (n - 1) / 2, tid, s_hist, s_sel, &s_key));
    if (!(n & 1)) med = (med + dkey_val(block_kth_key(s_all, n, n / 2, tid, s_hist, s_sel, &s_key))) / 2.0;
  }
  const double tgt = inrange(med, 0.25, 0.75) ? .5 : 0;
  const double* ll = lines + (int64_t)slot * LINES_STRIDE + LL2 * MAX_LINES;
  double* lf = lines + (int64_t)slot * LINES_STRIDE + LLF * MAX_LINES;
  for (int l = tid; l < nl; l += 256) {
    double v = ll[l];
    if (meta[3 * l + 0] > 0) v += (tgt - meta[3 * l + 2]) * (C.freq / 3.75) * .25;
    lf[l] = v;
  }
}
