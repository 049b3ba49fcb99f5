// Device restatements of the numpy / Python primitives the reference's
// per-field logic is built from, with their exact semantics (summation order,
// first-occurrence argmax, Python slicing / negative indexing, banker's
// rounding).  Used by field.hip and tbc.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ldg {

// numpy pairwise summation (numpy/_core/src/umath/loops_utils.h.src,
// PW_BLOCKSIZE = 128, 8-way unrolled); np.sum/np.mean of a float64 array.
__device__ inline double pw_block(const double* a, int n) {
  if (n < 8) {
    double r = -0.0;
    for (int i = 0; i < n; i++) r += a[i];
    return r;
  }
  double r[8];
  for (int j = 0; j < 8; j++) r[j] = a[j];
  int i = 8;
  for (; i < n - (n % 8); i += 8)
    for (int j = 0; j < 8; j++) r[j] += a[i + j];
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; i++) res += a[i];
  return res;
}

// pw_block of a[0..n) (n <= 128) on one wave, result in every lane: lanes 0..7
// run the eight accumulators, a shuffle tree combines them in numpy's order.
__device__ inline double wave_pw_block(const double* a, int n, int lane) {
  if (n < 8) return __shfl(lane == 0 ? pw_block(a, n) : 0.0, 0);
  const int nb = n - (n % 8);
  double r = 0.0;
  if (lane < 8) {
    r = a[lane];
    for (int i = 8 + lane; i < nb; i += 8) r += a[i];
  }
  r = r + __shfl_xor(r, 1);
  r = r + __shfl_xor(r, 2);
  r = r + __shfl_xor(r, 4);
  double res = __shfl(r, 0);
  for (int i = nb; i < n; i++) res += a[i];
  return res;
}

template <int L> __device__ inline double pw_sum_l(const double* a, int n) {
  if (n <= 128) return pw_block(a, n);
  int n2 = n / 2;
  n2 -= n2 % 8;
  return pw_sum_l<L - 1>(a, n2) + pw_sum_l<L - 1>(a + n2, n - n2);
}
template <> __device__ inline double pw_sum_l<0>(const double* a, int n) { return pw_block(a, n); }

__device__ inline double pw_sum(const double* a, int n) { return 0.0 + pw_sum_l<8>(a, n); }
__device__ inline double np_mean(const double* a, int n) { return pw_sum(a, n) / (double)n; }

// np.std (ddof 0): mean, deviations, squares, pairwise sum, / n, sqrt.  `tmp` >= n doubles.
__device__ inline double np_std(const double* a, int n, double* tmp) {
  const double m = pw_sum(a, n) / (double)n;
  for (int i = 0; i < n; i++) { const double d = a[i] - m; tmp[i] = d * d; }
  return sqrt(pw_sum(tmp, n) / (double)n);
}

// pw_sum on one wave, result in every lane.  numpy's recursion splits n at
// (n/2 rounded down to a multiple of 8) until a piece has <= 128 elements; the
// pieces (at most 64 here) are summed one per lane with pw_block, then the
// recursion is replayed with each piece's sum fetched from its lane, so every
// addition happens in numpy's order.  Wave-uniform control flow throughout.
template <int L> __device__ inline void pw_leaves(int off, int n, int& cnt, int lane, int& my_off, int& my_n) {
  if (L == 0 || n <= 128) {
    if (cnt == lane) { my_off = off; my_n = n; }
    cnt++;
    return;
  }
  int n2 = n / 2;
  n2 -= n2 % 8;
  pw_leaves<(L > 0 ? L - 1 : 0)>(off, n2, cnt, lane, my_off, my_n);
  pw_leaves<(L > 0 ? L - 1 : 0)>(off + n2, n - n2, cnt, lane, my_off, my_n);
}
template <int L> __device__ inline double pw_combine(int n, int& cnt, double leaf) {
  if (L == 0 || n <= 128) return __shfl(leaf, cnt++);
  int n2 = n / 2;
  n2 -= n2 % 8;
  const double l = pw_combine<(L > 0 ? L - 1 : 0)>(n2, cnt, leaf);
  return l + pw_combine<(L > 0 ? L - 1 : 0)>(n - n2, cnt, leaf);
}
// n <= 64 * 128 (callers here: a field's sync peaks, <= MAX_PEAKS)
__device__ inline double wave_pw_sum(const double* a, int n, int lane) {
  int cnt = 0, off = 0, m = 0;
  pw_leaves<6>(0, n, cnt, lane, off, m);
  const double leaf = (lane < cnt) ? pw_block(a + off, m) : 0.0;
  cnt = 0;
  return 0.0 + pw_combine<6>(n, cnt, leaf);
}
// np_std on one wave (tmp: n doubles of scratch, in LDS), result in every lane.
__device__ inline double wave_np_std(const double* a, int n, double* tmp, int lane) {
  const double m = wave_pw_sum(a, n, lane) / (double)n;
  for (int i = lane; i < n; i += 64) { const double d = a[i] - m; tmp[i] = d * d; }
  __syncthreads();
  return sqrt(wave_pw_sum(tmp, n, lane) / (double)n);
}

__device__ inline bool inrange(double a, double lo, double hi) { return (a >= lo) && (a <= hi); }

// np.round / Python round on doubles: half to even.
__device__ inline double np_round(double x) { return rint(x); }

// Python slice [a:b] of a length-n sequence -> [lo, hi) (empty if lo >= hi).
__device__ inline void py_slice(int64_t a, int64_t b, int64_t n, int64_t& lo, int64_t& hi) {
  if (a < 0) { a += n; if (a < 0) a = 0; } else if (a > n) a = n;
  if (b < 0) { b += n; if (b < 0) b = 0; } else if (b > n) b = n;
  lo = a; hi = b;
}

// Python index (negative wraps); returns false on IndexError.
__device__ inline bool py_index(int64_t i, int64_t n, int64_t& out) {
  if (i < 0) i += n;
  if (i < 0 || i >= n) return false;
  out = i;
  return true;
}

// int() of a Python float: truncation toward zero.
__device__ inline int64_t py_int(double x) { return (int64_t)x; }

// lddutils.calczc (lddutils.py:265-303) with edge='both', reverse=False.
// Returns 0 and sets *res on success, 1 for "None", -1 for an IndexError.
__device__ inline int calczc(const double* data, int64_t len, double start_offset, double target, int64_t count,
                             double* res) {
  const int64_t s = py_int(start_offset);
  const int64_t n = count + 1;
  int64_t si;
  if (!py_index(s, len, si)) return -1;         // data[start_offset] IndexError
  const bool rising = data[si] < target;
  int64_t lo, hi;
  py_slice(s, s + n, len, lo, hi);
  int64_t hit = -1;
  for (int64_t k = lo; k < hi; k++) {
    const double v = data[k];
    if (rising ? (v >= target) : (v <= target)) { hit = k - lo; break; }
  }
  if (hit < 0) return 1;
  const int64_t x = s + hit;
  if (x == 0) return 1;
  int64_t ia, ib;
  if (!py_index(x - 1, len, ia) || !py_index(x, len, ib)) return -1;
  const double a = data[ia] - target;
  const double b = data[ib] - target;
  *res = (double)(x - 1) + ((-a) / ((-a) + b));
  return 0;
}

// ---- one-wave (64 lanes, all calling) versions of the scans above ----------
// first k in [lo, hi) with data[k] >= target (rising) / <= target, or -1
template <class Src>
__device__ inline int64_t wave_find_first(const Src& data, int64_t lo, int64_t hi, bool rising, double target,
                                          int lane) {
  for (int64_t k0 = lo; k0 < hi; k0 += 64) {
    const int64_t k = k0 + lane;
    bool p = false;
    if (k < hi) { const double v = data[k]; p = rising ? (v >= target) : (v <= target); }
    const uint64_t m = __ballot(p);
    if (m) return k0 + (__ffsll((unsigned long long)m) - 1);
  }
  return -1;
}

// calczc above, wave-parallel search (same result and error semantics)
// (Src: a pointer or any indexable source)
template <class Src>
__device__ inline int wave_calczc(const Src& data, int64_t len, double start_offset, double target, int64_t count,
                                  int lane, double* res) {
  const int64_t s = py_int(start_offset);
  const int64_t n = count + 1;
  int64_t si;
  if (!py_index(s, len, si)) return -1;
  const bool rising = data[si] < target;
  int64_t lo, hi;
  py_slice(s, s + n, len, lo, hi);
  const int64_t k = wave_find_first(data, lo, hi, rising, target, lane);
  if (k < 0) return 1;
  const int64_t x = s + (k - lo);
  if (x == 0) return 1;
  int64_t ia, ib;
  if (!py_index(x - 1, len, ia) || !py_index(x, len, ib)) return -1;
  const double a = data[ia] - target;
  const double b = data[ib] - target;
  *res = (double)(x - 1) + ((-a) / ((-a) + b));
  return 0;
}

// wave_calczc with every load of the search issued at once (the sample at the
// start, up to 64 * MAXC window samples and their left neighbours), so the
// search costs one memory latency instead of one per 64-sample chunk.  Windows
// longer than 64 * MAXC samples, or a negative start, take wave_calczc.
template <int MAXC, class Src>
__device__ inline int wave_calczc_pf(const Src& data, int64_t len, double start_offset, double target,
                                     int64_t count, int lane, double* res) {
  const int64_t s = py_int(start_offset);
  const int64_t n = count + 1;
  int64_t si;
  if (!py_index(s, len, si)) return -1;
  int64_t lo, hi;
  py_slice(s, s + n, len, lo, hi);
  if (s < 0 || hi - lo > 64 * MAXC) return wave_calczc(data, len, start_offset, target, count, lane, res);
  const double v0 = data[si];
  double v[MAXC], vp[MAXC];
#pragma unroll
  for (int c = 0; c < MAXC; c++) {
    const int64_t k = lo + 64 * c + lane;
    v[c] = (k < hi) ? data[k] : 0.0;
    vp[c] = (k < hi && k >= 1) ? data[k - 1] : 0.0;
  }
  const bool rising = v0 < target;
#pragma unroll
  for (int c = 0; c < MAXC; c++) {
    const int64_t k = lo + 64 * c + lane;
    const bool p = k < hi && (rising ? (v[c] >= target) : (v[c] <= target));
    const uint64_t m = __ballot(p);
    if (m) {
      const int h = __ffsll((unsigned long long)m) - 1;
      const int64_t x = lo + 64 * c + h;           // lo == s here
      if (x == 0) return 1;
      const double a = __shfl(vp[c], h) - target;
      const double b = __shfl(v[c], h) - target;
      *res = (double)(x - 1) + ((-a) / ((-a) + b));
      return 0;
    }
  }
  return 1;
}

// np.min / np.max of data[a, b) (b > a): NaN if any element is NaN
__device__ inline double wave_minmax_np(const double* data, int64_t a, int64_t b, bool is_max, int lane) {
  double m = is_max ? -__builtin_inf() : __builtin_inf();
  bool nan = false;
  for (int64_t k = a + lane; k < b; k += 64) {
    const double v = data[k];
    if (v != v) nan = true;
    else m = is_max ? fmax(m, v) : fmin(m, v);
  }
  for (int o = 32; o > 0; o >>= 1) {
    const double t = __shfl_xor(m, o);
    m = is_max ? fmax(m, t) : fmin(m, t);
  }
  return __ballot(nan) ? __builtin_nan("") : m;
}

// np.min and np.max of data[a, b) (b > a) in one pass (each NaN if any element is NaN)
template <class Src>
__device__ inline void wave_minmax2_np(const Src& data, int64_t a, int64_t b, int lane, double& mn, double& mx) {
  double lo = __builtin_inf(), hi = -__builtin_inf();
  bool nan = false;
  for (int64_t k = a + lane; k < b; k += 64) {
    const double v = data[k];
    if (v != v) nan = true;
    else { lo = fmin(lo, v); hi = fmax(hi, v); }
  }
  for (int o = 32; o > 0; o >>= 1) {
    lo = fmin(lo, __shfl_xor(lo, o));
    hi = fmax(hi, __shfl_xor(hi, o));
  }
  const bool any_nan = __ballot(nan) != 0;
  mn = any_nan ? __builtin_nan("") : lo;
  mx = any_nan ? __builtin_nan("") : hi;
}

// Sorted-window median helper: median of a[0..n) already sorted ascending.
__device__ inline double sorted_median(const double* a, int n) {
  if (n <= 0) return __builtin_nan("");
  if (n & 1) return a[n / 2];
  return (a[n / 2 - 1] + a[n / 2]) / 2.0;
}

// In-place insertion sort (small n, one thread).  NaNs sort last like np.sort.
__device__ inline void isort(double* a, int n) {
  for (int i = 1; i < n; i++) {
    const double v = a[i];
    int j = i - 1;
    while (j >= 0 && (a[j] > v || (a[j] != a[j] && v == v))) { a[j + 1] = a[j]; j--; }
    a[j + 1] = v;
  }
}

// np.median of a[0..n) with a scratch copy (one thread).
__device__ inline double np_median(const double* a, int n, double* tmp) {
  if (n <= 0) return __builtin_nan("");
  for (int i = 0; i < n; i++) tmp[i] = a[i];
  isort(tmp, n);
  for (int i = 0; i < n; i++) if (tmp[i] != tmp[i]) return __builtin_nan("");
  return sorted_median(tmp, n);
}

// k-th smallest (0-based) of a[0..n) for non-negative, non-NaN doubles, one
// wave (all 64 lanes call it): radix select over the IEEE bit patterns (which
// order like the values for x >= 0), 8 bits per pass.  hist: 256 ints of LDS.
__device__ inline double wave_kth(const double* a, int n, int k, int lane, int* hist) {
  uint64_t prefix = 0, mask = 0;
  for (int shift = 56; shift >= 0; shift -= 8) {
    for (int d = lane; d < 256; d += 64) hist[d] = 0;
    __syncthreads();
    for (int i = lane; i < n; i += 64) {
      const uint64_t u = (uint64_t)__double_as_longlong(a[i]);
      if ((u & mask) == prefix) atomicAdd(&hist[(u >> shift) & 255], 1);
    }
    __syncthreads();
    // digit whose cumulative count passes k: lane owns digits 4*lane..4*lane+3
    int c[4], tot = 0;
#pragma unroll
    for (int e = 0; e < 4; e++) { c[e] = hist[4 * lane + e]; tot += c[e]; }
    int incl = tot;
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(incl, o);
      if (lane >= o) incl += v;
    }
    const int excl = incl - tot;
    int digit = -1, below = 0, cnt = 0;
    if (k >= excl && k < incl) {
      int run = excl;
#pragma unroll
      for (int e = 0; e < 4; e++) {
        if (digit < 0 && k < run + c[e]) { digit = 4 * lane + e; below = run; cnt = c[e]; }
        run += c[e];
      }
    }
    const uint64_t m = __ballot(digit >= 0);
    const int src = __ffsll((unsigned long long)m) - 1;
    digit = __shfl(digit, src);
    below = __shfl(below, src);
    cnt = __shfl(cnt, src);
    k -= below;
    prefix |= (uint64_t)digit << shift;
    mask |= (uint64_t)255 << shift;
    __syncthreads();
    if (cnt == 1 && shift > 0) {
      // one key left with this prefix: it is the k-th; fetch it instead of more passes
      uint64_t key = 0;
      bool hit = false;
      for (int i = lane; i < n && !hit; i += 64) {
        const uint64_t u = (uint64_t)__double_as_longlong(a[i]);
        if ((u & mask) == prefix) { key = u; hit = true; }
      }
      const uint64_t hm = __ballot(hit);
      const int hs = __ffsll((unsigned long long)hm) - 1;
      return __longlong_as_double((long long)__shfl((long long)key, hs));
    }
  }
  return __longlong_as_double((long long)prefix);
}

// Block-wide bitonic sort of a[0..npow2) in LDS (npow2 a power of two, pad with +inf).
__device__ inline void block_bitonic_sort(double* a, int npow2, int tid, int nthreads) {
  for (int k = 2; k <= npow2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < npow2; i += nthreads) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const double x = a[i], y = a[ixj];
          const bool up = (i & k) == 0;
          if (up ? (x > y) : (x < y)) { a[i] = y; a[ixj] = x; }
        }
      }
      __syncthreads();
    }
  }
}

}  // namespace ldg

// ---- selection over doubles of any sign (no NaNs) ------------------------------
// order-preserving unsigned key of a double (negative values bit-inverted)
__device__ inline uint64_t dkey(double x) {
  const uint64_t u = (uint64_t)__double_as_longlong(x);
  return (u >> 63) ? ~u : (u | (1ull << 63));
}
__device__ inline double dkey_val(uint64_t k) {
  const uint64_t u = (k >> 63) ? (k & ~(1ull << 63)) : ~k;
  return __longlong_as_double((long long)u);
}

// k-th smallest key (0-based) of dkey(a[0..n)), one wave: radix select, 8 bits
// per pass.  hist: 256 ints of LDS.
__device__ inline uint64_t wave_kth_key(const double* a, int n, int k, int lane, int* hist) {
  uint64_t prefix = 0, mask = 0;
  for (int shift = 56; shift >= 0; shift -= 8) {
    for (int d = lane; d < 256; d += 64) hist[d] = 0;
    __syncthreads();
    for (int i = lane; i < n; i += 64) {
      const uint64_t u = dkey(a[i]);
      if ((u & mask) == prefix) atomicAdd(&hist[(u >> shift) & 255], 1);
    }
    __syncthreads();
    int c[4], tot = 0;
#pragma unroll
    for (int e = 0; e < 4; e++) { c[e] = hist[4 * lane + e]; tot += c[e]; }
    int incl = tot;
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(incl, o);
      if (lane >= o) incl += v;
    }
    const int excl = incl - tot;
    int digit = -1, below = 0, cnt = 0;
    if (k >= excl && k < incl) {
      int run = excl;
#pragma unroll
      for (int e = 0; e < 4; e++) {
        if (digit < 0 && k < run + c[e]) { digit = 4 * lane + e; below = run; cnt = c[e]; }
        run += c[e];
      }
    }
    const uint64_t m = __ballot(digit >= 0);
    const int src = __ffsll((unsigned long long)m) - 1;
    digit = __shfl(digit, src);
    below = __shfl(below, src);
    cnt = __shfl(cnt, src);
    k -= below;
    prefix |= (uint64_t)digit << shift;
    mask |= (uint64_t)255 << shift;
    __syncthreads();
    if (cnt == 1 && shift > 0) {
      // one key left with this prefix: it is the k-th; fetch it instead of more passes
      uint64_t key = 0;
      bool hit = false;
      for (int i = lane; i < n && !hit; i += 64) {
        const uint64_t u = dkey(a[i]);
        if ((u & mask) == prefix) { key = u; hit = true; }
      }
      const uint64_t hm = __ballot(hit);
      const int hs = __ffsll((unsigned long long)hm) - 1;
      return (uint64_t)__shfl((long long)key, hs);
    }
  }
  return prefix;
}

// np.median of a[0..n) (n > 0, no NaNs), one wave: the middle order statistic(s)
// -- the value np.sort would put there (up to the sign of a zero).
__device__ inline double wave_median(const double* a, int n, int lane, int* hist) {
  if (n & 1) return dkey_val(wave_kth_key(a, n, n / 2, lane, hist));
  const uint64_t k0 = wave_kth_key(a, n, n / 2 - 1, lane, hist);
  // the next order statistic: k0 again if it occurs beyond rank n/2 - 1, else
  // the smallest key above k0
  int le = 0;
  uint64_t up = ~0ull;
  for (int i = lane; i < n; i += 64) {
    const uint64_t u = dkey(a[i]);
    if (u <= k0) le++;
    else if (u < up) up = u;
  }
  for (int o = 32; o > 0; o >>= 1) {
    le += __shfl_xor(le, o);
    const uint64_t t = (uint64_t)__shfl_xor((long long)up, o);
    up = t < up ? t : up;
  }
  const uint64_t k1 = (le >= n / 2 + 1) ? k0 : up;
  return (dkey_val(k0) + dkey_val(k1)) / 2.0;
}

