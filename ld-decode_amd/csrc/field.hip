// Per-field sync analysis and line location (one workgroup per field read).
//
// Restates Field.get_syncpeaks / get_hsync_median / is_regular_hsync /
// determine_field / determine_vsyncs (lddecode_core.py:497-636), the
// Field.__init__ branch that sets nextfieldoffset / istop / linecount
// (:909-933), compute_linelocs (:638-713), refine_linelocs_hsync (:715-787),
// decodephillipscode / processphilipscode (:814-884).
//
// These are data-dependent sequential scans over ~1000 sync peaks and ~263
// lines; they run wave-parallel where the reference has array work (window
// argmax, medians, per-line crossing searches) and on lane 0 where the
// reference is a scalar recurrence.  Many field reads run concurrently, one
// workgroup each.
#include <hip/hip_runtime.h>
#include "common.hpp"
#include "field_rec.hpp"
#include "pyops.hpp"
#include "chan.hpp"

using namespace ldg;

namespace {

constexpr int SEG_K = 64;      // walk segments per read
constexpr int SEG_NMAX = 96;   // visited positions recorded per segment

struct SyncView {
  const int32_t* pk;   // peak positions
  const double* lv;    // ds[pk[i]]
  int np;
  double med, tol;
  // is_regular_hsync (lddecode_core.py:534-542) with Python negative indexing
  __device__ bool regular(int64_t n, int64_t len_ds, bool& err) const {
    if (n >= np) return false;
    int64_t idx;
    if (!py_index(n, np, idx)) { err = true; return false; }
    if (pk[idx] > len_ds) return false;
    return inrange(lv[idx], med - tol, med + tol);
  }
  __device__ int64_t peak(int64_t n, bool& err) const {
    int64_t idx;
    if (!py_index(n, np, idx)) { err = true; return 0; }
    return pk[idx];
  }
};

// First-occurrence argmax of ds[i, wend) with numpy semantics (a NaN is the
// maximum; the first NaN wins), one wave: 20 coalesced loads per lane issued
// back to back, then a cross-lane reduction.  Window <= 1280 samples.
constexpr int ARGMAX_PER = 20;
template <class Src>
__device__ inline void wave_argmax(const Src& ds, int64_t i, int64_t wend, int lane, double& best,
                                   int64_t& bidx) {
  double vv[ARGMAX_PER];
#pragma unroll
  for (int q = 0; q < ARGMAX_PER; q++) {
    const int64_t k = i + lane + 64 * q;
    vv[q] = (k < wend) ? ds[k] : -__builtin_inf();
  }
  best = -__builtin_inf();
  bidx = 0x7fffffffffffffffLL;
#pragma unroll
  for (int q = 0; q < ARGMAX_PER; q++)
    if (am_beats(vv[q], i + lane + 64 * q, best, bidx)) { best = vv[q]; bidx = i + lane + 64 * q; }
  for (int o = 32; o > 0; o >>= 1) {
    const double ov = __shfl_xor(best, o);
    const int64_t oi = __shfl_xor(bidx, o);
    if (am_beats(ov, oi, best, bidx)) { best = ov; bidx = oi; }
  }
}

// wave_argmax from the sync tiles: whole tiles inside [i, wend) plus the raw
// samples of the two ragged ends (one load per lane each instead of 20).
template <class Src>
__device__ inline void tile_argmax(const Src& ds, const SyncTile* __restrict__ tiles, int64_t i,
                                   int64_t wend, int lane, double& best, int64_t& bidx) {
  const int64_t t0 = (i + 31) >> 5, t1 = wend >> 5;         // whole tiles [t0, t1)
  if (t0 >= t1) { wave_argmax(ds, i, wend, lane, best, bidx); return; }
  const int64_t h1 = t0 << 5, s1 = t1 << 5;               // raw [i, h1) and [s1, wend), < 32 each
  double v = -__builtin_inf();
  int64_t vi = 0x7fffffffffffffffLL;
  {
    const int64_t k = (lane < 32) ? i + lane : s1 + (lane - 32);
    const bool in = (lane < 32) ? (k < h1) : (k < wend);
    if (in) { v = ds[k]; vi = k; }
  }
  for (int64_t t = t0 + lane; t < t1; t += 64) {
    const SyncTile T = tiles[t];
    if (am_beats(T.v, T.idx, v, vi)) { v = T.v; vi = T.idx; }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const double ov = __shfl_xor(v, o);
    const int64_t oi = __shfl_xor(vi, o);
    if (am_beats(ov, oi, v, vi)) { v = ov; vi = oi; }
  }
  best = v;
  bidx = vi;
}

// get_syncpeaks walk geometry for one read (lddecode_core.py:497-515).
struct WalkGeom {
  int64_t len, stop, seg;
  int win, jump, ov;
  __device__ WalkGeom(int64_t n_out, int linelen) {
    len = n_out;
    win = linelen / 2;                     // inlinelen // 2 (and the no-peak step linelen // 2)
    jump = (int)((double)linelen * .4);    // int(rf.linelen * .4)
    stop = len - 2 * (int64_t)linelen;
    seg = stop > 0 ? (stop + SEG_K - 1) / SEG_K : 0;
    ov = 4 * linelen;                      // a walker runs this far into the next segment
  }
};

// binary search of p in the ascending list a[0..n): index or -1
__device__ __forceinline__ int find_sorted(const int32_t* a, int n, int64_t p) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] < p) lo = mid + 1; else hi = mid;
  }
  return (lo < n && a[lo] == p) ? lo : -1;
}

}  // namespace

// ---------------------------------------------------------------------------
// get_syncpeaks, part 1: the walk is a chain i -> next(i) (window argmax at i,
// then bidx + jump or i + win).  Each read is cut into SEG_K segments and one
// wave per segment walks the chain from the segment start to OV samples past
// the next segment's start, recording every visited position.  Chains that
// share a position coincide from there on (next() is a function of i alone),
// so ldg_k_sync stitches the reference's exact walk from these lists.
// grid: n_reads * SEG_K workgroups of 64 threads.
extern "C" __global__ __launch_bounds__(64) void ldg_k_sync_walk(
    const int32_t* __restrict__ smap, const ReadDesc* __restrict__ reads, const double* __restrict__ video,
    int64_t vread_stride, int64_t vchan_stride, SysConst C, const int32_t* __restrict__ status,
    int32_t* __restrict__ node_pos, int32_t* __restrict__ node_pk, double* __restrict__ node_lv,
    int32_t* __restrict__ node_n, const SyncTile* __restrict__ stiles, const double* __restrict__ sst,
    const uint32_t* __restrict__ sbits) {
  prio_latency();

  const int lane = threadIdx.x;
  const int slot = smap[blockIdx.x / SEG_K];
  const int k = blockIdx.x % SEG_K;
  const int64_t L = (int64_t)slot * SEG_K + k;
  if (status[slot] == FS_EOF || status[slot] == FS_MIGRATED) {
    if (lane == 0) node_n[L] = 0;
    return;
  }
  const ReadDesc rd = reads[slot];
  const WalkGeom G(rd.n_out, C.linelen);
  const SyncSrc ds(sst, sbits, slot, C);
  const SyncTile* tl = stiles + (int64_t)slot * STILE_PER_SLOT;
  int64_t i = (int64_t)k * G.seg;
  int64_t e = (k == SEG_K - 1) ? G.stop : (int64_t)(k + 1) * G.seg + G.ov;
  if (e > G.stop) e = G.stop;
  int n = 0;
  int32_t* P = node_pos + L * SEG_NMAX;
  int32_t* K = node_pk + L * SEG_NMAX;
  double* V = node_lv + L * SEG_NMAX;
  while (i < e && n < SEG_NMAX) {
    double best;
    int64_t bidx;
    tile_argmax(ds, tl, i, i + G.win, lane, best, bidx);
    const bool pk = best > .2;
    if (lane == 0) { P[n] = (int32_t)i; K[n] = pk ? (int32_t)bidx : -1; V[n] = best; }
    n++;
    i = pk ? bidx + G.jump : i + G.win;
  }
  if (lane == 0) node_n[L] = n;
}

// ---------------------------------------------------------------------------
// Sync peaks, hsync median/tolerance, vsyncs and the Field.__init__ branch.
// grid: n_reads workgroups of 64 threads (one wave).
extern "C" __global__ __launch_bounds__(64) void ldg_k_sync(
    const int32_t* __restrict__ smap, const ReadDesc* __restrict__ reads, const double* __restrict__ video, int64_t vread_stride,
    int64_t vchan_stride, SysConst C, FieldRec* __restrict__ recs, int32_t* __restrict__ peaks,
    const int32_t* __restrict__ status, const int32_t* __restrict__ node_pos, const int32_t* __restrict__ node_pk,
    const double* __restrict__ node_lv, const int32_t* __restrict__ node_n, const SyncTile* __restrict__ stiles,
    const double* __restrict__ sst, const uint32_t* __restrict__ sbits, int nofast) {
  prio_latency();

  __shared__ int32_t s_npos[SEG_K * SEG_NMAX];
  __shared__ int32_t s_npk[SEG_K * SEG_NMAX];
  __shared__ int32_t s_cnt[SEG_K];
  __shared__ int32_t s_pk[MAX_PEAKS];
  __shared__ double s_lv[MAX_PEAKS];
  __shared__ double s_tmp[2 * MAX_PEAKS];
  __shared__ int32_t s_cand[MAX_PEAKS];
  __shared__ int s_hist[256];
  __shared__ double s_sd;
  const int lane = threadIdx.x;
  const int slot = smap[blockIdx.x];
  FieldRec* R = recs + slot;
  const ReadDesc rd = reads[slot];
  if (lane == 0) R->n_out = rd.n_out;
  if (status[slot] == FS_EOF || status[slot] == FS_MIGRATED) {
    if (lane == 0) { R->status = status[slot]; R->npeaks = 0; R->nvsync = 0; R->log_flags = 0; }
    return;
  }
  const SyncSrc ds(sst, sbits, slot, C);
  const int64_t len = rd.n_out;
  const int linelen = C.linelen;
  const WalkGeom G(len, linelen);
  KSTAMP(3, 0);

  // ---- get_syncpeaks, part 2: stitch the segment chains ------------------------
  for (int q = lane; q < SEG_K; q += 64) s_cnt[q] = node_n[(int64_t)slot * SEG_K + q];
  for (int q = lane; q < SEG_K * SEG_NMAX; q += 64) {
    s_npos[q] = node_pos[(int64_t)slot * SEG_K * SEG_NMAX + q];
    s_npk[q] = node_pk[(int64_t)slot * SEG_K * SEG_NMAX + q];
  }
  __syncthreads();
  KSTAMP(3, 1);
  const double* nlv = node_lv + (int64_t)slot * SEG_K * SEG_NMAX;
  // the walk's peak levels are gathered after the stitch, all at once: here each
  // peak records where its level is (node index, or -1 when the direct walk
  // below already stored it), so no global load sits on the stitch's serial path
  int32_t* s_lvi = s_cand;                 // s_cand is not used until the vsync candidates
  int np = 0;
  bool overflow = false;
  // append path nodes [a, b) of chain k (their peaks, in order)
  auto emit = [&](int k, int a, int b) {
    for (int j0 = a; j0 < b && !overflow; j0 += 64) {
      const int j = j0 + lane;
      const bool isp = j < b && s_npk[k * SEG_NMAX + j] >= 0;
      const uint64_t m = __ballot(isp);
      const int rank = __popcll(m & ((1ull << lane) - 1ull));
      const int tot = __popcll(m);
      if (np + tot > MAX_PEAKS) { overflow = true; break; }
      if (isp) { s_pk[np + rank] = s_npk[k * SEG_NMAX + j]; s_lvi[np + rank] = k * SEG_NMAX + j; }
      np += tot;
    }
  };
  // per chain (lane k): the first node j* of chain k that chain k+1 also visits,
  // and its index jn* there -- a merge of the two sorted position lists from the
  // first position of chain k+1, all chains at once.  From j* on the two chains
  // coincide (next() is a function of the position), so the stitch below needs
  // no search when it enters chain k at or before j*, and one check otherwise.
  static_assert(SEG_K == 64, "one lane per chain");
  int jstar = -1, jnstar = -1;
  if (G.stop > 0 && lane + 1 < SEG_K) {
    const int c0 = s_cnt[lane], c1 = s_cnt[lane + 1];
    if (c0 > 0 && c1 > 0) {
      const int32_t* P = s_npos + lane * SEG_NMAX;
      const int32_t* Q = s_npos + (lane + 1) * SEG_NMAX;
      const int32_t q0 = Q[0];
      int lo = 0, hi = c0;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (P[mid] < q0) lo = mid + 1; else hi = mid;
      }
      int i = lo, t = 0;
      while (i < c0 && t < c1) {
        const int32_t pi = P[i], qt = Q[t];
        if (pi == qt) { jstar = i; jnstar = t; break; }
        if (pi < qt) i++; else t++;
      }
    }
  }
  // Fast path: when every chain k < 63 is entered at or before its j* (the usual
  // case), the path is chain k's nodes [a_k, j*_k) with a_0 = 0, a_k = jn*_{k-1},
  // then chain 63 to its end; if that end's next position is past the walk's
  // stop there is no direct-walk tail.  Then every chain's peaks go out at once
  // (counts, a wave prefix sum, per-lane writes); otherwise the serial stitch.
  bool done = false;
  if (G.stop > 0 && !nofast) {
    const int c0 = s_cnt[lane];
    const int prev_jn = __shfl(jnstar, lane > 0 ? lane - 1 : 0);   // all lanes active for the shuffle
    const int ak = (lane == 0) ? 0 : prev_jn;
    int bk = c0;
    bool ok = c0 > 0;
    if (lane + 1 < SEG_K) {
      ok = ok && s_cnt[lane + 1] > 0 && jstar >= 0 && ak <= jstar;
      bk = jstar;
    } else {
      const int L = lane * SEG_NMAX + c0 - 1;
      const int64_t pn = (c0 > 0) ? (s_npk[L] >= 0 ? (int64_t)s_npk[L] + G.jump : (int64_t)s_npos[L] + G.win) : 0;
      ok = ok && ak <= c0 && pn >= G.stop;
    }
    if (__ballot(ok) == ~0ull) {
      int c = 0;
      for (int j = ak; j < bk; j++) c += s_npk[lane * SEG_NMAX + j] >= 0;
      int incl = c;
      for (int d = 1; d < 64; d <<= 1) {
        const int v = __shfl_up(incl, d);
        if (lane >= d) incl += v;
      }
      const int total = __shfl(incl, 63);
      if (total <= MAX_PEAKS) {
        int w = incl - c;
        for (int j = ak; j < bk; j++) {
          const int32_t pk = s_npk[lane * SEG_NMAX + j];
          if (pk >= 0) { s_pk[w] = pk; s_lvi[w] = lane * SEG_NMAX + j; w++; }
        }
        np = total;
        done = true;
      }
    }
  }
  if (G.stop > 0 && !done) {
    int k = 0, a = 0;
    while (!overflow) {
      const int cnt = s_cnt[k];
      const int32_t* pos = s_npos + k * SEG_NMAX;
      // b: first node j >= a of chain k that chain k+1 also visits
      int b = -1, jn = -1;
      bool search = false;
      if (k + 1 < SEG_K && s_cnt[k + 1] > 0) {
        const int js = __shfl(jstar, k), jns = __shfl(jnstar, k);
        if (js >= a) {
          b = js; jn = jns;
        } else if (js >= 0 && a < cnt) {
          const int t = jns + (a - js);
          if (t < s_cnt[k + 1] && s_npos[(k + 1) * SEG_NMAX + t] == pos[a]) { b = a; jn = t; }
          else search = true;                // not expected: fall back to the search
        }
      }
      if (search) {
        const int32_t* pn = s_npos + (k + 1) * SEG_NMAX;
        for (int j0 = a; j0 < cnt && b < 0; j0 += 64) {
          const int j = j0 + lane;
          const int f = (j < cnt) ? find_sorted(pn, s_cnt[k + 1], pos[j]) : -1;
          const uint64_t m = __ballot(f >= 0);
          if (m) {
            const int src = __ffsll((unsigned long long)m) - 1;
            b = j0 + src;
            jn = __shfl(f, src);
          }
        }
      }
      if (b >= 0) {
        emit(k, a, b);
        k += 1; a = jn;
        continue;
      }
      emit(k, a, cnt);
      if (overflow || cnt == 0) break;
      // chain k ended without meeting chain k+1: walk on directly until the
      // path lands on a position some later chain visits (or the walk ends)
      const int last = k * SEG_NMAX + cnt - 1;
      int64_t p = s_npk[last] >= 0 ? (int64_t)s_npk[last] + G.jump : (int64_t)s_npos[last] + G.win;
      bool joined = false;
      while (p < G.stop && !overflow) {
        for (int j = k + 1; j < SEG_K && !joined; j++) {
          const int c = s_cnt[j];
          if (c == 0 || s_npos[j * SEG_NMAX] > p || s_npos[j * SEG_NMAX + c - 1] < p) continue;
          const int f = find_sorted(s_npos + j * SEG_NMAX, c, p);
          if (f >= 0) { k = j; a = f; joined = true; }
        }
        if (joined) break;
        double best;
        int64_t bidx;
        tile_argmax(ds, stiles + (int64_t)slot * STILE_PER_SLOT, p, p + G.win, lane, best, bidx);
        if (best > .2) {
          if (np >= MAX_PEAKS) { overflow = true; break; }
          if (lane == 0) { s_pk[np] = (int32_t)bidx; s_lv[np] = best; s_lvi[np] = -1; }
          np++;
          p = bidx + G.jump;
        } else {
          p += G.win;
        }
      }
      if (!joined) break;
    }
  }
  __syncthreads();
  for (int q = lane; q < np; q += 64)
    if (s_lvi[q] >= 0) s_lv[q] = nlv[s_lvi[q]];
  __syncthreads();
  KSTAMP(3, 2);
  if (lane == 0) R->npeaks = np;
  for (int k = lane; k < np; k += 64) peaks[(int64_t)slot * MAX_PEAKS + k] = s_pk[k];
  if (overflow) {
    if (lane == 0) { R->status = FS_CRASH; R->nvsync = 0; R->log_flags = 0; }
    return;
  }
  // ---- determine_vsyncs -------------------------------------------------------
  int64_t vs[MAX_VSYNCS][3];
  int nf = 0;
  double med = 0, tol = 0;
  bool err = false;
  if (lane == 0) { R->nvsync = 0; R->status = FS_PENDING; R->log_flags = 0; }
  int ncand = 0;
  if (np >= 200) {
    // get_hsync_median: the in-range levels in peak order (compacted by ballot)
    int nh = 0;
    for (int j0 = 0; j0 < np; j0 += 64) {
      const int j = j0 + lane;
      const bool ok = j < np && inrange(s_lv[j], 0.6, 0.8);
      const uint64_t m = __ballot(ok);
      if (ok) s_tmp[nh + __popcll(m & ((1ull << lane) - 1ull))] = s_lv[j];
      nh += __popcll(m);
    }
    __syncthreads();
    // np.median: the middle order statistic(s), by radix select
    if (nh > 0) {
      med = (nh & 1) ? wave_kth(s_tmp, nh, nh / 2, lane, s_hist)
                     : (wave_kth(s_tmp, nh, nh / 2 - 1, lane, s_hist) + wave_kth(s_tmp, nh, nh / 2, lane, s_hist)) / 2.0;
    } else {
      med = __builtin_nan("");
    }
    // np.std over the list in peak order (numpy's pairwise order, on the wave)
    KSTAMP(3, 3);
    const double sdv = nh > 0 ? wave_np_std(s_tmp, nh, s_tmp + nh, lane) : __builtin_nan("");
    if (lane == 0) s_sd = sdv;
    __syncthreads();
    KSTAMP(3, 4);
    const double sd = s_sd;
    const double t2 = sd * 2;
    tol = (.01 > t2) ? .01 : t2;                     // Python max(t2, .01): keeps t2 unless .01 > t2
    // vsync candidates: peak > .9 after a peak below med - 2 tol
    for (int j0 = 0; j0 < np; j0 += 64) {
      const int j = j0 + lane;
      const bool c = j < np && s_lv[j] > .9 && (j ? s_lv[j - 1] : 1.0) < med - (tol * 2);
      const uint64_t m = __ballot(c);
      if (c) s_cand[ncand + __popcll(m & ((1ull << lane) - 1ull))] = j;
      ncand += __popcll(m);
    }
    __syncthreads();
    KSTAMP(3, 5);
  }
  if (lane != 0) return;
  if (np >= 200) {
    R->med_hsync = med;
    R->hsync_tol = tol;
    SyncView V{s_pk, s_lv, np, med, tol};
    for (int ci = 0; ci < ncand; ci++) {
      const int k = s_cand[ci];
      {
        if (k < 11) { R->status = FS_CRASH; return; }     // determine_field -> None, unpacked
        // determine_field (lddecode_core.py:544-588)
        int vote = 0;
        int64_t line0 = 0;
        bool have0 = false;
        int64_t gap1 = 0;
        for (int64_t q = k - 1; q > k - 20; q--) {
          if (V.regular(q, len, err)) {
            line0 = q; have0 = true;
            gap1 = V.peak(line0 + 1, err) - V.peak(line0, err);
            break;
          }
        }
        if (have0 && (double)gap1 > linelen * .75) vote -= 1;
        for (int64_t q = k; q < k + 20; q++) {
          if (V.regular(q, len, err)) {
            const int64_t gap2 = V.peak(q, err) - V.peak(q - 1, err);
            if ((double)gap2 > linelen * .75) vote += (C.system == 0) ? 1 : -1;
            break;
          }
        }
        if (C.system == 1) vote += 1;
        if (err) { R->status = FS_CRASH; return; }
        if (have0) {
          if (nf >= MAX_VSYNCS) { R->status = FS_CRASH; return; }
          vs[nf][0] = k; vs[nf][1] = line0; vs[nf][2] = vote;
          nf++;
        }
      }
    }
    if (nf >= 2) {
      // vote repair + line0 override + bool conversion, in place like the numpy array va
      int64_t orig[MAX_VSYNCS];
      for (int q = 0; q < nf; q++) orig[q] = vs[q][2];
      for (int q = 0; q < nf; q++) {
        if (vs[q][2] == 0) {
          vs[q][1] = -1;
          R->log_flags |= 1 << q;                     // print("vsync vote needed", i)
          if ((q < nf - 1) && orig[q + 1] != 0) vs[q][2] = -vs[q + 1][2];
          else if ((q >= 1) && orig[q - 1] != 0) vs[q][2] = -vs[q - 1][2];
        }
        if (vs[q][1] <= 0) vs[q][1] = vs[q][0] - ((C.system == 1) ? 6 : 7);
        vs[q][2] = vs[q][2] < 0 ? 1 : 0;
      }
    }
  }
  R->nvsync = nf;
  for (int q = 0; q < nf && q < MAX_VSYNCS; q++) {
    R->vsync[q][0] = (int32_t)vs[q][0]; R->vsync[q][1] = (int32_t)vs[q][1]; R->vsync[q][2] = (int32_t)vs[q][2];
  }
  SyncView V{s_pk, s_lv, np, med, tol};
  // ---- Field.__init__ branch (lddecode_core.py:909-933) ------------------------
  if (nf == 0) {
    R->nextfieldoffset = (int64_t)C.linelen * 200;
    R->status = FS_NO_VSYNC;
    return;
  }
  if (nf == 1 || np < vs[1][1] + 4) {
    const int64_t jumpto = V.peak(vs[0][1] - 10, err);
    if (err) { R->status = FS_CRASH; return; }
    R->nextfieldoffset = jumpto;
    if (jumpto == 0) {
      R->nextfieldoffset = (int64_t)C.linelen * 240;
      R->log_flags |= LDG_LOG_NO_VSYNC;               // "no/corrupt VSYNC found, jumping forward"
    }
    R->status = FS_SHORT;
    return;
  }
  const int64_t nfo = V.peak(vs[1][1] - 10, err);
  if (err) { R->status = FS_CRASH; return; }
  R->nextfieldoffset = nfo;
  R->tbcstart = nfo;
  R->istop = (int32_t)vs[0][2];
  R->linecount = C.frame_lines / 2 + (vs[0][2] ? 1 : 0);
  R->nlines = R->linecount + 4;
  R->status = FS_PENDING;
}

// ---------------------------------------------------------------------------
// compute_linelocs (lddecode_core.py:638-713), one wave per read.
// The reference's loop is a recurrence only through prevlinenum and the
// window of the last 25 accepted line lengths; both are prefix quantities, so
// it runs as: regular-peak compaction, accepted-gap compaction (ballots), the
// running median only where a peak's gap is not accepted (rank counting over
// <= 25 values), and a prefix sum of the line-number increments.  The gap
// fill is parallel except the tail extrapolation past the last valid line,
// which chains through earlier fills and stays sequential.
// grid: n_reads workgroups of 64 threads.
extern "C" __global__ __launch_bounds__(64) void ldg_k_linelocs(
    const int32_t* __restrict__ smap, const double* __restrict__ video, int64_t vread_stride, int64_t vchan_stride, SysConst C,
    FieldRec* __restrict__ recs, const int32_t* __restrict__ peaks, double* __restrict__ lines,
    int8_t* __restrict__ bad, const double* __restrict__ sst, const uint32_t* __restrict__ sbits) {
  prio_latency();

  __shared__ double s_key[LINENUM_SPAN];
  __shared__ uint8_t s_has[LINENUM_SPAN];
  __shared__ uint8_t s_orig[LINENUM_SPAN];
  __shared__ double s_lv[MAX_PEAKS];
  __shared__ int32_t s_pkl[MAX_PEAKS];
  __shared__ int32_t s_ridx[MAX_PEAKS];     // regular peaks, in order
  __shared__ int32_t s_nb[MAX_PEAKS];       // accepted gaps before regular peak m; < 0: m's gap accepted
  __shared__ int32_t s_num[MAX_PEAKS];      // line number of regular peak m
  __shared__ double s_agap[MAX_PEAKS];      // accepted gaps, in order
  __shared__ int s_flag;
  const int lane = threadIdx.x;
  const int slot = smap[blockIdx.x];
  FieldRec* R = recs + slot;
  if (R->status != FS_PENDING) return;
  const int np = R->npeaks;
  const int32_t* pkg = peaks + (int64_t)slot * MAX_PEAKS;
  const SyncSrc ds(sst, sbits, slot, C);
  for (int k = lane; k < LINENUM_SPAN; k += 64) { s_has[k] = 0; s_orig[k] = 0; }
  for (int k = lane; k < np; k += 64) { const int32_t p = pkg[k]; s_pkl[k] = p; s_lv[k] = ds[p]; }
  if (lane == 0) s_flag = 0;
  __syncthreads();
  const int32_t* pk = s_pkl;
  const double inl = (double)C.linelen;
  SyncView V{pk, s_lv, np, R->med_hsync, R->hsync_tol};
  const int v11 = R->vsync[1][1];
  const int64_t v01 = R->vsync[0][1];
  const int linecount = R->linecount;
  bool err = false;
  // 1. regular hsync peaks among [0, vsyncs[1][1])
  int nr = 0;
  for (int i0 = 0; i0 < v11; i0 += 64) {
    const int i = i0 + lane;
    const bool r = i < v11 && V.regular(i, 0x7fffffffffffLL, err);
    const uint64_t m = __ballot(r);
    if (r) s_ridx[nr + __popcll(m & ((1ull << lane) - 1ull))] = i;
    nr += __popcll(m);
  }
  __syncthreads();
  // 2. accepted gaps (inrange(gap / inlinelen, .98, 1.02)) and their running count
  int nacc = 0;
  for (int m0 = 0; m0 < nr; m0 += 64) {
    const int m = m0 + lane;
    bool acc = false;
    int64_t gap = 0;
    if (m >= 1 && m < nr) {
      gap = (int64_t)pk[s_ridx[m]] - pk[s_ridx[m - 1]];
      acc = inrange((double)gap / inl, .98, 1.02);
    }
    const uint64_t msk = __ballot(acc);
    const int rank = __popcll(msk & ((1ull << lane) - 1ull));
    if (m < nr) s_nb[m] = acc ? -1 - (nacc + rank) : nacc + rank;
    if (acc) s_agap[nacc + rank] = (double)gap;
    nacc += __popcll(msk);
  }
  __syncthreads();
  // 3. line-number increments; np.median(linelens[-25:]) only where it is used
  int64_t base_peak = 0;
  if (nr > 0) {
    base_peak = V.peak(v01, err);       // plist[vsyncs[0][1]] (first regular peak's reference)
    if (err) {
      if (lane == 0) R->status = FS_CRASH;
      return;
    }
  }
  for (int m0 = 0; m0 < nr; m0 += 64) {
    const int m = m0 + lane;
    if (m < nr) {
      const int nbv = s_nb[m];
      int inc;
      if (nbv < 0) {
        inc = 1;
      } else {
        // linelens = [inlinelen] + accepted gaps before m; median of the last 25
        const int nl_ = 1 + nbv;
        const int lo0 = nl_ > 25 ? nl_ - 25 : 0;
        const int wn = nl_ - lo0;
        auto L = [&](int q) { return q == 0 ? inl : s_agap[q - 1]; };
        auto kth = [&](int r) {
          for (int a = lo0; a < nl_; a++) {
            const double va = L(a);
            int lt = 0, le = 0;
            for (int b2 = lo0; b2 < nl_; b2++) { const double vb = L(b2); lt += vb < va; le += vb <= va; }
            if (lt <= r && r < le) return va;
          }
          return __builtin_nan("");
        };
        const double med = (wn & 1) ? kth(wn / 2) : (kth(wn / 2 - 1) + kth(wn / 2)) / 2.0;
        const int64_t ref = (m == 0) ? base_peak : (int64_t)pk[s_ridx[m - 1]];
        inc = (int)(int64_t)np_round((double)((int64_t)pk[s_ridx[m]] - ref) / med);
      }
      s_num[m] = inc;
    }
  }
  __syncthreads();
  // 4. inclusive prefix sum -> line numbers; dict assignment (last write wins)
  int carry = 0;
  for (int m0 = 0; m0 < nr; m0 += 64) {
    const int m = m0 + lane;
    int v = (m < nr) ? s_num[m] : 0;
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(v, o);
      if (lane >= o) v += t;
    }
    if (m < nr) s_num[m] = carry + v;
    carry += __shfl(v, 63);
  }
  __syncthreads();
  for (int m0 = 0; m0 < nr; m0 += 64) {
    const int m = m0 + lane;
    if (m < nr) {
      const int key = s_num[m] + LINENUM_OFF;
      if (key < 0 || key >= LINENUM_SPAN) {
        s_flag = 1;
      } else if (m == nr - 1 || s_num[m + 1] != s_num[m]) {
        s_key[key] = (double)pk[s_ridx[m]];
        s_has[key] = 1;
        s_orig[key] = 1;
      }
    }
  }
  __syncthreads();
  if (s_flag) {
    if (lane == 0) R->status = FS_LINELOCS;
    return;
  }
  // 5. fill missing line numbers 1..linecount+4: interpolation / head
  //    extrapolation in parallel (they read original entries only)
  for (int l = 1 + lane; l < linecount + 5; l += 64) {
    const int kl = l + LINENUM_OFF;
    if (s_orig[kl]) continue;
    int pv = -100000, nv = -100000;
    for (int q = l; q > -10; q--) if (s_orig[q + LINENUM_OFF]) { pv = q; break; }
    for (int q = l; q < linecount + 1; q++) if (s_orig[q + LINENUM_OFF]) { nv = q; break; }
    if (nv == -100000) {
      if (pv == -100000) s_flag = 1;    // linelocs[None] KeyError
      continue;                         // tail: step 6
    }
    double v;
    if (pv == -100000) {
      v = s_key[nv + LINENUM_OFF] - (inl * (double)(nv - l));
    } else {
      const double step = (s_key[nv + LINENUM_OFF] - s_key[pv + LINENUM_OFF]) / (double)(nv - pv);
      v = s_key[pv + LINENUM_OFF] + (step * (double)(l - pv));
    }
    s_key[kl] = v;
    s_has[kl] = 1;
  }
  __syncthreads();
  if (s_flag) {
    if (lane == 0) R->status = FS_LINELOCS;
    return;
  }
  // 6. tail extrapolation past the last valid line (uses earlier fills), in order
  if (lane == 0) {
    for (int l = 1; l < linecount + 5; l++) {
      const int kl = l + LINENUM_OFF;
      if (s_has[kl]) continue;
      int pv = -100000;
      for (int q = l; q > -10; q--) if (s_orig[q + LINENUM_OFF]) { pv = q; break; }
      const int kprev = pv - 1 + LINENUM_OFF;
      if (!s_has[kprev]) { s_flag = 1; break; }   // linelocs2[prev_valid - 1] KeyError
      const double step = s_key[pv + LINENUM_OFF] - s_key[kprev];
      s_key[kl] = s_key[pv + LINENUM_OFF] + (step * (double)(l - pv));
      s_has[kl] = 1;
    }
  }
  __syncthreads();
  if (s_flag) {
    if (lane == 0) R->status = FS_LINELOCS;
    return;
  }
  double* L1 = lines + (int64_t)slot * LINES_STRIDE + LL1 * MAX_LINES;
  int8_t* B1 = bad + (int64_t)slot * MAX_LINES;
  for (int l = 1 + lane; l < linecount + 5; l += 64) {
    L1[l - 1] = s_key[l + LINENUM_OFF];
    B1[l - 1] = (l - 1 < 10) ? 0 : (s_orig[l + LINENUM_OFF] ? 0 : 1);
  }
}

// ---------------------------------------------------------------------------
// refine_linelocs_hsync (lddecode_core.py:715-787), part 1: the per-line
// crossing search and bad-line tests, one wave per line.  Writes the line's
// refined location to LL2 and its flag to bad[] (0 ok, 1 bad, 2 the reference
// raises on this line).  grid: n_reads * MAX_LINES workgroups of 64 threads.
// demod_05 is read from the channel the demod stores.
namespace {

template <class Src>
__device__ void hsync_line(const Src& d05, int64_t len, const SysConst& C, int i, double v, bool lb, int lane,
                           double* s_tmp, double& out, int& flag) {
  const double fr = C.freq;
  auto hz = [&](double ire) { return C.ire0 + (C.hz_ire * ire); };
  if (i < 9) v -= 200;
  const double ll1 = v;
  double zc;
  const int rc = wave_calczc_pf<7>(d05, len, v, hz(-20), 400, lane, &zc);
  if (rc < 0) { out = v; flag = 2; return; }
  if (rc == 0 && !lb) {
    v = zc;
    if (i >= 10) {
      int64_t a1, b1, ah, bh, ab, bb;
      py_slice(py_int(ll1 - (fr * 2)), py_int(ll1 + (fr * 2)), len, a1, b1);
      py_slice(py_int(zc - (fr * 1)), py_int(zc + (fr * 3)), len, ah, bh);
      py_slice(py_int(zc + (fr * 1)), py_int(zc + (fr * 3)), len, ab, bb);
      // evaluation order of the reference's `or` chain; an empty window raises
      bool isbad = false, raised = false;
      auto grp = [&](int64_t a, int64_t b, double lo, double hi) -> bool {
        if (a >= b) { raised = true; return true; }
        double mn, mx;
        wave_minmax2_np(d05, a, b, lane, mn, mx);
        if (mn < lo) return true;
        return mx > hi;
      };
      if (grp(ah, bh, hz(-60), hz(20))) isbad = true;
      else if (grp(a1, b1, hz(-60), hz(100))) isbad = true;
      else if (grp(ab, bb, hz(-10), hz(10))) isbad = true;
      if (raised) { out = v; flag = 2; return; }
      if (isbad) {
        lb = true;
      } else {
        const int64_t wl = bh - ah;
        int64_t lo, hi;
        py_slice(0, 20, wl, lo, hi);
        if (lane < hi - lo) s_tmp[lane] = d05[ah + lo + lane];
        __syncthreads();
        const double low = np_mean(s_tmp, (int)(hi - lo));
        __syncthreads();
        py_slice(100, 120, wl, lo, hi);
        if (lane < hi - lo) s_tmp[lane] = d05[ah + lo + lane];
        __syncthreads();
        const double high = np_mean(s_tmp, (int)(hi - lo));
        double zc2;
        const int rc2 = wave_calczc_pf<3>(d05 + ah, wl, 0, (low + high) / 2, wl, lane, &zc2);
        if (rc2 != 0) { out = v; flag = 2; return; }   // None += ... -> TypeError
        zc2 += ((double)py_int(zc) - (fr * 1));
        if (fabs(zc2 - zc) < (fr / 4)) v = zc2;
        else lb = true;
      }
    }
  } else {
    lb = true;
  }
  out = v;
  flag = lb ? 1 : 0;
}
}  // namespace

extern "C" __global__ __launch_bounds__(64) void ldg_k_hsync_lines(
    const int32_t* __restrict__ smap, const double* __restrict__ video, int64_t vread_stride, int64_t vchan_stride,
    SysConst C, FieldRec* __restrict__ recs, double* __restrict__ lines, int8_t* __restrict__ bad) {
  prio_latency();

  __shared__ double s_tmp[20];
  const int lane = threadIdx.x;
  const int slot = smap[blockIdx.y];
  const int i = blockIdx.x;
  FieldRec* R = recs + slot;
  const double* L1 = lines + (int64_t)slot * LINES_STRIDE + LL1 * MAX_LINES;
  double* L2 = lines + (int64_t)slot * LINES_STRIDE + LL2 * MAX_LINES;
  int8_t* B = bad + (int64_t)slot * MAX_LINES;
  // the record, the line's location and flag in one memory round trip
  const int status = R->status, nl = R->nlines;
  const int64_t len = R->n_out;
  const double v = L1[i];
  const int lbi = B[i];
  asm volatile("" ::"v"(v), "v"(status), "v"(nl), "v"(lbi));
  if (status != FS_PENDING) return;
  if (i >= nl) return;
  // demod_05 as the demod stored it
  const double* d05 = video + (int64_t)slot * vread_stride + (int64_t)CH_05 * vchan_stride;
  const bool lb = lbi != 0;
  double out;
  int flag;
  hsync_line(d05, len, C, i, v, lb, lane, s_tmp, out, flag);
  if (lane == 0) { L2[i] = out; B[i] = (int8_t)flag; }
}

// refine_linelocs_hsync, part 2 (per read): bad-line extrapolation and the
// two end fix-ups, sequential as in the reference, in LDS on thread 0.
extern "C" __global__ __launch_bounds__(256) void ldg_k_hsync_field(const int32_t* __restrict__ smap, SysConst C,
                                                                   FieldRec* __restrict__ recs,
                                                                   double* __restrict__ lines,
                                                                   int8_t* __restrict__ bad) {
  prio_latency();

  __shared__ double s_v[MAX_LINES];
  __shared__ int8_t s_bad[MAX_LINES];
  __shared__ int s_err;
  const int tid = threadIdx.x;
  const int slot = smap[blockIdx.x];
  FieldRec* R = recs + slot;
  if (R->status != FS_PENDING) return;
  const int nl = R->nlines;
  double* L2 = lines + (int64_t)slot * LINES_STRIDE + LL2 * MAX_LINES;
  int8_t* B = bad + (int64_t)slot * MAX_LINES;
  if (tid == 0) s_err = 0;
  __syncthreads();
  for (int i = tid; i < nl; i += 256) {
    s_v[i] = L2[i];
    const int8_t f = B[i];
    s_bad[i] = f;
    if (f == 2) atomicOr(&s_err, 1);
  }
  __syncthreads();
  if (s_err) {
    if (tid == 0) R->status = FS_LINELOCS;
    return;
  }
  const double fr = C.freq;
  if (tid == 0) {
    for (int i = 0; i < nl; i++) {
      if (i < 10) s_v[i] += 4.72 * fr;
      if (i > 10 && s_bad[i]) {
        const double gap = s_v[i - 1] - s_v[i - 2];
        s_v[i] = s_v[i - 1] + gap;
      }
    }
    const double lo = C.linelen - (fr * .2), hi = C.linelen + (fr * .2);
    for (int i = 9; i >= 0; i--) {
      double gap = s_v[i + 1] - s_v[i];
      if (!inrange(gap, lo, hi)) gap = C.linelen;
      s_v[i] = s_v[i + 1] - gap;
    }
    for (int i = nl - 10; i < nl; i++) {
      double gap = s_v[i] - s_v[i - 1];
      if (!inrange(gap, lo, hi)) gap = C.linelen;
      s_v[i] = s_v[i - 1] + gap;
    }
  }
  __syncthreads();
  for (int i = tid; i < nl; i += 256) { L2[i] = s_v[i]; B[i] = s_bad[i]; }
}

// ---------------------------------------------------------------------------
// Philips VBI decode (lddecode_core.py:814-884).  grid: n_reads x 192; wave w
// decodes code line w (decodephillipscode), thread 0 then interprets the three.
// Each crossing search issues its loads at once (wave_calczc_pf), together with
// the previous crossing's bit sample, so a crossing costs ~one memory latency.
extern "C" __global__ __launch_bounds__(192) void ldg_k_philips(
    const int32_t* __restrict__ smap, const double* __restrict__ video, int64_t vread_stride, int64_t vchan_stride, SysConst C,
    FieldRec* __restrict__ recs, const double* __restrict__ lines, const ReadDesc* __restrict__ reads) {
  prio_latency();
  __shared__ int32_t s_code[3][6];
  __shared__ int32_t s_ok[3];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int slot = smap[blockIdx.x];
  FieldRec* R = recs + slot;
  if (R->status != FS_PENDING) return;
  const double* dm = video + (int64_t)slot * vread_stride + (int64_t)CH_DEMOD * vchan_stride;
  const int64_t len = R->n_out;
  const double* L2 = lines + (int64_t)slot * LINES_STRIDE + LL2 * MAX_LINES;
  const double fr = C.freq;
  const double thr = C.ire0 + (C.hz_ire * 50);
  {
    // the three code lines' searches stay within ~60 us of their line starts; past the
    // read's video cut the read is decoded in full (uniform over the workgroup)
    double hi = 0.0;
    for (int q = 0; q < 3; q++) hi = fmax(hi, L2[C.codelines[q]]);
    if (!(hi + 80 * fr < (double)reads[slot].vcut)) {
      if (tid == 0) R->status = FS_VCUT;
      return;
    }
  }
  {
    int ok = 0;
    const int ln = C.codelines[w];
    const double start = L2[ln];
    double cur;
    int rc = wave_calczc_pf<8>(dm, len, (double)py_int(start + 2 * fr), thr, py_int(12 * fr), lane, &cur);
    int n = 0;
    uint32_t bits = 0;                        // bit n at position 23 - n (n < 24)
    double prevz = 0, gmin = __builtin_inf(), gmax = -__builtin_inf();
    bool crash = false;
    while (rc == 0) {
      int64_t bi;
      if (!py_index(py_int(cur - 0.5 * fr), len, bi)) { crash = true; break; }
      const double vb = dm[bi];               // in flight with the next search's loads
      if (n > 0) {
        const double g = (cur - prevz) / fr;
        gmin = fmin(gmin, g); gmax = fmax(gmax, g);
      }
      prevz = cur;
      const double c0 = cur;
      if (n + 1 > 100000) { if (n < 24 && vb < thr) bits |= 1u << (23 - n); n++; break; }
      rc = wave_calczc_pf<1>(dm, len, c0 + 1.9 * fr, thr, py_int(0.2 * fr), lane, &cur);
      if (n < 24 && vb < thr) bits |= 1u << (23 - n);
      n++;
    }
    if (rc < 0 || crash) ok = -1;
    else if (n == 24 && gmin > 1.85 && gmax < 2.15) {
      ok = 1;
      if (lane == 0)
        for (int b = 0; b < 6; b++) s_code[w][b] = (int32_t)((bits >> (20 - 4 * b)) & 15u);
    }
    if (lane == 0) s_ok[w] = ok;
  }
  __syncthreads();
  if (tid != 0) return;
  for (int q = 0; q < 3; q++)
    if (s_ok[q] < 0) { R->status = FS_CRASH; return; }   // IndexError outside the reference's try
  int minutes = VBI_NONE, seconds = VBI_NONE, clvframe = VBI_NONE, framenr = VBI_NONE, statusv = VBI_NONE;
  int isclv = 0;
  for (int q = 0; q < 3; q++) {
    R->linecode_ok[q] = s_ok[q];
    for (int b = 0; b < 6; b++) R->linecode[q][b] = s_ok[q] ? s_code[q][b] : 0;
    if (!s_ok[q]) continue;
    const int32_t* lc = s_code[q];
    if (lc[0] == 15 && lc[2] == 13) {
      minutes = 60 * lc[1] + lc[4] * 10 + lc[5];
      isclv = 1;
    } else if (lc[0] == 15) {
      framenr = (lc[1] & 7) * 10000 + (lc[2] * 1000) + (lc[3] * 100) + (lc[4] * 10) + lc[5];
    } else {
      const int h = (lc[0] << 20) | (lc[1] << 16) | (lc[2] << 12) | (lc[3] << 8) | (lc[4] << 4) | lc[5];
      if (lc[2] == 0xE) {
        seconds = (lc[1] - 10) * 10 + lc[3];
        clvframe = lc[4] * 10 + lc[5];
        isclv = 1;
      }
      const int htop = h >> 12;
      if (htop == 0x8dc || htop == 0x8ba) statusv = h;
      if (h == 0x87ffff) isclv = 1;
    }
  }
  R->vbi_minutes = minutes; R->vbi_seconds = seconds; R->vbi_clvframe = clvframe;
  R->vbi_framenr = framenr; R->vbi_status = statusv; R->vbi_isclv = isclv;
}
