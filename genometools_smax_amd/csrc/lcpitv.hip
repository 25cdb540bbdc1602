// lcpitv.hip -- the lcp-interval tree on the GPU and the generic bottom-up
// visitor replay, gfx950.
//
// The reference walks the LCP array once with an explicit stack
// (gt_esa_bottomup, src/match/esa-bottomup.c:116-273), popping every
// lcp-interval [lb..rb] of depth l > 0 at rb and calling the visitor's
// leaf-edge / branching-edge / lcp-interval callbacks.  Here the tree is
// computed data-parallel from all-nearest-smaller-value (ANSV) searches:
//
//   * row k with v = LCP[k] > 0 is the leftmost l-index of an interval iff
//     the nearest p < k with LCP[p] <= v has LCP[p] < v; then lb = p and
//     rb = q - 1 for the nearest q > k with LCP[q] < v (LCP[0] = LCP[N] = 0);
//   * its father has depth max(LCP[lb], LCP[rb+1]) and lb = the nearest
//     p' < lb with LCP[p'] < LCP[lb] when LCP[lb] is the larger (else lb);
//   * leaf idx hangs (when LCP[idx+1] <= LCP[idx]) below the interval of
//     depth LCP[idx] whose lb is the nearest p < idx with LCP[p] < LCP[idx].
//
// Each search climbs a 64-ary min hierarchy over the exact LCP array (u32)
// and descends again: at most 63 reads per level, 6 levels for 10^10 rows.
// One thread per row; the intervals are compacted and radix-sorted into pop
// order (rb ascending, depth descending).  The tree stays in HBM
// (GtLcpitvPlan); the visitor's event stream is generated there too, every
// event at its position in the reference's order, no stack and no replay
// loop (li_events_*): per row idx (X = LCP[idx], Y = LCP[idx+1]) the
// traversal emits exactly one leaf edge, then for every interval popped at
// idx (pop order) its lcp-interval and branching-edge events, so with
// P(idx) = #intervals with rb < idx the leaf of row idx sits at
// idx + 2 P(idx) and popped interval r of row idx at idx + 2 P(idx) + 1 + 2r.
// The host entry points download the events in chunks and call the
// visitor.
#include <hip/hip_runtime.h>
#include <vector>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gt_lcpitv_hip.h"
#include "smax_internal.h"

static void li_seterr(char *errbuf, size_t errlen, const char *fmt, ...) {
  if (errbuf == NULL || errlen == 0) return;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(errbuf, errlen, fmt, ap);
  va_end(ap);
}

#define LICHK(call)                                                          \
  do {                                                                       \
    hipError_t e_ = (call);                                                  \
    if (e_ != hipSuccess) {                                                  \
      li_seterr(errbuf, errlen, "%s: %s (%s:%d)", #call, hipGetErrorString(e_), \
                __FILE__, __LINE__);                                         \
      goto fail;                                                             \
    }                                                                        \
  } while (0)

#define LI_MAXLEV 8

struct LiLevels {
  const uint32_t *lv[LI_MAXLEV];   // lv[0] = exact LCP (N+1), lv[i] = mins of 64 of lv[i-1]
  uint64_t n[LI_MAXLEV];
  int nlev;
};

// ------------------------------------------------------------ kernels

// grid-stride loop over [0, n) of a 1-D launch (li_blocks caps the grid)
#define LI_FOR(i, n)                                                          \
  for (uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x,         \
                i##_stride = (uint64_t) gridDim.x * blockDim.x;               \
       i < (n); i += i##_stride)

__global__ void __launch_bounds__(256) li_expand_kernel(const uint8_t *lcp, uint64_t N,
                                                        uint32_t *X) {
  LI_FOR(k, N + 1) X[k] = (k == 0 || k == N) ? 0u : (uint32_t) lcp[k];
}

__global__ void __launch_bounds__(256) li_llv_kernel(const GtSmaxLlv *llv, uint64_t numllv,
                                                     const uint8_t *lcp, uint64_t N, uint32_t *X,
                                                     uint32_t *err) {
  LI_FOR(e, numllv) {
    const uint64_t pos = llv[e].position, v = llv[e].value;
    if (pos < 1 || pos >= N) continue;
    if (v > 0xfffffffeull) atomicOr(err, 1u);
    if (lcp[pos] != 255) atomicOr(err, 2u);
    X[pos] = (uint32_t) v;
  }
}

__global__ void __launch_bounds__(256) li_min64_kernel(const uint32_t *in, uint64_t n_in,
                                                       uint32_t *out, uint64_t n_out) {
  LI_FOR(g, n_out) {
    uint32_t m = 0xffffffffu;
    const uint64_t b = g * 64, e = b + 64 < n_in ? b + 64 : n_in;
    for (uint64_t i = b; i < e; i++) m = in[i] < m ? in[i] : m;
    out[g] = m;
  }
}

__device__ __forceinline__ bool li_ok(uint32_t x, uint32_t v, bool strict) {
  return strict ? x < v : x <= v;
}

// The searches read a level's whole 64-entry block at once (16 independent
// 16-byte loads, then a bit mask of the entries that qualify) instead of one
// dependent load per entry: a search that climbs the hierarchy paid up to
// 64 round trips per level, and a wave waits for its slowest lane
// (li_write_kernel 14.7 -> 9.2 ms, li_count_kernel 5.2 -> 3.4 ms at C2,
// profiles/s7/kernel_stats_lcpitv_c2*.csv; checking the 16 bytes next to
// the row first changed nothing: the slowest lane of a wave, on a long
// search, sets its time).  Levels are allocated LI_PAD
// entries long past their end; bits past it are masked off.
#define LI_PAD 64
__device__ __forceinline__ uint64_t li_block_mask(const uint32_t *lv, uint64_t b, uint64_t n,
                                                  uint32_t v, bool strict) {
  const uint4 *p = reinterpret_cast<const uint4 *>(lv + b);
  uint4 t[16];
#pragma unroll
  for (int j = 0; j < 16; j++) t[j] = p[j];
  uint64_t m = 0;
#pragma unroll
  for (int j = 0; j < 16; j++) {
    m |= (uint64_t) (li_ok(t[j].x, v, strict) ? 1u : 0u) << (4 * j);
    m |= (uint64_t) (li_ok(t[j].y, v, strict) ? 1u : 0u) << (4 * j + 1);
    m |= (uint64_t) (li_ok(t[j].z, v, strict) ? 1u : 0u) << (4 * j + 2);
    m |= (uint64_t) (li_ok(t[j].w, v, strict) ? 1u : 0u) << (4 * j + 3);
  }
  if (n - b < 64) m &= (1ull << (n - b)) - 1;
  return m;
}

// nearest p < k with X[p] < v (strict) / <= v; X[0] == 0 guarantees one
// for v > 0 (strict) and any v (<=)
__device__ static uint64_t li_prev(const LiLevels &L, uint64_t k, uint32_t v, bool strict) {
  uint64_t i = k, p = 0;
  int lev = 0;
  for (;;) {
    const uint64_t b = (i >> 6) << 6;
    const uint64_t below = i - b;   // entries [b, i)
    const uint64_t m = below ? li_block_mask(L.lv[lev], b, L.n[lev], v, strict) &
                                   ((below >= 64 ? 0ull : (1ull << below)) - 1ull)
                             : 0ull;
    if (m) { p = b + 63 - (uint64_t) __builtin_clzll(m); break; }
    if (lev + 1 >= L.nlev || i < 64) return 0;   // only row 0 is left
    i >>= 6;
    lev++;
  }
  while (lev > 0) {                // last child of p whose subtree qualifies
    lev--;
    const uint64_t b = p << 6;
    const uint64_t m = li_block_mask(L.lv[lev], b, L.n[lev], v, strict);
    p = b + 63 - (uint64_t) __builtin_clzll(m);
  }
  return p;
}

// nearest q > k with X[q] < v (X[N] == 0 guarantees one for v > 0)
__device__ static uint64_t li_next(const LiLevels &L, uint64_t k, uint32_t v) {
  uint64_t i = k, p = 0;
  int lev = 0;
  for (;;) {
    const uint64_t b = (i >> 6) << 6;
    const uint64_t upto = i - b;    // entries (i, b + 64)
    const uint64_t m = upto >= 63 ? 0ull
                                  : li_block_mask(L.lv[lev], b, L.n[lev], v, true) & ~((2ull << upto) - 1ull);
    if (m) { p = b + (uint64_t) __builtin_ctzll(m); break; }
    if (lev + 1 >= L.nlev) return L.n[0] - 1;    // row N
    i >>= 6;
    lev++;
  }
  while (lev > 0) {                // first child of p whose subtree qualifies
    lev--;
    const uint64_t b = p << 6;
    p = b + (uint64_t) __builtin_ctzll(li_block_mask(L.lv[lev], b, L.n[lev], v, true));
  }
  return p;
}

// workgroup-wide exclusive prefix; *total = sum
__device__ __forceinline__ uint32_t li_block_excl(uint32_t v, uint32_t *total) {
  __shared__ uint32_t sW[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(incl, d, 64);
    if (lane >= d) incl += o;
  }
  if (lane == 63) sW[wave] = incl;
  __syncthreads();
  uint32_t wo = 0;
  for (int w = 0; w < wave; w++) wo += sW[w];
  *total = sW[0] + sW[1] + sW[2] + sW[3];
  return wo + incl - v;
}

// row k (1 <= k < N) opens an interval: leftmost l-index
__device__ __forceinline__ bool li_leftmost(const LiLevels &L, uint64_t k, uint64_t N,
                                            uint64_t *lb) {
  if (k < 1 || k >= N) return false;
  const uint32_t v = L.lv[0][k];
  if (v == 0) return false;
  const uint64_t p = li_prev(L, k, v, false);
  *lb = p;
  return L.lv[0][p] < v;
}

// groups of 256 rows, group-stride over a capped grid (every thread of a
// workgroup runs the same number of groups: li_block_excl synchronises)
__global__ void __launch_bounds__(256) li_count_kernel(LiLevels L, uint64_t N, uint64_t ngroups,
                                                       uint32_t *wg_cnt) {
  for (uint64_t g = blockIdx.x; g < ngroups; g += gridDim.x) {
    const uint64_t k = g * 256 + threadIdx.x;
    uint64_t lb;
    uint32_t tot;
    (void) li_block_excl(li_leftmost(L, k, N, &lb) ? 1u : 0u, &tot);
    if (threadIdx.x == 0) wg_cnt[g] = tot;
    __syncthreads();                 // sW is reused by the next group
  }
}

__device__ __forceinline__ void li_write_one(const LiLevels &L, uint64_t k, uint64_t lb,
                                             uint64_t pos, uint64_t *rec, uint64_t *key,
                                             uint64_t *idx) {
  const uint32_t v = L.lv[0][k];
  const uint64_t q = li_next(L, k, v);
  const uint32_t xl = L.lv[0][lb], xq = L.lv[0][q];
  const uint32_t fl = xl > xq ? xl : xq;
  uint64_t flb = lb;
  if (fl == 0) flb = 0;
  else if (xl >= xq) flb = li_prev(L, lb, xl, true);
  uint64_t *r = rec + 5 * pos;
  r[0] = v;
  r[1] = lb;
  r[2] = q - 1;
  r[3] = fl;
  r[4] = flb;
  key[pos] = q - 1;   // rb (past 2^32 rows li_key_kernel rewrites the keys)
  idx[pos] = pos;
}

// records (lcp, lb, rb, fatherlcp, fatherlb) in row order of their
// leftmost l-index, and the pop-order sort key rb alone: within a run of
// equal rb the records stay in row order (lcp ascending) through the stable
// sort, and li_gather_rev_kernel reverses each run into pop order -- so this
// kernel must keep writing in row order
__global__ void __launch_bounds__(256) li_write_kernel(LiLevels L, uint64_t N, uint64_t ngroups,
                                                       const uint64_t *wg_off, uint64_t *rec,
                                                       uint64_t *key, uint64_t *idx) {
  for (uint64_t g = blockIdx.x; g < ngroups; g += gridDim.x) {
    const uint64_t k = g * 256 + threadIdx.x;
    uint64_t lb = 0;
    const bool open = li_leftmost(L, k, N, &lb);
    uint32_t tot;
    const uint64_t pos = wg_off[g] + li_block_excl(open ? 1u : 0u, &tot);
    __syncthreads();                 // sW is reused by the next group
    if (open) li_write_one(L, k, lb, pos, rec, key, idx);
  }
}


// keys of the two-pass sort (rb >= 2^32): pass 0 ~lcp, pass 1 rb, of the
// records in the current permutation
__global__ void __launch_bounds__(256) li_key_kernel(const uint64_t *rec, const uint64_t *perm,
                                                     uint64_t n, int pass, uint64_t *key) {
  LI_FOR(i, n) {
    const uint64_t *r = rec + 5 * perm[i];
    key[i] = pass == 0 ? (uint64_t) (0xffffffffu - (uint32_t) r[0]) : r[2];
  }
}

// the records sorted by rb alone into pop order: each run of equal rb is in
// row order of its intervals' first l-index, i.e. lcp ascending (an outer
// interval's l-indices lie at or before an inner one's lb), and the pops
// take the deepest first -- the run reversed
__global__ void __launch_bounds__(256) li_gather_rev_kernel(const uint64_t *rec, const uint64_t *idx,
                                                            const uint64_t *rb,
                                                            const uint32_t *before, uint64_t n,
                                                            uint64_t *out) {
  LI_FOR(i, n) {
    const uint64_t v = rb[i];
    const uint64_t dst = (uint64_t) before[v] + before[v + 1] - 1 - i;
    const uint64_t *r = rec + 5 * (uint64_t) idx[i];
    uint64_t *w = out + 5 * dst;
#pragma unroll
    for (int f = 0; f < 5; f++) w[f] = r[f];
  }
}

__global__ void __launch_bounds__(256) li_gather_kernel(const uint64_t *rec, const uint64_t *idx,
                                                        uint64_t n, uint64_t *out) {
  LI_FOR(i, n) {
    const uint64_t *r = rec + 5 * (uint64_t) idx[i];
    uint64_t *w = out + 5 * i;
#pragma unroll
    for (int f = 0; f < 5; f++) w[f] = r[f];
  }
}

// ------------------------------------------------------------ events

// rows [lo, hi) of the sorted intervals: first index whose rb >= v
__device__ __forceinline__ uint64_t li_lower_rb(const uint64_t *itv, uint64_t n, uint64_t v) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (itv[5 * mid + 2] < v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// intervals with rb < v: the plan's prefix array (one load) when it has
// one, else a binary search over the pop-ordered records (26 dependent
// loads at C2, in four kernels: 16.5 ms of the events pass, profiles/s7/)
__device__ __forceinline__ uint64_t li_before(const uint32_t *C, const uint64_t *itv, uint64_t n,
                                              uint64_t v) {
  return C != nullptr ? (uint64_t) C[v] : li_lower_rb(itv, n, v);
}

// the prefix array's input: at rb + 1 of the last interval of each run of
// equal rb (rb sorted), the number of intervals up to it (a max-scan fills
// the rest)
__global__ void __launch_bounds__(256) li_rb_marks_kernel(const uint64_t *rb, uint64_t n,
                                                          uint32_t *D) {
  LI_FOR(j, n) {
    if (j + 1 == n || rb[j + 1] != rb[j]) D[rb[j] + 1] = (uint32_t) (j + 1);
  }
}

// event positions of root edges that consume the reference's
// firstedgefromroot flag (leaf edges to the root attached in step 1 and
// branching edges to the root of pops); the first one in stream order gets
// firstsucc = 1 (src/match/esa-bottomup.c:134-141)
__global__ void __launch_bounds__(256) li_rootfirst_leaf_kernel(LiLevels L, uint64_t N,
                                                                const uint64_t *itv, uint64_t nitv,
                                                                const uint32_t *C,
                                                                unsigned long long *first) {
  LI_FOR(idx, N) {
    const uint32_t X = L.lv[0][idx], Y = L.lv[0][idx + 1];
    if (X != 0 || Y > X) continue;
    const uint64_t pos = idx + 2 * li_before(C, itv, nitv, idx);
    atomicMin(first, (unsigned long long) pos);
  }
}

__global__ void __launch_bounds__(256) li_rootfirst_itv_kernel(const uint64_t *itv, uint64_t nitv,
                                                               const uint32_t *C,
                                                               unsigned long long *first) {
  LI_FOR(j, nitv) {
    const uint64_t *r = itv + 5 * j;
    if (r[3] != 0) continue;
    const uint64_t g = li_before(C, itv, nitv, r[2]);
    const uint64_t pos = r[2] + 2 * g + 1 + 2 * (j - g) + 1;
    atomicMin(first, (unsigned long long) pos);
  }
}

// leaf edge of row idx: (0, firstsucc, fd, flb, leafnumber, 0, 0)
template <typename SufT>
__global__ void __launch_bounds__(256) li_events_leaf_kernel(LiLevels L, uint64_t N,
                                                             const uint64_t *itv, uint64_t nitv,
                                                             const uint32_t *C, const void *suf,
                                                             const unsigned long long *first,
                                                             uint64_t *ev) {
  LI_FOR(idx, N) {
    const uint32_t X = L.lv[0][idx], Y = L.lv[0][idx + 1];
    const uint64_t pos = idx + 2 * li_before(C, itv, nitv, idx);
    uint64_t e1, e2, e3;
    if (Y <= X) {            // attached to the interval of depth X holding idx
      e1 = (X == 0 && pos == *first) ? 1u : 0u;
      e2 = X;
      e3 = X == 0 ? 0 : li_prev(L, idx, X, true);
    } else {                 // firstsucc leaf of the new interval (Y, idx)
      e1 = 1;
      e2 = Y;
      e3 = idx;
    }
    const uint64_t e4 = suf == nullptr ? 0 : (uint64_t) reinterpret_cast<const SufT *>(suf)[idx];
    uint64_t *w = ev + 7 * pos;   // 16-byte pieces, as li_events_itv_kernel
    if ((pos & 1) == 0) {
      reinterpret_cast<ulonglong2 *>(w)[0] = make_ulonglong2(0, e1);
      reinterpret_cast<ulonglong2 *>(w)[1] = make_ulonglong2(e2, e3);
      reinterpret_cast<ulonglong2 *>(w)[2] = make_ulonglong2(e4, 0);
      w[6] = 0;
    } else {
      w[0] = 0;
      reinterpret_cast<ulonglong2 *>(w + 1)[0] = make_ulonglong2(e1, e2);
      reinterpret_cast<ulonglong2 *>(w + 1)[1] = make_ulonglong2(e3, e4);
      reinterpret_cast<ulonglong2 *>(w + 1)[2] = make_ulonglong2(0, 0);
    }
  }
}

// popped interval j: (2, 0, lcp, lb, rb, 0, 0) then its branching edge
// (1, firstsucc, fd, flb, sd, slb, srb); a father that is new at rb (same
// lb, pushed after the pops) gets the firstsucc edge with its own lb
__global__ void __launch_bounds__(256) li_events_itv_kernel(const uint64_t *itv, uint64_t nitv,
                                                            const uint32_t *C,
                                                            const unsigned long long *first,
                                                            uint64_t *ev) {
  LI_FOR(j, nitv) {
    const uint64_t *r = itv + 5 * j;
    const uint64_t g = li_before(C, itv, nitv, r[2]);
    const uint64_t pos = r[2] + 2 * g + 1 + 2 * (j - g);
    const uint64_t r0 = r[0], r1 = r[1], r2 = r[2], r3 = r[3], r4 = r[4];
    const bool newfather = r3 > 0 && r4 == r1;
    // the pop record and its branching edge: 14 consecutive words, stored
    // as 16-byte pieces (8-byte stores: 9.0 ms at C2, profiles/s7/)
    const uint64_t e[14] = {2, 0, r0, r1, r2, 0, 0,
                            1, newfather ? 1u : ((r3 == 0 && pos + 1 == *first) ? 1u : 0u), r3,
                            newfather ? r1 : r4, r0, r1, r2};
    uint64_t *w = ev + 7 * pos;
    if ((pos & 1) == 0) {   // 56 * pos: 16-byte aligned
#pragma unroll
      for (int q = 0; q < 7; q++)
        reinterpret_cast<ulonglong2 *>(w)[q] = make_ulonglong2(e[2 * q], e[2 * q + 1]);
    } else {
      w[0] = e[0];
#pragma unroll
      for (int q = 0; q < 6; q++)
        reinterpret_cast<ulonglong2 *>(w + 1)[q] = make_ulonglong2(e[2 * q + 1], e[2 * q + 2]);
      w[13] = e[13];
    }
  }
}

// ------------------------------------------------------------ plan

// a dispatch holds fewer than 2^32 work-items and N + 1 rows exceed that past
// 2^32 suffixes: per-row kernels are grid-stride loops (LI_FOR) over a
// capped grid, the 256-row group kernels group-stride loops
#define LI_MAX_BLOCKS (1ull << 22)
static unsigned li_blocks(uint64_t n) {
  const uint64_t b = (n + 255) / 256;
  return (unsigned) (b > LI_MAX_BLOCKS ? LI_MAX_BLOCKS : (b ? b : 1));
}

struct GtLcpitvPlan {
  GtLcpitvDevInput in;
  uint32_t *lev[LI_MAXLEV];
  LiLevels L;
  uint64_t nitv;
  uint64_t *itv;                 // 5 * nitv, pop order
  uint32_t *before;              // N + 1: intervals with rb < v (NULL past 2^32 rows)
  unsigned long long *first;     // position of the first root edge
};

extern "C" void gt_lcpitv_plan_delete(GtLcpitvPlan *p) {
  if (p == NULL) return;
  (void) hipSetDevice(p->in.device);
  // the plan's buffers go back to the runtime's cache (smax_dev_alloc): the
  // work still queued on them (an events pass on a caller's stream) first
  (void) hipDeviceSynchronize();
  for (int l = 0; l < LI_MAXLEV; l++)
    if (p->lev[l]) smax_dev_free(p->lev[l]);
  if (p->itv) smax_dev_free(p->itv);
  if (p->before) smax_dev_free(p->before);
  if (p->first) smax_dev_free(p->first);
  free(p);
}

extern "C" int gt_lcpitv_plan_create(GtLcpitvPlan **planp, const GtLcpitvDevInput *in,
                                     char *errbuf, size_t errlen) {
  GtLcpitvPlan *p = NULL;
  uint32_t *derr = NULL, herr = 0, *wg_cnt = NULL, *dmarks = NULL;
  uint64_t *wg_off = NULL, *rec = NULL, *key_a = NULL, *key_b = NULL, *idx_a = NULL,
           *idx_b = NULL;
  void *tmp = NULL;
  size_t tmp_bytes = 0;
  uint64_t N, nwg;
  *planp = NULL;
  if (in == NULL || in->lcp_dev == NULL) {
    li_seterr(errbuf, errlen, "missing device lcptab");
    return -1;
  }
  if (in->numllv > 0 && in->llv_dev == NULL) {
    li_seterr(errbuf, errlen, "missing device llvtab");
    return -1;
  }
  if (in->suf_dev != NULL && in->suf_bytes != 4 && in->suf_bytes != 8) {
    li_seterr(errbuf, errlen, "suftab entries must be 4 or 8 bytes (got %d)", in->suf_bytes);
    return -1;
  }
  p = (GtLcpitvPlan *) calloc(1, sizeof *p);
  if (p == NULL) {
    li_seterr(errbuf, errlen, "out of memory");
    return -1;
  }
  p->in = *in;
  N = in->nonspecials;
  LICHK(hipSetDevice(in->device));
  LICHK(smax_dev_alloc((void **) &derr, sizeof (uint32_t)));
  LICHK(hipMemset(derr, 0, sizeof (uint32_t)));
  LICHK(smax_dev_alloc((void **) &p->first, sizeof (unsigned long long)));
  // level 0: exact LCP, then 64-ary mins until one entry remains
  p->L.n[0] = N + 1;
  LICHK(smax_dev_alloc((void **) &p->lev[0], sizeof (uint32_t) * (p->L.n[0] + LI_PAD)));
  hipLaunchKernelGGL(li_expand_kernel, dim3(li_blocks(N + 1)), dim3(256), 0, 0, in->lcp_dev, N,
                     p->lev[0]);
  LICHK(hipGetLastError());
  if (in->numllv > 0) {
    hipLaunchKernelGGL(li_llv_kernel, dim3(li_blocks(in->numllv)), dim3(256), 0, 0, in->llv_dev,
                       in->numllv, in->lcp_dev, N, p->lev[0], derr);
    LICHK(hipGetLastError());
  }
  p->L.nlev = 1;
  while (p->L.n[p->L.nlev - 1] > 1 && p->L.nlev < LI_MAXLEV) {
    const int l = p->L.nlev;
    p->L.n[l] = (p->L.n[l - 1] + 63) / 64;
    LICHK(smax_dev_alloc((void **) &p->lev[l], sizeof (uint32_t) * (p->L.n[l] + LI_PAD)));
    hipLaunchKernelGGL(li_min64_kernel, dim3(li_blocks(p->L.n[l])), dim3(256), 0, 0, p->lev[l - 1],
                       p->L.n[l - 1], p->lev[l], p->L.n[l]);
    LICHK(hipGetLastError());
    p->L.nlev++;
  }
  if (p->L.n[p->L.nlev - 1] > 1) {
    li_seterr(errbuf, errlen, "too many suffixes for the minimum hierarchy");
    goto fail;
  }
  for (int l = 0; l < p->L.nlev; l++) p->L.lv[l] = p->lev[l];
  LICHK(hipMemcpy(&herr, derr, sizeof herr, hipMemcpyDeviceToHost));
  if (herr & 1u) { li_seterr(errbuf, errlen, "lcp value >= 2^32-1 in .llv"); goto fail; }
  if (herr & 2u) { li_seterr(errbuf, errlen, "inconsistent .llv entry (lcp byte is not 255)"); goto fail; }
  // intervals: count per workgroup, scan, write, sort into pop order
  nwg = (N + 255) / 256;
  if (nwg > 0x7fffffffull) { li_seterr(errbuf, errlen, "too many suffixes"); goto fail; }
  LICHK(smax_dev_alloc((void **) &wg_cnt, sizeof (uint32_t) * (nwg + 1)));
  LICHK(smax_dev_alloc((void **) &wg_off, sizeof (uint64_t) * (nwg + 1)));
  if (nwg > 0) {
    hipLaunchKernelGGL(li_count_kernel, dim3(li_blocks(N)), dim3(256), 0, 0, p->L, N, nwg, wg_cnt);
    LICHK(hipGetLastError());
    LICHK(rocprim::exclusive_scan(nullptr, tmp_bytes, wg_cnt, wg_off, (uint64_t) 0, (size_t) nwg,
                                  rocprim::plus<uint64_t>(), (hipStream_t) 0));
    LICHK(smax_dev_alloc((void **) &tmp, tmp_bytes ? tmp_bytes : 16));
    LICHK(rocprim::exclusive_scan(tmp, tmp_bytes, wg_cnt, wg_off, (uint64_t) 0, (size_t) nwg,
                                  rocprim::plus<uint64_t>(), (hipStream_t) 0));
    uint64_t lo = 0;
    uint32_t lc = 0;
    LICHK(hipMemcpy(&lo, wg_off + nwg - 1, sizeof lo, hipMemcpyDeviceToHost));
    LICHK(hipMemcpy(&lc, wg_cnt + nwg - 1, sizeof lc, hipMemcpyDeviceToHost));
    p->nitv = lo + lc;
  }
  LICHK(smax_dev_alloc((void **) &p->itv, sizeof (uint64_t) * 5 * (p->nitv ? p->nitv : 1)));
  if (p->nitv > 0) {
    const uint64_t n = p->nitv;
    LICHK(smax_dev_alloc((void **) &rec, sizeof (uint64_t) * 5 * n));
    LICHK(smax_dev_alloc((void **) &key_a, sizeof (uint64_t) * n));
    LICHK(smax_dev_alloc((void **) &key_b, sizeof (uint64_t) * n));
    LICHK(smax_dev_alloc((void **) &idx_a, sizeof (uint64_t) * n));
    LICHK(smax_dev_alloc((void **) &idx_b, sizeof (uint64_t) * n));
    hipLaunchKernelGGL(li_write_kernel, dim3(li_blocks(N)), dim3(256), 0, 0, p->L, N, nwg, wg_off,
                       rec, key_a, idx_a);
    LICHK(hipGetLastError());
    smax_dev_free(tmp);   // the scan is done: the copies above waited for it
    tmp = NULL;
    tmp_bytes = 0;
    LICHK(rocprim::radix_sort_pairs(nullptr, tmp_bytes, key_a, key_b, idx_a, idx_b, (size_t) n, 0,
                                    64, (hipStream_t) 0));
    LICHK(smax_dev_alloc((void **) &tmp, tmp_bytes ? tmp_bytes : 16));
    if (N < 0xffffffffull) {
      // by rb alone: bits(N) radix bits instead of 64 (rb << 32 | ~lcp, 8
      // onesweep passes, 4.1 ms of the C2 step), then the run reversal
      const int rbits = 64 - __builtin_clzll((unsigned long long) N);
      LICHK(rocprim::radix_sort_pairs(tmp, tmp_bytes, key_a, key_b, idx_a, idx_b, (size_t) n, 0,
                                      rbits, (hipStream_t) 0));
      // before[v] = intervals with rb < v (the events pass's positions, and
      // the runs here): a max-scan over the run ends, staged in key_a's
      // space (free after the sort) where it fits
      uint32_t *D = (uint32_t *) key_a;
      LICHK(smax_dev_alloc((void **) &p->before, sizeof (uint32_t) * (N + 1)));
      if (sizeof (uint64_t) * n < sizeof (uint32_t) * (N + 1)) {
        LICHK(smax_dev_alloc((void **) &dmarks, sizeof (uint32_t) * (N + 1)));
        D = dmarks;
      }
      LICHK(hipMemsetAsync(D, 0, sizeof (uint32_t) * (N + 1), 0));
      hipLaunchKernelGGL(li_rb_marks_kernel, dim3(li_blocks(n)), dim3(256), 0, 0, key_b, n, D);
      LICHK(hipGetLastError());
      size_t sb = 0;
      LICHK(rocprim::inclusive_scan(nullptr, sb, D, p->before, (size_t) (N + 1),
                                    rocprim::maximum<uint32_t>(), (hipStream_t) 0));
      if (sb > tmp_bytes) {
        LICHK(hipDeviceSynchronize());   // the sort is done with tmp
        smax_dev_free(tmp);
        tmp = NULL;
        LICHK(smax_dev_alloc((void **) &tmp, sb));
        tmp_bytes = sb;
      }
      LICHK(rocprim::inclusive_scan(tmp, sb, D, p->before, (size_t) (N + 1),
                                    rocprim::maximum<uint32_t>(), (hipStream_t) 0));
      hipLaunchKernelGGL(li_gather_rev_kernel, dim3(li_blocks(n)), dim3(256), 0, 0, rec, idx_b, key_b,
                         p->before, n, p->itv);
      LICHK(hipGetLastError());
    } else {
      // rb >= 2^32 possible: stable passes by ~lcp, then by rb (past 2^32
      // rows the events pass finds positions by binary search)
      hipLaunchKernelGGL(li_key_kernel, dim3(li_blocks(n)), dim3(256), 0, 0, rec, idx_a, n, 0, key_a);
      LICHK(hipGetLastError());
      LICHK(rocprim::radix_sort_pairs(tmp, tmp_bytes, key_a, key_b, idx_a, idx_b, (size_t) n, 0, 32,
                                      (hipStream_t) 0));
      hipLaunchKernelGGL(li_key_kernel, dim3(li_blocks(n)), dim3(256), 0, 0, rec, idx_b, n, 1, key_a);
      LICHK(hipGetLastError());
      LICHK(rocprim::radix_sort_pairs(tmp, tmp_bytes, key_a, key_b, idx_b, idx_a, (size_t) n, 0, 64,
                                      (hipStream_t) 0));
      hipLaunchKernelGGL(li_gather_kernel, dim3(li_blocks(n)), dim3(256), 0, 0, rec, idx_a, n, p->itv);
      LICHK(hipGetLastError());
    }
  }
  LICHK(hipDeviceSynchronize());
  {
    void *bufs[] = {derr, wg_cnt, wg_off, rec, key_a, key_b, idx_a, idx_b, tmp, dmarks};
    for (size_t i = 0; i < sizeof bufs / sizeof bufs[0]; i++)
      if (bufs[i]) smax_dev_free(bufs[i]);
  }
  *planp = p;
  return 0;
fail:
  {
    (void) hipDeviceSynchronize();   // nothing queued may still use a cached block
    void *bufs[] = {derr, wg_cnt, wg_off, rec, key_a, key_b, idx_a, idx_b, tmp, dmarks};
    for (size_t i = 0; i < sizeof bufs / sizeof bufs[0]; i++)
      if (bufs[i]) smax_dev_free(bufs[i]);
  }
  gt_lcpitv_plan_delete(p);
  return -1;
}

extern "C" uint64_t gt_lcpitv_plan_intervals(const GtLcpitvPlan *p, const uint64_t **itv_dev) {
  if (itv_dev) *itv_dev = p->itv;
  return p->nitv;
}

extern "C" uint64_t gt_lcpitv_plan_num_events(const GtLcpitvPlan *p) {
  return p->in.nonspecials + 2 * p->nitv;
}

extern "C" int gt_lcpitv_plan_events(GtLcpitvPlan *p, uint64_t *events_dev, void *stream) {
  hipStream_t s = (hipStream_t) stream;
  const uint64_t N = p->in.nonspecials, n = p->nitv;
  const unsigned long long none = ~0ull;
  if (hipSetDevice(p->in.device) != hipSuccess) return -1;
  if (N == 0) return 0;
  if (hipMemcpyAsync(p->first, &none, sizeof none, hipMemcpyHostToDevice, s) != hipSuccess) return -1;
  hipLaunchKernelGGL(li_rootfirst_leaf_kernel, dim3(li_blocks(N)), dim3(256), 0, s, p->L, N, p->itv,
                     n, p->before, p->first);
  if (n > 0)
    hipLaunchKernelGGL(li_rootfirst_itv_kernel, dim3(li_blocks(n)), dim3(256), 0, s, p->itv, n,
                       p->before, p->first);
  if (p->in.suf_bytes == 4)
    hipLaunchKernelGGL(li_events_leaf_kernel<uint32_t>, dim3(li_blocks(N)), dim3(256), 0, s, p->L, N,
                       p->itv, n, p->before, p->in.suf_dev, p->first, events_dev);
  else
    hipLaunchKernelGGL(li_events_leaf_kernel<uint64_t>, dim3(li_blocks(N)), dim3(256), 0, s, p->L, N,
                       p->itv, n, p->before, p->in.suf_dev, p->first, events_dev);
  if (n > 0)
    hipLaunchKernelGGL(li_events_itv_kernel, dim3(li_blocks(n)), dim3(256), 0, s, p->itv, n,
                       p->before, p->first, events_dev);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ------------------------------------------------------------ host boundary

// host tables -> HBM -> plan (device 0); *buf holds the device copies
struct LiHostTables {
  uint8_t *lcp;
  GtSmaxLlv *llv;
  void *suf;
};

static void li_host_free(LiHostTables *h) {
  // the plan's kernels ran on the null stream (the staging ring synchronised
  // its own stream): after them the tables go back to the runtime's cache
  (void) hipStreamSynchronize(nullptr);
  smax_dev_free(h->lcp);
  smax_dev_free(h->llv);
  smax_dev_free(h->suf);
  memset(h, 0, sizeof *h);
}

static int li_host_plan(const GtSmaxInput *in, bool with_suf, LiHostTables *h, GtLcpitvPlan **plan,
                        char *errbuf, size_t errlen) {
  GtLcpitvDevInput din;
  uint64_t N;
  memset(h, 0, sizeof *h);
  *plan = NULL;
  if (in == NULL || in->lcptab == NULL) {
    li_seterr(errbuf, errlen, "missing lcptab");
    return -1;
  }
  if (in->numllv > 0 && in->llvtab == NULL) {
    li_seterr(errbuf, errlen, "missing llvtab");
    return -1;
  }
  if (in->nonspecials > in->totallength) {
    li_seterr(errbuf, errlen, "nonspecials (%lu) exceeds totallength (%lu)",
              (unsigned long) in->nonspecials, (unsigned long) in->totallength);
    return -1;
  }
  N = in->nonspecials;
  // the caller's current device (the entry points restore it); tables from
  // the runtime's caching allocator, staged through its pinned ring
  int dev = 0;
  LICHK(hipGetDevice(&dev));
  LICHK(smax_dev_alloc((void **) &h->lcp, N + 1));
  LICHK(smax_stage_upload(h->lcp, in->lcptab, N + 1));
  if (in->numllv > 0) {
    LICHK(smax_dev_alloc((void **) &h->llv, sizeof (GtSmaxLlv) * in->numllv));
    LICHK(smax_stage_upload(h->llv, in->llvtab, sizeof (GtSmaxLlv) * in->numllv));
  }
  if (with_suf && N > 0) {
    LICHK(smax_dev_alloc(&h->suf, (size_t) in->suftab_bytes * N));
    LICHK(smax_stage_upload(h->suf, in->suftab, (size_t) in->suftab_bytes * N));
  }
  din.lcp_dev = h->lcp;
  din.llv_dev = h->llv;
  din.numllv = in->numllv;
  din.suf_dev = h->suf;
  din.suf_bytes = with_suf ? in->suftab_bytes : 8;
  din.nonspecials = N;
  din.device = dev;
  if (gt_lcpitv_plan_create(plan, &din, errbuf, errlen) != 0) {
    li_host_free(h);
    return -1;
  }
  return 0;
fail:
  li_host_free(h);
  return -1;
}

extern "C" int gt_lcpitv_hip_enumerate_to_buffer(const GtSmaxInput *in, uint64_t **itv,
                                                 uint64_t *count, char *errbuf, size_t errlen) {
  LiHostTables h;
  GtLcpitvPlan *plan = NULL;
  SmaxDeviceGuard keep;
  *itv = NULL;
  *count = 0;
  if (li_host_plan(in, false, &h, &plan, errbuf, errlen) != 0) return -1;
  const uint64_t n = plan->nitv;
  if (n > 0) {
    *itv = (uint64_t *) malloc(sizeof (uint64_t) * 5 * n);
    if (*itv == NULL) {
      li_seterr(errbuf, errlen, "out of memory");
    } else if (smax_stage_download(*itv, plan->itv, sizeof (uint64_t) * 5 * n) != hipSuccess) {
      li_seterr(errbuf, errlen, "device to host copy failed");
      free(*itv);
      *itv = NULL;
    }
    if (*itv == NULL) {
      gt_lcpitv_plan_delete(plan);
      li_host_free(&h);
      return -1;
    }
  }
  *count = n;
  gt_lcpitv_plan_delete(plan);
  li_host_free(&h);
  return 0;
}

// gt_esa_bottomup's callback sequence from the device event stream, downloaded
// in chunks of LI_EV_CHUNK events
#define LI_EV_CHUNK (1ull << 20)

// The tree's visitor event stream, built in HBM and handed to sink(r) in
// chunks in the reference's order (r: one 7-word event record); a non-zero
// sink return stops.  need_suf: leaf numbers from the suffix array.
template <typename Sink>
static int li_replay(const GtSmaxInput *in, bool need_suf, Sink sink, char *errbuf, size_t errlen) {
  LiHostTables h;
  GtLcpitvPlan *plan = NULL;
  uint64_t *ev = NULL, *host = NULL, E;
  int rc = 0;
  SmaxDeviceGuard keep;
  if (need_suf && (in == NULL || in->suftab == NULL ||
                   (in->suftab_bytes != 4 && in->suftab_bytes != 8))) {
    li_seterr(errbuf, errlen, "leaf edges need suftab (4 or 8 bytes per entry)");
    return -1;
  }
  if (li_host_plan(in, need_suf, &h, &plan, errbuf, errlen) != 0) return -1;
  E = gt_lcpitv_plan_num_events(plan);
  if (E > 0) {
    LICHK(hipMalloc(&ev, sizeof (uint64_t) * 7 * E));
    if (gt_lcpitv_plan_events(plan, ev, NULL) != 0) {
      li_seterr(errbuf, errlen, "event generation failed");
      goto fail;
    }
    LICHK(hipHostMalloc((void **) &host, sizeof (uint64_t) * 7 * (E < LI_EV_CHUNK ? E : LI_EV_CHUNK),
                        hipHostMallocDefault));
  }
  for (uint64_t e0 = 0; e0 < E && rc == 0; e0 += LI_EV_CHUNK) {
    const uint64_t n = E - e0 < LI_EV_CHUNK ? E - e0 : LI_EV_CHUNK;
    LICHK(hipMemcpy(host, ev + 7 * e0, sizeof (uint64_t) * 7 * n, hipMemcpyDeviceToHost));
    for (uint64_t k = 0; k < n && rc == 0; k++) rc = sink(host + 7 * k);
  }
  if (ev) (void) hipFree(ev);
  if (host) (void) hipHostFree(host);
  gt_lcpitv_plan_delete(plan);
  li_host_free(&h);
  if (rc != 0) {
    li_seterr(errbuf, errlen, "visitor callback returned non-zero");
    return -1;
  }
  return 0;
fail:
  if (ev) (void) hipFree(ev);
  if (host) (void) hipHostFree(host);
  gt_lcpitv_plan_delete(plan);
  li_host_free(&h);
  return -1;
}

extern "C" int gt_esa_bottomup_hip(const GtSmaxInput *in, const GtLcpitvVisitor *v, void *data,
                                   char *errbuf, size_t errlen) {
  if (v == NULL) {
    li_seterr(errbuf, errlen, "missing visitor");
    return -1;
  }
  return li_replay(in, v->leaf_edge != NULL, [&](const uint64_t *r) {
    if (r[0] == 0) return v->leaf_edge ? v->leaf_edge(data, (int) r[1], r[2], r[3], r[4]) : 0;
    if (r[0] == 1)
      return v->branching_edge ? v->branching_edge(data, (int) r[1], r[2], r[3], r[4], r[5], r[6]) : 0;
    return v->lcp_interval ? v->lcp_interval(data, r[2], r[3], r[4]) : 0;
  }, errbuf, errlen);
}

// GtESAVisitorInfo emulation (src/match/esa-bottomup.c:20-110): the
// reference binds one info object to each STACK SLOT, created with
// info_new in chunks of 32 as the stack grows and deleted, slot by slot, at
// the end; a pushed interval reuses its slot's object, and a father pushed
// right after its first child popped takes that child's slot -- so its
// branching edge sees soninfo NULL and fatherinfo == the child's info.  The
// event stream carries everything needed to follow the stack: a push is a
// firstsucc leaf edge or a firstsucc branching edge of father depth > 0, a
// pop is an lcp-interval event (firstsucc edges of depth 0 are the root's).
extern "C" int gt_esa_bottomup_info_hip(const GtSmaxInput *in, const GtLcpitvInfoVisitor *v,
                                        void *data, char *errbuf, size_t errlen) {
  if (v == NULL || v->info_new == NULL) {
    li_seterr(errbuf, errlen, "missing visitor or info_new");
    return -1;
  }
  std::vector<void *> slot;
  uint64_t depth = 0, last = 0;
  auto grow = [&]() {
    for (int k = 0; k < 32; k++) slot.push_back(v->info_new(data));   // allocateBUstack
  };
  grow();
  depth = 1;                                                           // PUSH(0, 0): the root
  const int rc = li_replay(in, v->leaf_edge != NULL, [&](const uint64_t *r) -> int {
    if (r[0] == 0) {                                                   // leaf edge
      if (r[1] != 0 && r[2] > 0) {                                     // PUSH(lcpvalue, idx)
        if (depth >= slot.size()) grow();
        depth++;
      }
      return v->leaf_edge ? v->leaf_edge(data, (int) r[1], r[2], r[3], slot[depth - 1], r[4]) : 0;
    }
    if (r[0] == 2) {                                                   // POP
      if (depth < 2) return -1;                                        // never the root
      last = --depth;
      return v->lcp_interval ? v->lcp_interval(data, r[2], r[3], r[4], slot[last]) : 0;
    }
    void *son = slot[last];
    if (r[1] != 0 && r[2] > 0) {                                       // PUSH(lcpvalue, last.lb)
      depth++;                                                         // = the popped child's slot
      son = nullptr;
    }
    return v->branching_edge
               ? v->branching_edge(data, (int) r[1], r[2], r[3], slot[depth - 1], r[4], r[5], r[6], son)
               : 0;
  }, errbuf, errlen);
  if (v->info_delete)
    for (void *x : slot) v->info_delete(x, data);                      // gt_GtArrayGtBUItvinfo_delete
  return rc;
}
