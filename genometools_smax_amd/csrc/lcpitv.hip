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
// All of it follows from one ANSV quantity, the strict previous-smaller
// value PL(k), computed per tile of 2048 rows in LDS (per-thread pointer
// jumping inside 8-row segments, a segment-minimum search across the tile,
// the 64-ary min hierarchy over the exact LCP array (u32) only for the few
// rows with no smaller value earlier in their tile): the stack of the
// reference after row idx is the PL chain from idx, so the intervals popped
// at a row are read off that chain (li_walk) -- no sort, no per-row global
// searches.  The tree stays in HBM (GtLcpitvPlan: the pop-ordered interval
// records and the intervals popped before each tile); the visitor's event
// stream is generated there too, every event at its position in the
// reference's order, no stack and no replay loop (li_tile_events_kernel):
// per row idx (X = LCP[idx], Y = LCP[idx+1]) the traversal emits exactly
// one leaf edge, then for every interval popped at idx (pop order) its
// lcp-interval and branching-edge events, so with P(idx) = #intervals with
// rb < idx the leaf of row idx sits at idx + 2 P(idx) and popped interval r
// of row idx at idx + 2 P(idx) + 1 + 2r.  The host entry points download
// the events in chunks and call the visitor.
#include <hip/hip_runtime.h>
#include <type_traits>
#include <vector>
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

// workgroup-wide exclusive prefix (256 threads); *total = sum
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
  __syncthreads();                     // sW is reused by the next call
  return wo + incl - v;
}

// ------------------------------------------------------------ tiles
//
// The tree from the strict previous-smaller value PL(k) = the nearest p < k
// with X[p] < X[k] alone.  The reference's stack after row idx holds
// exactly the chain c0 = idx, c1 = PL(c0), c2 = PL(c1), ... (depths X[cj]
// strictly decreasing, the interval of depth X[cj] starting at c(j+1)), so
// the lcp-intervals popped at row idx (Y = X[idx+1]) are, deepest first,
// [c(j+1), idx] of depth X[cj] for every cj with X[cj] > Y; the father of
// pop j has depth max(X[c(j+1)], Y) and lb PL(c(j+1)) when X[c(j+1)] >= Y,
// else it is the new interval (Y, c(j+1)) pushed after the pops.  The leaf
// of row idx hangs below (X[idx], PL(idx)) when Y <= X[idx], else it is the
// first child of (Y, idx).  Every interval is popped once, so the walks
// cost O(N) over the whole table.
//
// A workgroup owns LI_T consecutive rows (a tile).  Pass 0 computes PL of
// its rows in LDS -- per-thread pointer jumping inside 8-row segments, the
// rows left unresolved by a segment-minimum search across the tile, and
// the tile's prefix minima (no smaller value in the tile before them, a
// handful per tile) by the global 64-ary hierarchy (li_prev) -- and stores
// it in HBM.  Chains that leave a tile (intervals open at its start)
// continue along the chain from the row before the tile, t0-1, PL(t0-1),
// ... (every PL out of the tile lies on it): its first LI_BD entries are
// gathered once per tile (li_bchain_kernel, one thread per tile) and
// loaded with the tile.  Three passes walk the chains: a count per tile
// (plan), the pop-ordered interval records (plan) and the visitor event
// stream (events); the last two stage their output in LDS per 64-row wave
// step and store it as contiguous 16-byte pieces.
#define LI_T 2048                       // rows per tile
#define LI_TPB 256                      // threads per tile workgroup
#define LI_RPT (LI_T / LI_TPB)          // rows per segment (one thread)
#define LI_GSEG 16                      // segments per group
#define LI_NGRP (LI_TPB / LI_GSEG)
#define LI_BD 64                        // boundary-chain entries kept per tile
#define LI_ITV_CAP 384                  // interval records staged per workgroup
#define LI_EV_STAGE 16384               // event staging bytes per workgroup

template <typename RowT>
__device__ __forceinline__ RowT li_none() { return (RowT) ~(RowT) 0; }

// pass 0's LDS
template <typename RowT>
struct LiAnsvTile {
  uint32_t x[LI_T + 1];                 // X[t0 .. t0 + LI_T] (0 past row N)
  RowT pl[LI_T];                        // PL of the tile's rows (~0: none / pending)
  uint32_t segmin[LI_TPB];
  uint32_t grpmin[LI_NGRP];
};

// the walking passes' LDS: the tile, its boundary chain, the output stage
template <typename RowT, int STAGE>
struct LiWalkTile {
  uint32_t x[LI_T + 1];
  RowT pl[LI_T];
  RowT brow[LI_BD];                     // t0-1, PL(t0-1), ... (rows strictly decreasing)
  uint32_t bx[LI_BD];                   // their X (strictly decreasing)
  int nb;                               // entries held; the chain goes on past them iff
                                        // nb == LI_BD and bx[nb-1] > 0
  alignas(16) unsigned char stage[STAGE];
};

// PL of every row of the tile [t0, t0 + LI_T) into S.pl (rows with X = 0
// have none).  Ends with a barrier.
template <typename RowT>
__device__ void li_tile_ansv(const LiLevels &L, uint64_t N, uint64_t t0, LiAnsvTile<RowT> &S) {
  const int tid = threadIdx.x;
  const RowT none = li_none<RowT>();
  for (int k = tid; k <= LI_T; k += LI_TPB) {
    const uint64_t g = t0 + (uint64_t) k;
    S.x[k] = g <= N ? L.lv[0][g] : 0u;   // lv[0] holds rows 0..N, X[N] = 0
  }
  __syncthreads();
  // the thread's segment, left to right: p jumps along PL inside it
  const int lo = tid * LI_RPT;
  uint32_t m = 0xffffffffu;
  for (int i = lo; i < lo + LI_RPT; i++) {
    const uint32_t v = S.x[i];
    m = v < m ? v : m;
    int p = i - 1;
    while (p >= lo && S.x[p] >= v) {
      const RowT q = S.pl[p];
      p = q == none ? lo - 1 : (int) (q - (RowT) t0);
    }
    S.pl[i] = p >= lo ? (RowT) (t0 + (uint64_t) p) : none;
  }
  S.segmin[tid] = m;
  __syncthreads();
  if (tid < LI_NGRP) {
    uint32_t g = 0xffffffffu;
    for (int s = tid * LI_GSEG; s < (tid + 1) * LI_GSEG; s++) g = S.segmin[s] < g ? S.segmin[s] : g;
    S.grpmin[tid] = g;
  }
  __syncthreads();
  // rows with no smaller value earlier in their segment: the nearest segment
  // before with a smaller minimum (then the last row below v along that
  // segment's own PL chain, which stays inside it), else the global search
  for (int i = lo; i < lo + LI_RPT; i++) {
    const uint32_t v = S.x[i];
    if (v == 0 || S.pl[i] != none) continue;
    int found = -1;
    for (int s = tid - 1; s >= (tid / LI_GSEG) * LI_GSEG; s--)
      if (S.segmin[s] < v) { found = s; break; }
    if (found < 0)
      for (int g = tid / LI_GSEG - 1; g >= 0 && found < 0; g--)
        if (S.grpmin[g] < v)
          for (int s = g * LI_GSEG + LI_GSEG - 1; s >= g * LI_GSEG; s--)
            if (S.segmin[s] < v) { found = s; break; }
    if (found >= 0) {
      int p = found * LI_RPT + LI_RPT - 1;
      while (S.x[p] >= v) p = (int) (S.pl[p] - (RowT) t0);
      S.pl[i] = (RowT) (t0 + (uint64_t) p);
    } else {
      S.pl[i] = t0 > 0 ? (RowT) li_prev(L, t0, v, true) : none;
    }
  }
  __syncthreads();
}

// pass 0 (plan): PL of every row into HBM (RowT each, ~0 where X = 0)
template <typename RowT>
__global__ void __launch_bounds__(LI_TPB) li_pl_kernel(LiLevels L, uint64_t N, uint64_t ntiles,
                                                       RowT *PL) {
  __shared__ LiAnsvTile<RowT> S;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint64_t t0 = t * LI_T;
    li_tile_ansv(L, N, t0, S);
    const int nrows = N - t0 < LI_T ? (int) (N - t0) : LI_T;
    for (int i = threadIdx.x; i < nrows; i += LI_TPB) PL[t0 + i] = S.pl[i];
    __syncthreads();                     // S is rewritten by the next tile
  }
}

// each tile's boundary chain t0-1, PL(t0-1), ... down to the first X = 0
// entry, at most LI_BD entries (one thread per tile: a latency chain of
// dependent loads, thousands of them in flight)
template <typename RowT>
__global__ void __launch_bounds__(256) li_bchain_kernel(const uint32_t *X, const RowT *PL,
                                                        uint64_t ntiles, RowT *brow, uint32_t *bx,
                                                        uint32_t *bn) {
  LI_FOR(t, ntiles) {
    int k = 0;
    if (t > 0) {
      uint64_t s = t * LI_T - 1;
      for (; k < LI_BD;) {
        const uint32_t xs = X[s];
        brow[t * LI_BD + k] = (RowT) s;
        bx[t * LI_BD + k] = xs;
        k++;
        if (xs == 0) break;
        s = PL[s];
      }
    }
    bn[t] = (uint32_t) k;
  }
}

// the tile's X (rows t0 .. t0 + LI_T, 0 past row N), PL and boundary chain
// into LDS
template <typename RowT, int STAGE>
__device__ __forceinline__ void li_tile_load(const uint32_t *X, const RowT *PL, const RowT *brow,
                                             const uint32_t *bx, const uint32_t *bn, uint64_t N,
                                             uint64_t t, LiWalkTile<RowT, STAGE> &S) {
  const uint64_t t0 = t * LI_T;
  for (int k = threadIdx.x; k <= LI_T; k += LI_TPB) {
    const uint64_t g = t0 + (uint64_t) k;
    S.x[k] = g <= N ? X[g] : 0u;
    if (k < LI_T) S.pl[k] = g < N ? PL[g] : li_none<RowT>();
  }
  const int nb = (int) bn[t];
  if (threadIdx.x < (unsigned) nb) {
    S.brow[threadIdx.x] = brow[t * LI_BD + threadIdx.x];
    S.bx[threadIdx.x] = bx[t * LI_BD + threadIdx.x];
  }
  if (threadIdx.x == 0) S.nb = nb;
  __syncthreads();
}

// a row before the tile: its index in the boundary chain, -1 past the
// entries held (binary search, rows strictly decreasing)
template <typename RowT, int STAGE>
__device__ __forceinline__ int li_bfind(const LiWalkTile<RowT, STAGE> &S, uint64_t c) {
  int lo = 0, hi = S.nb - 1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    const uint64_t r = (uint64_t) S.brow[mid];
    if (r == c) return mid;
    if (r > c) lo = mid + 1; else hi = mid - 1;
  }
  return -1;
}

// Rows deeper down the boundary chain than the LDS copy holds (rare) are
// read by calls: inlined, the compiler would wait for every memory
// operation of the wave (vmcnt counts the stage's 16-byte stores too) at
// each join after the branch, taken or not -- the walks would pay the
// store latency on every step
// (counted: how often the LDS copy of the chain falls short, a diagnostic
// read by gt_lcpitv_far_reads)
__device__ unsigned long long li_far_reads;

__device__ __noinline__ uint32_t li_x_far(const uint32_t *X, uint64_t c) {
  atomicAdd(&li_far_reads, 1ull);
  return X[c];
}

template <typename RowT>
__device__ __noinline__ uint64_t li_pl_far(const RowT *PL, uint64_t c) {
  atomicAdd(&li_far_reads, 1ull);
  return (uint64_t) PL[c];
}

// X and PL of any row at or before the tile's end: the tile's and the
// boundary chain's from LDS, rows deeper down the chain from HBM
template <typename RowT, int STAGE>
__device__ __forceinline__ uint32_t li_tx(const uint32_t *X, const LiWalkTile<RowT, STAGE> &S,
                                          uint64_t t0, uint64_t c) {
  if (c >= t0) return S.x[c - t0];
  const int k = li_bfind(S, c);
  return k >= 0 ? S.bx[k] : li_x_far(X, c);
}

template <typename RowT, int STAGE>
__device__ __forceinline__ uint64_t li_tpl(const RowT *PL, const LiWalkTile<RowT, STAGE> &S,
                                           uint64_t t0, uint64_t c) {
  if (c >= t0) return (uint64_t) S.pl[c - t0];
  const int k = li_bfind(S, c);
  return k >= 0 && k + 1 < S.nb ? (uint64_t) S.brow[k + 1] : li_pl_far(PL, c);
}

// intervals popped at row t0 + i
template <typename RowT, int STAGE>
__device__ __forceinline__ uint32_t li_pops(const uint32_t *X, const RowT *PL,
                                            const LiWalkTile<RowT, STAGE> &S, uint64_t t0, int i) {
  const uint32_t Y = S.x[i + 1];
  uint64_t c = t0 + (uint64_t) i;
  uint32_t xc = S.x[i], n = 0;
  while (xc > Y) {
    n++;
    c = li_tpl(PL, S, t0, c);
    xc = li_tx(X, S, t0, c);
  }
  return n;
}

// the pops of row idx = t0 + i in order, deepest first: f(j, lcp, lb, fd, flb, newfather)
template <typename RowT, int STAGE, typename F>
__device__ __forceinline__ void li_walk(const uint32_t *X, const RowT *PL,
                                        const LiWalkTile<RowT, STAGE> &S, uint64_t t0, int i, F f) {
  const uint32_t Y = S.x[i + 1];
  uint32_t xc = S.x[i];
  if (xc <= Y) return;
  uint64_t nx = S.pl[i];
  uint32_t xn = li_tx(X, S, t0, nx);
  for (uint32_t j = 0;; j++) {
    const uint32_t fd = xn > Y ? xn : Y;
    uint64_t nn = 0, flb = 0;
    if (xn >= Y && fd > 0) {
      nn = li_tpl(PL, S, t0, nx);
      flb = nn;
    } else if (fd > 0) {
      flb = nx;                          // the new father (Y, nx)
    }
    f(j, xc, nx, fd, flb, xn < Y);
    if (xn <= Y) break;
    xc = xn;
    nx = nn;
    xn = li_tx(X, S, t0, nx);
  }
}

// pass 1 (plan): intervals popped in each tile
template <typename RowT>
__global__ void __launch_bounds__(LI_TPB) li_tile_count_kernel(const uint32_t *X, const RowT *PL,
                                                               const RowT *brow, const uint32_t *bx,
                                                               const uint32_t *bn, uint64_t N,
                                                               uint64_t ntiles, uint32_t *tile_cnt) {
  __shared__ LiWalkTile<RowT, 16> S;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint64_t t0 = t * LI_T;
    li_tile_load(X, PL, brow, bx, bn, N, t, S);
    const int nrows = N - t0 < LI_T ? (int) (N - t0) : LI_T;
    uint32_t n = 0;
    for (int i = threadIdx.x; i < nrows; i += LI_TPB) n += li_pops(X, PL, S, t0, i);
    uint32_t tot;
    (void) li_block_excl(n, &tot);
    if (threadIdx.x == 0) tile_cnt[t] = tot;
  }
}

// The writing passes split a tile into four 512-row quarters, one per
// wave: the waves' interval totals are exchanged once per tile (the only
// workgroup barriers besides the tile load), then each wave walks its
// quarter in 64-row steps on its own -- wave-level scans for the offsets,
// its own part of the stage, its own 16-byte stores.
#define LI_WAVES (LI_TPB / 64)
#define LI_QROWS (LI_T / LI_WAVES)

__device__ __forceinline__ uint32_t li_wave_excl(uint32_t v, uint32_t *total) {
  const int lane = threadIdx.x & 63;
  uint32_t incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(incl, d, 64);
    if (lane >= d) incl += o;
  }
  *total = __shfl(incl, 63, 64);
  return incl - v;
}

// the wave's LDS stores before its loads (and its loads before the next
// stores): LDS operations of one wave complete in order once waited for
__device__ __forceinline__ void li_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// intervals popped before each wave's quarter, from tile_off[t]; ends with
// a barrier
template <typename RowT, int STAGE, typename Weight>
__device__ __forceinline__ uint64_t li_wave_base(const uint32_t *X, const RowT *PL,
                                                 const LiWalkTile<RowT, STAGE> &S, uint64_t t0,
                                                 int nrows, uint64_t tile_base, uint32_t *sWT) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t n = 0;
  for (int r = 0; r < LI_QROWS / 64; r++) {
    const int i = wave * LI_QROWS + r * 64 + lane;
    if (i < nrows) n += li_pops(X, PL, S, t0, i);
  }
  uint32_t tot;
  (void) li_wave_excl(n, &tot);
  if (lane == 0) sWT[wave] = tot;
  __syncthreads();
  uint64_t base = tile_base;
  for (int w = 0; w < wave; w++) base += sWT[w];
  return base;
}

// pass 2 (plan): the interval records (lcp, lb, rb, father lcp, father lb)
// in pop order at tile_off[t] on (staged per 64-row step, stored as
// contiguous 16-byte pieces), and the stream position of the first edge to
// the root (the reference's firstedgefromroot, esa-bottomup.c:134-141)
#define LI_ITV_WCAP (LI_ITV_CAP / LI_WAVES)   // records staged per wave step
template <typename RowT>
__global__ void __launch_bounds__(LI_TPB) li_tile_itv_kernel(const uint32_t *X, const RowT *PL,
                                                             const RowT *brow, const uint32_t *bx,
                                                             const uint32_t *bn, uint64_t N,
                                                             uint64_t ntiles, const uint64_t *tile_off,
                                                             uint64_t *itv, unsigned long long *first) {
  __shared__ LiWalkTile<RowT, 40 * LI_ITV_CAP> S;
  __shared__ uint32_t sWT[LI_WAVES];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint64_t *stage = reinterpret_cast<uint64_t *>(S.stage) + 5 * LI_ITV_WCAP * wave;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint64_t t0 = t * LI_T;
    li_tile_load(X, PL, brow, bx, bn, N, t, S);
    const int nrows = N - t0 < LI_T ? (int) (N - t0) : LI_T;
    uint64_t base = li_wave_base<RowT, 40 * LI_ITV_CAP, int>(X, PL, S, t0, nrows, tile_off[t], sWT);
    for (int r = 0; r < LI_QROWS / 64; r++) {
      const int i = wave * LI_QROWS + r * 64 + lane;
      const bool row = i < nrows;
      const uint32_t n = row ? li_pops(X, PL, S, t0, i) : 0u;
      uint32_t tot;
      const uint32_t off = li_wave_excl(n, &tot);
      if (row) {
        const uint64_t idx = t0 + (uint64_t) i;
        const uint64_t pos = idx + 2 * (base + off);       // the row's leaf event
        if (S.x[i] == 0 && S.x[i + 1] == 0) atomicMin(first, (unsigned long long) pos);
        li_walk(X, PL, S, t0, i, [&](uint32_t j, uint32_t lcp, uint64_t lb, uint32_t fd, uint64_t flb,
                                     bool) {
          const uint32_t k = off + j;
          uint64_t *w = k < LI_ITV_WCAP ? stage + 5 * k : itv + 5 * (base + k);
          w[0] = lcp;
          w[1] = lb;
          w[2] = idx;
          w[3] = fd;
          w[4] = flb;
          if (fd == 0) atomicMin(first, (unsigned long long) (pos + 2 + 2 * j));
        });
      }
      li_wave_sync();
      const uint32_t staged = tot < LI_ITV_WCAP ? tot : LI_ITV_WCAP;
      // words [5 base, 5 (base + staged)) as aligned 16-byte pairs
      const uint64_t w0 = 5 * base, w1 = 5 * (base + staged);
      for (uint64_t q = (w0 >> 1) + lane; 2 * q < w1; q += 64) {
        const uint64_t a = 2 * q;
        const bool lo_ok = a >= w0, hi_ok = a + 1 < w1;
        const uint64_t v0 = lo_ok ? stage[a - w0] : 0, v1 = hi_ok ? stage[a + 1 - w0] : 0;
        if (lo_ok && hi_ok) reinterpret_cast<ulonglong2 *>(itv)[q] = make_ulonglong2(v0, v1);
        else if (lo_ok) itv[a] = v0;
        else if (hi_ok) itv[a + 1] = v1;   // (neither: an empty step at an odd word)
      }
      li_wave_sync();
      base += tot;
    }
    __syncthreads();                     // S and sWT are rewritten by the next tile
  }
}

// pass 3 (events): the gt_esa_bottomup event stream of the tile's rows,
// every event at its position in the reference's order: per row its leaf
// edge, then per pop its lcp-interval and branching-edge events
//   (0, firstsucc, fd, flb, leafnumber, 0, 0)   visit_leaf_edge
//   (2, 0, lcp, lb, rb, 0, 0)                   visit_lcp_interval
//   (1, firstsucc, fd, flb, sd, slb, srb)       visit_branching_edge
// staged per 64-row wave step as 4-word descriptors (a leaf's holds its
// leaf number, read while walking; the branching edge takes sd, slb, srb
// from the lcp-interval event before it) and stored as aligned 16-byte
// pieces of the 7-word records; events past the stage go straight to memory
template <typename DT>
struct LiDesc {                         // one staged event
  DT a, b, c, d;                        // a: kind | firstsucc << 2
};

template <typename DT>
__device__ __forceinline__ uint64_t li_event_word(const LiDesc<DT> *st, uint32_t e, uint32_t f) {
  const LiDesc<DT> d = st[e];
  const uint32_t kind = (uint32_t) d.a & 3u;
  if (f == 0) return kind;
  if (f == 1) return kind == 2u ? 0u : (uint64_t) (d.a >> 2);
  if (f == 2) return d.b;
  if (f == 3) return d.c;
  if (kind == 1u) {                      // sd, slb, srb: the lcp-interval event before
    const LiDesc<DT> p = st[e - 1];
    return f == 4 ? (uint64_t) p.b : f == 5 ? (uint64_t) p.c : (uint64_t) p.d;
  }
  return f == 4 ? (uint64_t) d.d : 0u;   // leaf number / rb
}

template <typename RowT, typename SufT>
__global__ void __launch_bounds__(LI_TPB) li_tile_events_kernel(const uint32_t *X, const RowT *PL,
                                                                const RowT *brow, const uint32_t *bx,
                                                                const uint32_t *bn, uint64_t N,
                                                                uint64_t ntiles,
                                                                const uint64_t *tile_off,
                                                                const SufT *suf,
                                                                const unsigned long long *firstp,
                                                                uint64_t *ev) {
  // descriptor words wide enough for row indices and leaf numbers
  using DT = typename std::conditional<(sizeof (RowT) >= sizeof (SufT)), RowT, SufT>::type;
  __shared__ LiWalkTile<RowT, LI_EV_STAGE> S;
  __shared__ uint32_t sWT[LI_WAVES];
  constexpr uint32_t cap = LI_EV_STAGE / sizeof (LiDesc<DT>) / LI_WAVES;   // per wave step
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  LiDesc<DT> *stage = reinterpret_cast<LiDesc<DT> *>(S.stage) + cap * wave;
  const uint64_t first = *firstp;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint64_t t0 = t * LI_T;
    li_tile_load(X, PL, brow, bx, bn, N, t, S);
    const int nrows = N - t0 < LI_T ? (int) (N - t0) : LI_T;
    // stream position of the wave's next event: the rows before it and two
    // events per interval popped before it
    const uint64_t ib = li_wave_base<RowT, LI_EV_STAGE, int>(X, PL, S, t0, nrows, tile_off[t], sWT);
    uint64_t ebase = t0 + (uint64_t) (wave * LI_QROWS) + 2 * ib;
    // the leaf numbers of the wave's rows, loaded before its first store (a
    // load inside the steps would wait for the stores before it)
    uint64_t leaves[LI_QROWS / 64];
#pragma unroll
    for (int r = 0; r < LI_QROWS / 64; r++) {
      const int i = wave * LI_QROWS + r * 64 + lane;
      leaves[r] = i < nrows && suf != nullptr ? (uint64_t) suf[t0 + (uint64_t) i] : 0u;
    }
#pragma unroll
    for (int r = 0; r < LI_QROWS / 64; r++) {
      const int i = wave * LI_QROWS + r * 64 + lane;
      const bool row = i < nrows;
      const uint64_t idx = t0 + (uint64_t) i;
      const uint64_t leaf = leaves[r];
      const uint32_t n = row ? li_pops(X, PL, S, t0, i) : 0u;
      uint32_t tot;
      const uint32_t off = li_wave_excl(row ? 1u + 2u * n : 0u, &tot);
      if (row) {
        const uint32_t xi = S.x[i], Y = S.x[i + 1];
        const uint64_t pos = ebase + off;
        uint64_t fs, fd, flb;
        if (Y <= xi) {
          fs = (xi == 0 && pos == first) ? 1u : 0u;
          fd = xi;
          flb = xi == 0 ? 0 : (uint64_t) S.pl[i];
        } else {
          fs = 1;
          fd = Y;
          flb = idx;
        }
        if (off < cap) {
          stage[off] = LiDesc<DT>{(DT) (fs << 2), (DT) fd, (DT) flb, (DT) leaf};
        } else {
          uint64_t *w = ev + 7 * pos;
          w[0] = 0; w[1] = fs; w[2] = fd; w[3] = flb; w[4] = leaf; w[5] = 0; w[6] = 0;
        }
        li_walk(X, PL, S, t0, i, [&](uint32_t j, uint32_t lcp, uint64_t lb, uint32_t pfd,
                                     uint64_t pflb, bool newfather) {
          const uint32_t k = off + 1 + 2 * j;
          const uint64_t bfs = newfather ? 1u : (pfd == 0 && pos + 2 + 2 * j == first) ? 1u : 0u;
          if (k < cap) stage[k] = LiDesc<DT>{(DT) 2, (DT) lcp, (DT) lb, (DT) idx};
          if (k + 1 < cap) {
            stage[k + 1] = LiDesc<DT>{(DT) (1u | (bfs << 2)), (DT) pfd, (DT) pflb, (DT) 0};
          } else {
            uint64_t *w = ev + 7 * (ebase + k);
            if (k >= cap) { w[0] = 2; w[1] = 0; w[2] = lcp; w[3] = lb; w[4] = idx; w[5] = 0; w[6] = 0; }
            w[7] = 1; w[8] = bfs; w[9] = pfd; w[10] = pflb; w[11] = lcp; w[12] = lb; w[13] = idx;
          }
        });
      }
      li_wave_sync();
      const uint32_t staged = tot < cap ? tot : cap;
      const uint64_t w0 = 7 * ebase, w1 = 7 * (ebase + staged);
      for (uint64_t q = (w0 >> 1) + lane; 2 * q < w1; q += 64) {
        const uint64_t a = 2 * q;
        const bool lo_ok = a >= w0, hi_ok = a + 1 < w1;
        uint64_t v0 = 0, v1 = 0;
        if (lo_ok) {
          const uint32_t e = (uint32_t) (a - w0);
          v0 = li_event_word(stage, e / 7, e % 7);
        }
        if (hi_ok) {
          const uint32_t e = (uint32_t) (a + 1 - w0);
          v1 = li_event_word(stage, e / 7, e % 7);
        }
        if (lo_ok && hi_ok) reinterpret_cast<ulonglong2 *>(ev)[q] = make_ulonglong2(v0, v1);
        else if (lo_ok) ev[a] = v0;
        else if (hi_ok) ev[a + 1] = v1;
      }
      li_wave_sync();
      ebase += tot;
    }
    __syncthreads();                     // S and sWT are rewritten by the next tile
  }
}

// ------------------------------------------------------------ plan

// a dispatch holds fewer than 2^32 work-items and N + 1 rows exceed that past
// 2^32 suffixes: per-row kernels are grid-stride loops (LI_FOR) over a
// capped grid, the tile kernels tile-stride loops
#define LI_MAX_BLOCKS (1ull << 22)
static unsigned li_blocks(uint64_t n) {
  const uint64_t b = (n + 255) / 256;
  return (unsigned) (b > LI_MAX_BLOCKS ? LI_MAX_BLOCKS : (b ? b : 1));
}

static unsigned li_tile_grid(uint64_t ntiles) {
  return (unsigned) (ntiles > LI_MAX_BLOCKS ? LI_MAX_BLOCKS : (ntiles ? ntiles : 1));
}

struct GtLcpitvPlan {
  GtLcpitvDevInput in;
  uint32_t *lev[LI_MAXLEV];
  LiLevels L;
  bool wide;                     // rows past 2^32: 64-bit row indices in the tiles
  uint64_t ntiles;
  uint64_t nitv;
  uint64_t *itv;                 // 5 * nitv, pop order
  uint64_t *tile_off;            // intervals popped before each tile
  void *pl;                      // PL of every row (RowT: u32, u64 when wide)
  void *brow;                    // boundary chain of every tile (LI_BD RowT each)
  uint32_t *bx, *bn;             // its X values, its length
  unsigned long long *first;     // stream position of the first root edge
  SmaxStreamMarks marks;         // streams the plan's work ran on
};

extern "C" void gt_lcpitv_plan_delete(GtLcpitvPlan *p) {
  if (p == NULL) return;
  (void) hipSetDevice(p->in.device);
  // the buffers return to the runtime's cache behind the plan's own work
  // (events recorded where it was enqueued): nothing here waits, and no
  // other stream of the device is involved
  SmaxFence *fence = smax_marks_fence(&p->marks);
  for (int l = 0; l < LI_MAXLEV; l++) smax_dev_free_fenced(p->lev[l], fence);
  smax_dev_free_fenced(p->itv, fence);
  smax_dev_free_fenced(p->tile_off, fence);
  smax_dev_free_fenced(p->pl, fence);
  smax_dev_free_fenced(p->brow, fence);
  smax_dev_free_fenced(p->bx, fence);
  smax_dev_free_fenced(p->bn, fence);
  smax_dev_free_fenced(p->first, fence);
  smax_fence_release(fence);
  free(p);
}

extern "C" int gt_lcpitv_plan_create_stream(GtLcpitvPlan **planp, const GtLcpitvDevInput *in,
                                            void *stream, char *errbuf, size_t errlen) {
  GtLcpitvPlan *p = NULL;
  hipStream_t s = (hipStream_t) stream;
  uint32_t *derr = NULL, herr = 0, *tile_cnt = NULL;
  void *tmp = NULL;
  size_t tmp_bytes = 0;
  uint64_t N;
  const unsigned long long none = ~0ull;
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
  smax_marks_init(&p->marks);
  p->in = *in;
  N = in->nonspecials;
  p->wide = N + 1 >= 0xffffffffull;
  p->ntiles = (N + LI_T - 1) / LI_T;
  LICHK(hipSetDevice(in->device));
  LICHK(smax_dev_alloc((void **) &derr, sizeof (uint32_t)));
  LICHK(hipMemsetAsync(derr, 0, sizeof (uint32_t), s));
  LICHK(smax_dev_alloc((void **) &p->first, sizeof (unsigned long long)));
  LICHK(hipMemcpyAsync(p->first, &none, sizeof none, hipMemcpyHostToDevice, s));
  // level 0: exact LCP, then 64-ary mins until one entry remains
  p->L.n[0] = N + 1;
  LICHK(smax_dev_alloc((void **) &p->lev[0], sizeof (uint32_t) * (p->L.n[0] + LI_PAD)));
  hipLaunchKernelGGL(li_expand_kernel, dim3(li_blocks(N + 1)), dim3(256), 0, s, in->lcp_dev, N,
                     p->lev[0]);
  LICHK(hipGetLastError());
  if (in->numllv > 0) {
    hipLaunchKernelGGL(li_llv_kernel, dim3(li_blocks(in->numllv)), dim3(256), 0, s, in->llv_dev,
                       in->numllv, in->lcp_dev, N, p->lev[0], derr);
    LICHK(hipGetLastError());
  }
  p->L.nlev = 1;
  while (p->L.n[p->L.nlev - 1] > 1 && p->L.nlev < LI_MAXLEV) {
    const int l = p->L.nlev;
    p->L.n[l] = (p->L.n[l - 1] + 63) / 64;
    LICHK(smax_dev_alloc((void **) &p->lev[l], sizeof (uint32_t) * (p->L.n[l] + LI_PAD)));
    hipLaunchKernelGGL(li_min64_kernel, dim3(li_blocks(p->L.n[l])), dim3(256), 0, s, p->lev[l - 1],
                       p->L.n[l - 1], p->lev[l], p->L.n[l]);
    LICHK(hipGetLastError());
    p->L.nlev++;
  }
  if (p->L.n[p->L.nlev - 1] > 1) {
    li_seterr(errbuf, errlen, "too many suffixes for the minimum hierarchy");
    goto fail;
  }
  for (int l = 0; l < p->L.nlev; l++) p->L.lv[l] = p->lev[l];
  // PL per row, pops per tile, their exclusive scan, the records
  LICHK(smax_dev_alloc(&p->pl, (p->wide ? 8 : 4) * (N ? N : 1)));
  if (p->ntiles > 0) {
    if (p->wide)
      hipLaunchKernelGGL(li_pl_kernel<uint64_t>, dim3(li_tile_grid(p->ntiles)), dim3(LI_TPB), 0, s, p->L, N,
                         p->ntiles, (uint64_t *) p->pl);
    else
      hipLaunchKernelGGL(li_pl_kernel<uint32_t>, dim3(li_tile_grid(p->ntiles)), dim3(LI_TPB), 0, s, p->L, N,
                         p->ntiles, (uint32_t *) p->pl);
    LICHK(hipGetLastError());
  }
  LICHK(smax_dev_alloc(&p->brow, (p->wide ? 8 : 4) * LI_BD * (p->ntiles ? p->ntiles : 1)));
  LICHK(smax_dev_alloc((void **) &p->bx, 4 * LI_BD * (p->ntiles ? p->ntiles : 1)));
  LICHK(smax_dev_alloc((void **) &p->bn, 4 * (p->ntiles ? p->ntiles : 1)));
  if (p->ntiles > 0) {
    if (p->wide)
      hipLaunchKernelGGL(li_bchain_kernel<uint64_t>, dim3(li_blocks(p->ntiles)), dim3(256), 0, s,
                         p->lev[0], (const uint64_t *) p->pl, p->ntiles, (uint64_t *) p->brow, p->bx,
                         p->bn);
    else
      hipLaunchKernelGGL(li_bchain_kernel<uint32_t>, dim3(li_blocks(p->ntiles)), dim3(256), 0, s,
                         p->lev[0], (const uint32_t *) p->pl, p->ntiles, (uint32_t *) p->brow, p->bx,
                         p->bn);
    LICHK(hipGetLastError());
  }
  LICHK(smax_dev_alloc((void **) &tile_cnt, sizeof (uint32_t) * (p->ntiles + 1)));
  LICHK(smax_dev_alloc((void **) &p->tile_off, sizeof (uint64_t) * (p->ntiles + 1)));
  LICHK(hipMemsetAsync(tile_cnt + p->ntiles, 0, sizeof (uint32_t), s));
  if (p->ntiles > 0) {
    if (p->wide)
      hipLaunchKernelGGL(li_tile_count_kernel<uint64_t>, dim3(li_tile_grid(p->ntiles)), dim3(LI_TPB), 0,
                         s, p->lev[0], (const uint64_t *) p->pl, (const uint64_t *) p->brow, p->bx, p->bn, N, p->ntiles, tile_cnt);
    else
      hipLaunchKernelGGL(li_tile_count_kernel<uint32_t>, dim3(li_tile_grid(p->ntiles)), dim3(LI_TPB), 0,
                         s, p->lev[0], (const uint32_t *) p->pl, (const uint32_t *) p->brow, p->bx, p->bn, N, p->ntiles, tile_cnt);
    LICHK(hipGetLastError());
  }
  LICHK(rocprim::exclusive_scan(nullptr, tmp_bytes, tile_cnt, p->tile_off, (uint64_t) 0,
                                (size_t) (p->ntiles + 1), rocprim::plus<uint64_t>(), s));
  LICHK(smax_dev_alloc((void **) &tmp, tmp_bytes ? tmp_bytes : 16));
  LICHK(rocprim::exclusive_scan(tmp, tmp_bytes, tile_cnt, p->tile_off, (uint64_t) 0,
                                (size_t) (p->ntiles + 1), rocprim::plus<uint64_t>(), s));
  LICHK(hipMemcpyAsync(&p->nitv, p->tile_off + p->ntiles, sizeof (uint64_t), hipMemcpyDeviceToHost, s));
  LICHK(hipMemcpyAsync(&herr, derr, sizeof herr, hipMemcpyDeviceToHost, s));
  LICHK(hipStreamSynchronize(s));      // the interval count sizes the records
  if (herr & 1u) { li_seterr(errbuf, errlen, "lcp value >= 2^32-1 in .llv"); goto fail; }
  if (herr & 2u) { li_seterr(errbuf, errlen, "inconsistent .llv entry (lcp byte is not 255)"); goto fail; }
  LICHK(smax_dev_alloc((void **) &p->itv, sizeof (uint64_t) * 5 * (p->nitv ? p->nitv : 1)));
  if (p->ntiles > 0) {
    if (p->wide)
      hipLaunchKernelGGL(li_tile_itv_kernel<uint64_t>, dim3(li_tile_grid(p->ntiles)), dim3(LI_TPB), 0, s,
                         p->lev[0], (const uint64_t *) p->pl, (const uint64_t *) p->brow, p->bx, p->bn, N, p->ntiles, p->tile_off, p->itv, p->first);
    else
      hipLaunchKernelGGL(li_tile_itv_kernel<uint32_t>, dim3(li_tile_grid(p->ntiles)), dim3(LI_TPB), 0, s,
                         p->lev[0], (const uint32_t *) p->pl, (const uint32_t *) p->brow, p->bx, p->bn, N, p->ntiles, p->tile_off, p->itv, p->first);
    LICHK(hipGetLastError());
  }
  smax_marks_record(&p->marks, s);
  {
    // the scratch buffers go back behind the plan's work on s
    SmaxStreamMarks m;
    smax_marks_init(&m);
    smax_marks_record(&m, s);
    SmaxFence *f = smax_marks_fence(&m);
    smax_dev_free_fenced(derr, f);
    smax_dev_free_fenced(tile_cnt, f);
    smax_dev_free_fenced(tmp, f);
    smax_fence_release(f);
  }
  *planp = p;
  return 0;
fail:
  {
    (void) hipStreamSynchronize(s);    // nothing queued may still use a cached block
    void *bufs[] = {derr, tile_cnt, tmp};
    for (size_t i = 0; i < sizeof bufs / sizeof bufs[0]; i++)
      if (bufs[i]) smax_dev_free(bufs[i]);
  }
  smax_marks_record(&p->marks, s);
  gt_lcpitv_plan_delete(p);
  return -1;
}

extern "C" int gt_lcpitv_plan_create(GtLcpitvPlan **planp, const GtLcpitvDevInput *in, char *errbuf,
                                     size_t errlen) {
  if (gt_lcpitv_plan_create_stream(planp, in, NULL, errbuf, errlen) != 0) return -1;
  if (smax_marks_sync(&(*planp)->marks) != hipSuccess) {   // synchronous, as documented
    li_seterr(errbuf, errlen, "lcp-interval tree construction failed");
    gt_lcpitv_plan_delete(*planp);
    *planp = NULL;
    return -1;
  }
  return 0;
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
  const uint64_t N = p->in.nonspecials;
  if (((uintptr_t) events_dev & 15) != 0) return -1;   // 16-byte pieces
  if (hipSetDevice(p->in.device) != hipSuccess) return -1;
  if (N == 0) return 0;
  // the tree (plan create, maybe on another stream) before the events
  if (smax_marks_wait(&p->marks, s) != hipSuccess) return -1;
  const dim3 g(li_tile_grid(p->ntiles)), b(LI_TPB);
  const bool s4 = p->in.suf_dev != nullptr && p->in.suf_bytes == 4;
  const uint32_t *suf4 = s4 ? (const uint32_t *) p->in.suf_dev : nullptr;
  const uint64_t *suf8 = !s4 ? (const uint64_t *) p->in.suf_dev : nullptr;
  if (p->wide) {
    if (s4)
      hipLaunchKernelGGL((li_tile_events_kernel<uint64_t, uint32_t>), g, b, 0, s, p->lev[0],
                         (const uint64_t *) p->pl, (const uint64_t *) p->brow, p->bx, p->bn, N, p->ntiles, p->tile_off, suf4, p->first, events_dev);
    else
      hipLaunchKernelGGL((li_tile_events_kernel<uint64_t, uint64_t>), g, b, 0, s, p->lev[0],
                         (const uint64_t *) p->pl, (const uint64_t *) p->brow, p->bx, p->bn, N, p->ntiles, p->tile_off, suf8, p->first, events_dev);
  } else {
    if (s4)
      hipLaunchKernelGGL((li_tile_events_kernel<uint32_t, uint32_t>), g, b, 0, s, p->lev[0],
                         (const uint32_t *) p->pl, (const uint32_t *) p->brow, p->bx, p->bn, N, p->ntiles, p->tile_off, suf4, p->first, events_dev);
    else
      hipLaunchKernelGGL((li_tile_events_kernel<uint32_t, uint64_t>), g, b, 0, s, p->lev[0],
                         (const uint32_t *) p->pl, (const uint32_t *) p->brow, p->bx, p->bn, N, p->ntiles, p->tile_off, suf8, p->first, events_dev);
  }
  smax_marks_record(&p->marks, s);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// diagnostic: far reads since the last call (current device), -1 on error
extern "C" long long gt_lcpitv_far_reads(void) {
  unsigned long long v = 0, z = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(li_far_reads), sizeof v) != hipSuccess) return -1;
  if (hipMemcpyToSymbol(HIP_SYMBOL(li_far_reads), &z, sizeof z) != hipSuccess) return -1;
  return (long long) v;
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
    LICHK(smax_dev_alloc((void **) &ev, sizeof (uint64_t) * 7 * E));
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
  (void) hipStreamSynchronize(nullptr);   // (the copies above were synchronous)
  smax_dev_free(ev);
  if (host) (void) hipHostFree(host);
  gt_lcpitv_plan_delete(plan);
  li_host_free(&h);
  if (rc != 0) {
    li_seterr(errbuf, errlen, "visitor callback returned non-zero");
    return -1;
  }
  return 0;
fail:
  (void) hipStreamSynchronize(nullptr);
  smax_dev_free(ev);
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
