// lcpitv.hip -- the lcp-interval tree on the GPU and the generic bottom-up
// visitor replay, gfx950.
//
// The reference walks the LCP array once with an explicit stack
// (gt_esa_bottomup, src/match/esa-bottomup.c:116-273), popping every
// lcp-interval [lb..rb] of depth l > 0 at rb and calling the visitor's
// leaf-edge / branching-edge / lcp-interval callbacks.  Here the tree is
// data-parallel, O(1) per row and per interval: two nearest-smaller-value
// quantities of the exact LCP array (strict previous-smaller PL and whether
// a row opens an interval) computed per 2048-row tile in LDS, the depth of
// each row's previous-smaller chain (the reference's stack depth), and one
// exclusive scan of the pops per row (see "the tree" below).  Each row then
// writes the intervals it pops, deepest first, at their pop-order
// positions; the tree stays in HBM
// (GtLcpitvPlan), and the visitor's event stream is generated there too,
// every event at its position in the reference's order: per row idx the
// traversal emits exactly one leaf edge, then for every interval popped at
// idx (pop order) its lcp-interval and branching-edge events, so with
// P(idx) = #intervals with rb < idx the leaf of row idx sits at
// idx + 2 P(idx) and popped interval r of row idx at idx + 2 P(idx) + 1 + 2r.
// The host entry points download the events in chunks and call the
// visitor.
#include <hip/hip_runtime.h>
#include <type_traits>
#include <vector>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <rocprim/iterator/transform_iterator.hpp>
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
  // 16 rows per thread: one 16-byte load (an aligned table) and four
  // 16-byte stores (a byte and a word per row: 2.3 TB/s)
  const bool al = ((uintptr_t) lcp & 15) == 0;
  const uint64_t nq = (N + 1 + 15) / 16;
  LI_FOR(qd, nq) {
    const uint64_t k0 = 16 * qd;
    uint32_t b[16];
    if (al && k0 + 16 <= N) {
      const uint4 v = reinterpret_cast<const uint4 *>(lcp)[qd];
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 16; q++) b[q] = (w[q >> 2] >> (8 * (q & 3))) & 0xffu;
    } else {
#pragma unroll
      for (int q = 0; q < 16; q++) b[q] = k0 + q < N ? (uint32_t) lcp[k0 + q] : 0u;   // X[N] = 0
    }
    if (k0 == 0) b[0] = 0;
    if (k0 + 16 <= N + 1) {
      uint4 *o = reinterpret_cast<uint4 *>(X + k0);
#pragma unroll
      for (int q = 0; q < 4; q++) o[q] = make_uint4(b[4 * q], b[4 * q + 1], b[4 * q + 2], b[4 * q + 3]);
    } else {
#pragma unroll
      for (int q = 0; q < 16; q++)
        if (k0 + q <= N) X[k0 + q] = b[q];
    }
  }
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

// A search reads a level's whole 64-entry block (16-byte pieces, then a bit
// mask of the entries that qualify) instead of one dependent load per
// entry.  Levels are allocated LI_PAD entries long past their end; bits
// past it are masked off.
#define LI_PAD 64
// FAST: all 16 pieces in flight at once (one round trip per level, 64
// VGPRs: pass B, which holds nothing else); else four at a time, for the
// escape paths of the kernels that keep their occupancy
template <bool FAST>
__device__ __forceinline__ uint64_t li_block_mask(const uint32_t *lv, uint64_t b, uint64_t n,
                                                  uint32_t v, bool strict) {
  const uint4 *p = reinterpret_cast<const uint4 *>(lv + b);
  uint64_t m = 0;
  if constexpr (FAST) {
    uint4 t[16];
#pragma unroll
    for (int j = 0; j < 16; j++) t[j] = p[j];
#pragma unroll
    for (int j = 0; j < 16; j++) {
      m |= (uint64_t) (li_ok(t[j].x, v, strict) ? 1u : 0u) << (4 * j);
      m |= (uint64_t) (li_ok(t[j].y, v, strict) ? 1u : 0u) << (4 * j + 1);
      m |= (uint64_t) (li_ok(t[j].z, v, strict) ? 1u : 0u) << (4 * j + 2);
      m |= (uint64_t) (li_ok(t[j].w, v, strict) ? 1u : 0u) << (4 * j + 3);
    }
  } else {
#pragma unroll 4
    for (int j = 0; j < 16; j++) {
      const uint4 t = p[j];
      m |= (uint64_t) (li_ok(t.x, v, strict) ? 1u : 0u) << (4 * j);
      m |= (uint64_t) (li_ok(t.y, v, strict) ? 1u : 0u) << (4 * j + 1);
      m |= (uint64_t) (li_ok(t.z, v, strict) ? 1u : 0u) << (4 * j + 2);
      m |= (uint64_t) (li_ok(t.w, v, strict) ? 1u : 0u) << (4 * j + 3);
    }
  }
  if (n - b < 64) m &= (1ull << (n - b)) - 1;
  return m;
}

// nearest p < k with X[p] < v (strict) / <= v; X[0] == 0 guarantees one
// for v > 0 (strict) and any v (<=)
template <bool FAST>
__device__ static uint64_t li_prev(const LiLevels &L, uint64_t k, uint32_t v, bool strict) {
  uint64_t i = k, p = 0;
  int lev = 0;
  for (;;) {
    const uint64_t b = (i >> 6) << 6;
    const uint64_t below = i - b;   // entries [b, i)
    const uint64_t m = below ? li_block_mask<FAST>(L.lv[lev], b, L.n[lev], v, strict) &
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
    const uint64_t m = li_block_mask<FAST>(L.lv[lev], b, L.n[lev], v, strict);
    p = b + 63 - (uint64_t) __builtin_clzll(m);
  }
  return p;
}

// nearest q > k with X[q] < v (strict) / <= v; X[n-1] == 0 (row N, or the
// last tile's minimum 0) guarantees one for any v when !strict, v > 0 when
// strict
template <bool FAST>
__device__ static uint64_t li_next(const LiLevels &L, uint64_t k, uint32_t v, bool strict) {
  uint64_t i = k, p = 0;
  int lev = 0;
  for (;;) {
    const uint64_t b = (i >> 6) << 6;
    const uint64_t upto = i - b;    // entries (i, b + 64)
    const uint64_t m = upto >= 63 ? 0ull
                                  : li_block_mask<FAST>(L.lv[lev], b, L.n[lev], v, strict) & ~((2ull << upto) - 1ull);
    if (m) { p = b + (uint64_t) __builtin_ctzll(m); break; }
    if (lev + 1 >= L.nlev) return L.n[0] - 1;
    i >>= 6;
    lev++;
  }
  while (lev > 0) {                // first child of p whose subtree qualifies
    lev--;
    const uint64_t b = p << 6;
    p = b + (uint64_t) __builtin_ctzll(li_block_mask<FAST>(L.lv[lev], b, L.n[lev], v, strict));
  }
  return p;
}

// ------------------------------------------------------------ the tree
//
// Every lcp-interval of depth v > 0 has one "rightmost l-index" c: X[c] = v,
// and the nearest q > c with X[q] <= v has X[q] < v (NSE(c) = q, no equal
// value after c inside the interval).  With PL(c) = the nearest p < c with
// X[p] < X[c] (strict previous-smaller value), the interval is
//   [lb, rb] = [PL(c), NSE(c) - 1],  father depth max(X[lb], X[rb + 1]),
//   father lb = PL(lb) when X[lb] >= X[rb + 1], else lb (a new father).
// The reference pops it at row rb (src/match/esa-bottomup.c:154-196): its
// stack after row r holds exactly the PL chain r, PL(r), PL(PL(r)), ...
// (depths strictly decreasing), so with d(k) = the chain's length from k
// (d = 0 where X = 0, d(k) = 1 + d(PL(k))) the interval is the
// (d(rb) - d(c))-th pop of row rb, deepest first, and the number of pops of
// row r is
//   cnt(r) = d(r)                              when X[r+1] = 0,
//   cnt(r) = d(r) - d(r+1) + e(r+1)            else,
// e(k) = 1 when the nearest p < k with X[p] <= X[k] has X[p] < X[k] (k
// opens an interval).  P(r) = the pops of rows < r (an exclusive scan of
// cnt) places every interval: record P(rb) + d(rb) - d(c), events from
// r + 2 P(r) on.  Row r pops exactly the elements of its PL chain with X >
// X[r+1] (every row between such an element c and r lies above X[c], so
// NSE(c) = r + 1), so the records are written by walking those chains: the
// tree is two nearest-smaller-value quantities (PL, e) and one depth per
// row, each O(1) from its neighbours -- no stack walk, no sort.
//
// Pass A, per tile of LI_T rows in LDS: PL and e by comparisons inside each
// thread's 8-row segment (in registers), then the nearest segment with a
// small enough minimum and the nearest qualifying row in it; rows without
// an answer in their tile (the tile's prefix minima, a handful) are
// resolved by pass B over the tile minima (a 64-ary hierarchy) and the
// found tile's resolved suffix-minimum chain.  PL is stored as a u32
// distance (ESC: the rare distance >= 2^32 - 1, found again by search where
// it is read).  Depth: each tile's chain leaves the tile
// through the chain of the row before it (t0-1, PL(t0-1), ...: the
// boundary chain, its first LI_BD entries gathered per tile), so
// d(k) = (steps inside the tile) + D_t - m with D_t = d(t0-1) and m the
// exit's index on that chain; D(t+1) = a_t + b_t D_t is an inclusive scan
// of affine maps over the tiles, then one LDS pointer-jumping pass per
// tile gives every row's d.
#define LI_T 2048                       // rows per tile
#define LI_TPB 256                      // threads per tile workgroup
#define LI_RPT (LI_T / LI_TPB)          // rows per segment (one thread)
#define LI_GSEG 16                      // segments per group
#define LI_NGRP (LI_TPB / LI_GSEG)
#define LI_BD 64                        // boundary-chain entries kept per tile
#define LI_UNRES 0xfffffffeu            // distance not found inside the tile (pass A)
#define LI_ESC 0xffffffffu              // distance >= 2^32 - 1: search again where read
#define LI_EUNRES 2u
#define LI_UCAP 128                     // unresolved entries kept per tile (more: pass B scans the tile)
static_assert(LI_T * 4 <= 65536, "a slot entry (tile row << 2 | kind) fits 16 bits");

__device__ __forceinline__ uint32_t li_dist32(uint64_t dist) {
  return dist >= (uint64_t) LI_UNRES ? LI_ESC : (uint32_t) dist;
}

// LDS rows padded by one word per 8 (row i at i + i/8): a thread's 8-row
// segment is contiguous, and without the pad the 64 lanes' rows 8 apart
// fall on 8 banks
#define LI_PADI(i) ((i) + ((i) >> 3))
#define LI_TPAD (LI_T + LI_T / 8)
#define LI_CH 64                        // chain entries kept per tile (suffix minima)
// a chain's words: [0] length (| 0x80000000 when cut at LI_CH), [4, 4+LI_CH)
// the values, [4+LI_CH, 4+2 LI_CH) the tile-local rows (16-byte aligned
// value block: one round of 16-byte loads reads it whole)
#define LI_CHW (4 + 2 * LI_CH)

struct LiAnsvLds {
  uint32_t x[LI_TPAD];
  int16_t pl[LI_TPAD];                  // tile-local rows, -1: none found
  uint8_t e[LI_TPAD];
  uint32_t wsum[2][LI_TPB / 64];
  alignas(16) uint32_t segmin[LI_TPB];   // (16-byte reads of a group's 16)
  alignas(16) uint32_t grpmin[LI_NGRP];
  uint32_t gsuf[LI_NGRP];                  // minima of the groups after
  uint32_t uw[LI_TPB / 64];                 // unresolved entries per wave
  uint32_t tmin[LI_TPB / 64];
};

// 16 words of LDS (16-byte aligned) into registers
__device__ __forceinline__ void li_load16(const uint32_t *src, uint32_t (&d)[16]) {
  const uint4 *a = reinterpret_cast<const uint4 *>(src);
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint4 u = a[k];
    d[4 * k] = u.x;
    d[4 * k + 1] = u.y;
    d[4 * k + 2] = u.z;
    d[4 * k + 3] = u.w;
  }
}

// bit s: m[s] <= vt
template <int W>
__device__ __forceinline__ uint32_t li_lemask(const uint32_t (&m)[W], uint32_t vt) {
  uint32_t b = 0;
#pragma unroll
  for (int s = 0; s < W; s++) b |= m[s] <= vt ? (1u << s) : 0u;
  return b;
}

// the highest (left: the nearest before) or lowest set bit of b != 0
__device__ __forceinline__ int li_near(uint32_t b, bool left) {
  return left ? 31 - __builtin_clz(b) : __builtin_ctz(b);
}

// nearest segment before tid (after it when !left) whose minimum is <= vt
// (a strict query for v asks vt = v - 1); -1 if none in the tile: the
// minima of the thread's own group of segments, past it the group minima,
// then the hit group's 16 minima (four 16-byte LDS reads each) -- bit masks
// over registers, no dependent LDS chain
__device__ __forceinline__ int li_seg_find(const LiAnsvLds &S, int tid, uint32_t vt, bool left) {
  static_assert(LI_GSEG == 16 && LI_NGRP == 16, "16-bit masks");
  const int g = tid / LI_GSEG, o = tid % LI_GSEG;
  uint32_t smo[LI_GSEG];
  li_load16(S.segmin + g * LI_GSEG, smo);
  uint32_t b = li_lemask(smo, vt) & (left ? (1u << o) - 1u : 0xfffeu << o);
  if (b) return g * LI_GSEG + li_near(b, left);
  uint32_t gm[LI_NGRP];
  li_load16(S.grpmin, gm);
  b = li_lemask(gm, vt) & (left ? (1u << g) - 1u : 0xfffeu << g) & 0xffffu;
  if (!b) return -1;
  const int h = li_near(b, left);
  uint32_t sm[LI_GSEG];
  li_load16(S.segmin + h * LI_GSEG, sm);
  return h * LI_GSEG + li_near(li_lemask(sm, vt), left);
}

// the row of segment s (whose minimum qualifies) nearest its right end
// (from_right) or its left end with X <= vt: eight independent LDS reads
__device__ __forceinline__ int li_seg_row(const LiAnsvLds &S, int s, uint32_t vt, bool from_right) {
  uint32_t xs[LI_RPT];
#pragma unroll
  for (int q = 0; q < LI_RPT; q++) xs[q] = S.x[LI_PADI(s * LI_RPT + q)];
  return s * LI_RPT + li_near(li_lemask(xs, vt), from_right);
}

// pass A: rows [t0, t0 + LI_T) of the N + 1 rows 0..N.  Besides PL and e
// per row it stores the tile's strict suffix minima from the last row (the
// PL chain from there, X strictly decreasing), LI_CH of them, for pass B:
// the nearest row below v before a tile is on it, found by one masked read.
// The rows left unresolved go to the tile's slots for pass B: entries (tile
// row << 2 | kind), kind 0 PL, 1 PLE (e); ucount[t] counts them all, at
// most LI_UCAP are kept (past it pass B scans the tile's rows).  (NSE, the
// next smaller-or-equal value, was computed here too until the interval
// records were written by pop row: 0.84 -> 0.70 ms at C2 without it.)
// One tile per workgroup, tile t_base + blockIdx.x (the host launches the
// tiles past the grid cap in further launches): a tile loop made the
// compiler hoist its per-thread LDS and shuffle addresses out of it, spill
// them (1.4 GB of scratch traffic each way at C2) and reload them per tile.
__global__ void __launch_bounds__(LI_TPB, 6) li_ansv_kernel(const uint32_t *X, uint64_t N, uint64_t t_base,
                                                         uint32_t *pld, uint8_t *eb,
                                                         uint32_t *tmin, uint32_t *sch,
                                                         uint16_t *ulist, uint32_t *ucount) {
  __shared__ LiAnsvLds S;
  const int tid = threadIdx.x, lo = tid * LI_RPT;
  {
    const uint64_t t = t_base + blockIdx.x;
    const uint64_t t0 = t * LI_T;
    {
      // every load issued before the first wait (a load under the row
      // test had made each of the eight wait for the one before)
      uint32_t xv[LI_RPT];
#pragma unroll
      for (int j = 0; j < LI_RPT; j++) {
        const uint64_t g = t0 + (uint64_t) (tid + LI_TPB * j);
        xv[j] = X[g <= N ? g : N];
      }
#pragma unroll
      for (int j = 0; j < LI_RPT; j++) {
        const int k = tid + LI_TPB * j;
        S.x[LI_PADI(k)] = t0 + (uint64_t) k <= N ? xv[j] : 0xffffffffu;   // past row N: never an answer
      }
    }
    __syncthreads();
    // the thread's segment in registers: PLE / PL by comparisons
    // (no data-dependent loop; the pointer-jumping walks over LDS these
    // replace were the kernel's dependent-latency chains)
    uint32_t xr[LI_RPT];
#pragma unroll
    for (int q = 0; q < LI_RPT; q++) xr[q] = S.x[LI_PADI(lo + q)];
    uint32_t m = 0xffffffffu;
#pragma unroll
    for (int q = 0; q < LI_RPT; q++) m = xr[q] < m ? xr[q] : m;
    // queries left for outside the segment: bit 3 r + k, row lo + r, kind k
    // (0: PL, 1: PLE for e); e where the segment decides it (the
    // nearest row before with X <= v has X < v: it is also the nearest with
    // X < v), LI_EUNRES until a query does
    uint32_t qm = 0;
#pragma unroll
    for (int i = 0; i < LI_RPT; i++) {
      int pe = -1, ps = -1;
#pragma unroll
      for (int j = 0; j < i; j++) {
        pe = xr[j] <= xr[i] ? j : pe;      // nearest before with X <= v
        ps = xr[j] < xr[i] ? j : ps;       // nearest before with X < v
      }
      S.pl[LI_PADI(lo + i)] = (int16_t) (ps >= 0 ? lo + ps : -1);
      uint8_t e = 0;
      if (xr[i] > 0 && xr[i] != 0xffffffffu) {
        qm |= ((ps < 0 ? 1u : 0u) | (pe < 0 ? 2u : 0u)) << (3 * i);
        e = pe < 0 ? LI_EUNRES : ps == pe ? 1u : 0u;
      }
      S.e[LI_PADI(lo + i)] = e;
    }
    S.segmin[tid] = m;
    uint32_t wm = m;                     // the wave's minimum, for the tile's
    for (int o = 32; o > 0; o >>= 1) {
      const uint32_t y = __shfl_xor(wm, o, 64);
      wm = y < wm ? y : wm;
    }
    if ((tid & 63) == 0) S.tmin[tid >> 6] = wm;
    __syncthreads();
    if (tid < LI_NGRP) {                 // wave 0, lanes 0..15
      uint32_t g = 0xffffffffu;
      for (int s = tid * LI_GSEG; s < (tid + 1) * LI_GSEG; s++) g = S.segmin[s] < g ? S.segmin[s] : g;
      S.grpmin[tid] = g;
      uint32_t suf = g;                  // inclusive suffix minima over the groups
#pragma unroll
      for (int d = 1; d < LI_NGRP; d <<= 1) {
        const uint32_t c = __shfl_down(suf, d, LI_NGRP);
        if (tid + d < LI_NGRP) suf = c < suf ? c : suf;
      }
      const uint32_t es = __shfl_down(suf, 1, LI_NGRP);
      S.gsuf[tid] = tid + 1 < LI_NGRP ? es : 0xffffffffu;
    }
    if (tid == 0) {
      uint32_t g = S.tmin[0];
      for (int w = 1; w < LI_TPB / 64; w++) g = S.tmin[w] < g ? S.tmin[w] : g;
      tmin[t] = g;
    }
    __syncthreads();
    // the queries, one per lane per round (a lane takes its next one; kinds
    // mixed in one round): the nearest segment with a small enough minimum
    // (li_seg_find), then the nearest qualifying row in it (li_seg_row).
    // Only S.x of other segments is read, so the answers go straight back
    // into the thread's own LDS entries
    while (__ballot(qm != 0) != 0ull) {
      if (qm != 0) {
        const int b = __builtin_ctz(qm);
        qm &= qm - 1u;
        const int r = b / 3, k = b - 3 * r, i = lo + r;
        const uint32_t v = S.x[LI_PADI(i)];
        const uint32_t vt = k == 0 ? v - 1u : v;   // v > 0: X < v is X <= v - 1
        const bool left = k != 2;
        const int sg = li_seg_find(S, tid, vt, left);
        if (sg >= 0) {
          const int row = li_seg_row(S, sg, vt, left);
          if (k == 0) S.pl[LI_PADI(i)] = (int16_t) row;
          else S.e[LI_PADI(i)] = S.x[LI_PADI(row)] < v ? 1u : 0u;
        }
      }
    }
    // the suffix-minimum chain's members (x below every row after them),
    // from the minima of the later segments (rows past N: x = 2^32-1, never
    // members) and a pass over the thread's own rows
    uint32_t after;
    {
      // the other segments of the group (16 consecutive lanes: shuffles
      // of width 16), then the groups before / after
      const int g = tid / LI_GSEG, o = tid % LI_GSEG;
      uint32_t suf = m;
#pragma unroll
      for (int d = 1; d < LI_GSEG; d <<= 1) {
        const uint32_t c = __shfl_down(suf, d, LI_GSEG);
        if (o + d < LI_GSEG) suf = c < suf ? c : suf;
      }
      after = __shfl_down(suf, 1, LI_GSEG);
      if (o == LI_GSEG - 1) after = 0xffffffffu;
      const uint32_t gs = S.gsuf[g];
      after = gs < after ? gs : after;
    }
    uint32_t sflag = 0;
    {
      uint32_t run = after;
#pragma unroll
      for (int q = LI_RPT - 1; q >= 0; q--) {
        if (xr[q] < run) sflag |= 1u << q;
        run = xr[q] < run ? xr[q] : run;
      }
    }
    __syncthreads();
    // ranks: suffix members counted from the right
    {
      const uint32_t cs = (uint32_t) __builtin_popcount(sflag);
      const int lane = tid & 63, wave = tid >> 6;
      uint32_t is = cs;                  // inclusive prefix sums over the workgroup's threads
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t os = __shfl_up(is, d, 64);
        if (lane >= d) is += os;
      }
      if (lane == 63) S.wsum[0][wave] = is;
      __syncthreads();
      uint32_t ws = 0, ts = 0;
      for (int w = 0; w < LI_TPB / 64; w++) {
        if (w < wave) ws += S.wsum[0][w];
        ts += S.wsum[0][w];
      }
      uint32_t *so = sch + t * LI_CHW;
      // suffix members after this thread's: ts - (ws + is)
      uint32_t rs = ts - (ws + is);
#pragma unroll
      for (int q = LI_RPT - 1; q >= 0; q--)
        if (sflag >> q & 1u) {
          if (rs < LI_CH) { so[4 + rs] = xr[q]; so[4 + LI_CH + rs] = (uint32_t) (lo + q); }
          rs++;
        }
      if (tid == 0) so[0] = (ts < LI_CH ? ts : LI_CH) | (ts > LI_CH ? 0x80000000u : 0u);
      if (tid < LI_CH && (uint32_t) tid >= ts) so[4 + tid] = 0;   // (unused value slots: masked by the length)
    }
    // the rows' words, coalesced (row tid + 256 j), and the unresolved list
    uint32_t umask = 0;
    for (int j = 0; j < LI_RPT; j++) {
      const int i = tid + LI_TPB * j;
      const uint64_t k = t0 + (uint64_t) i;
      if (k > N) break;
      const uint32_t v = S.x[LI_PADI(i)];
      uint32_t dpl = 0;
      uint8_t e = 0;
      if (v > 0) {
        const int p = S.pl[LI_PADI(i)];
        dpl = p >= 0 ? (uint32_t) (i - p) : LI_UNRES;
        e = S.e[LI_PADI(i)];
      }
      pld[k] = dpl;
      eb[k] = e;
      umask |= ((dpl == LI_UNRES ? 1u : 0u) | (e == LI_EUNRES ? 2u : 0u))
               << (3 * j);
    }
    {
      // the tile's own slots (no device-wide counter: one returning atomic
      // per wave on a single word had bounded the kernel at ~88 of them per
      // microsecond, 2.2 ms at C2): the workgroup's prefix of the counts
      const uint32_t c = (uint32_t) __builtin_popcount(umask);
      const int lane = tid & 63, wave = tid >> 6;
      uint32_t incl = c;
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(incl, d, 64);
        if (lane >= d) incl += o;
      }
      if (lane == 63) S.uw[wave] = incl;
      __syncthreads();
      uint32_t at = incl - c, tot = 0;
      for (int w = 0; w < LI_TPB / 64; w++) {
        if (w < wave) at += S.uw[w];
        tot += S.uw[w];
      }
      uint16_t *ul = ulist + t * LI_UCAP;
      while (umask) {
        const int b = __builtin_ctz(umask);
        umask &= umask - 1;
        if (at < LI_UCAP) ul[at] = (uint16_t) (((tid + LI_TPB * (b / 3)) << 2) | (b % 3));
        at++;
      }
      if (tid == 0) ucount[t] = tot;
    }
  }
}

// PL / PLE (strict / !strict) of row k with value v > 0 by search: the
// nearest tile before with a small enough minimum, then the first entry of
// that tile's suffix-minimum chain with a small enough value, by binary
// search; a chain cut at LI_CH entries is followed on in HBM (pass A
// resolved every row on it inside the tile)
struct LiTree {                         // what the searches need
  LiLevels TL;                          // tile minima and their hierarchy
  const uint32_t *sch;                  // the tiles' suffix-minimum chains
};

template <bool FAST>
__device__ uint64_t li_search_prev(const LiTree &T, const uint32_t *X, const uint32_t *pld,
                                   uint64_t k, uint32_t v, bool strict) {
  const uint64_t t = k / LI_T;
  if (t == 0) return 0;                  // (never: X[0] = 0 lies in tile 0)
  const uint64_t s = li_prev<FAST>(T.TL, t, v, strict);
  const uint32_t *ch = T.sch + s * LI_CHW;
  const int n = (int) (ch[0] & 0xffffu);
  // the first entry with X < v (<= v) -- X strictly decreasing along the
  // chain -- from one read of the value block
  const uint64_t m = li_block_mask<FAST>(ch + 4, 0, (uint64_t) n, v, strict);
  if (m) return s * LI_T + ch[4 + LI_CH + __builtin_ctzll(m)];
  uint64_t p = s * LI_T + ch[4 + LI_CH + n - 1];   // past the entries held
  while (strict ? X[p] >= v : X[p] > v) p -= pld[p];
  return p;
}


// pass B: the rows pass A left unresolved, about 20 per tile.  Four rows
// per thread per step, their words read as 16-byte pieces; the searches
// (one 16-byte piece of a level's block per load, all in flight) run only
// on the rare lanes that found an unresolved row.
// pass B: one search per open row, from the tiles' slots packed densely, or
// (a tile with more open rows than its slots hold) every open row of it
__device__ __forceinline__ void li_resolve_one(const LiTree &T, const uint32_t *X, uint64_t k,
                                               uint32_t kind, uint32_t *pld, uint8_t *eb) {
  const uint32_t v = X[k];
  if (kind == 0) pld[k] = li_dist32(k - li_search_prev<true>(T, X, pld, k, v, true));
  else eb[k] = X[li_search_prev<true>(T, X, pld, k, v, false)] < v ? 1u : 0u;
}

// entries a tile's slots hold (a tile past them resolves its rows itself)
struct LiSlotLen {
  const uint32_t *ucount;
  __device__ __host__ uint32_t operator()(uint64_t t) const {
    const uint32_t n = ucount[t];
    return n <= LI_UCAP ? n : 0u;
  }
};

// the slots packed into one dense list at their scanned offsets (row << 2 |
// kind), a wave per tile; a tile past its slots scans its own rows here.
// *ntot = the list's length (written by the last tile)
__global__ void __launch_bounds__(256) li_compact_slots_kernel(LiTree T, const uint32_t *X, uint64_t N,
                                                               uint64_t ntiles, const uint16_t *ulist,
                                                               const uint32_t *ucount, const uint32_t *uoff,
                                                               uint64_t *dense, uint32_t *ntot,
                                                               uint32_t *pld, uint8_t *eb) {
  const int lane = threadIdx.x & 63;
  for (uint64_t t = blockIdx.x * 4ull + (threadIdx.x >> 6); t < ntiles; t += 4ull * gridDim.x) {
    const uint32_t n = ucount[t];
    const uint64_t t0 = t * LI_T;
    if (n <= LI_UCAP) {
      const uint64_t base = uoff[t];
      for (uint32_t j = lane; j < n; j += 64) {
        const uint32_t w = ulist[t * LI_UCAP + j];
        dense[base + j] = ((t0 + (w >> 2)) << 2) | (uint64_t) (w & 3u);
      }
    } else {
      for (int i = lane; i < LI_T; i += 64) {
        const uint64_t k = t0 + (uint64_t) i;
        if (k > N || X[k] == 0) continue;
        if (pld[k] == LI_UNRES) li_resolve_one(T, X, k, 0u, pld, eb);
        if (eb[k] == LI_EUNRES) li_resolve_one(T, X, k, 1u, pld, eb);
      }
    }
    if (t == ntiles - 1 && lane == 0) *ntot = uoff[t] + (n <= LI_UCAP ? n : 0u);
  }
}

// the dense list, one search per entry, every lane busy (a wave per tile
// woke 64 lanes for ~20 searches: 0.24 ms at C2)
__global__ void __launch_bounds__(256) li_resolve_list_kernel(LiTree T, const uint32_t *X,
                                                              const uint64_t *dense, const uint32_t *ntot,
                                                              uint32_t *pld, uint8_t *eb) {
  const uint64_t n = *ntot;
  for (uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; i < n;
       i += (uint64_t) gridDim.x * blockDim.x) {
    const uint64_t w = dense[i];
    li_resolve_one(T, X, w >> 2, (uint32_t) (w & 3u), pld, eb);
  }
}

// PL of row k (X[k] = v > 0) from the distances, searching on escape
__device__ __forceinline__ uint64_t li_pl(const LiTree &T, const uint32_t *X, const uint32_t *pld,
                                          uint64_t k, uint32_t v) {
  const uint32_t d = pld[k];
  return d != LI_ESC ? k - d : li_search_prev<false>(T, X, pld, k, v, true);
}


// each tile's boundary chain t0-1, PL(t0-1), ... down to the first X = 0
// entry, at most LI_BD entries (one thread per tile: a chain of dependent
// loads, thousands in flight)
__global__ void __launch_bounds__(256) li_bchain_kernel(LiTree T, const uint32_t *X, const uint32_t *pld,
                                                        uint64_t N, uint64_t ntiles, uint64_t *brow,
                                                        uint32_t *bx, uint32_t *bn) {
  LI_FOR(t, ntiles) {
    int k = 0;
    if (t > 0) {
      uint64_t s = t * LI_T - 1;
      while (k < LI_BD) {
        const uint32_t xs = X[s];
        brow[t * LI_BD + k] = s;
        bx[t * LI_BD + k] = xs;
        k++;
        if (xs == 0) break;
        s = li_pl(T, X, pld, s, xs);
      }
    }
    bn[t] = (uint32_t) k;
  }
}

// the index of row o on tile t's boundary chain (o lies on it, X[o] > 0):
// binary search over the entries held (rows strictly decreasing), else the
// chain followed on past them
__device__ int64_t li_bindex_far(const LiTree &T, const uint32_t *X, const uint32_t *pld,
                                              const uint64_t *brow, uint64_t t, uint64_t o) {
  int64_t m = LI_BD - 1;
  uint64_t s = brow[t * LI_BD + LI_BD - 1];
  while (s != o && X[s] > 0) {       // (o is on the chain: the guard only bounds the loop)
    s = li_pl(T, X, pld, s, X[s]);
    m++;
  }
  return m;
}

__device__ __forceinline__ int64_t li_bindex(const LiTree &T, const uint32_t *X, const uint32_t *pld,
                                             const uint64_t *brow, uint32_t nb, uint64_t t,
                                             uint64_t o) {
  int lo = 0, hi = (int) nb - 1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    const uint64_t r = brow[t * LI_BD + mid];
    if (r == o) return mid;
    if (r > o) lo = mid + 1; else hi = mid - 1;
  }
  return li_bindex_far(T, X, pld, brow, t, o);
}

// the affine map D(t+1) = a_t + b_t D_t of tile t: its last row's chain
// inside the tile, then where it leaves (one thread per tile)
struct LiAffine {
  int64_t a;
  int64_t b;
};

struct LiAffineCompose {
  __device__ __host__ LiAffine operator()(const LiAffine &f, const LiAffine &g) const {
    return LiAffine{g.a + g.b * f.a, g.b * f.b};   // g after f
  }
};

__global__ void __launch_bounds__(256) li_tail_kernel(LiTree T, const uint32_t *X, const uint32_t *pld,
                                                      uint64_t N, uint64_t ntiles, const uint64_t *brow,
                                                      const uint32_t *bn, LiAffine *aff) {
  LI_FOR(t, ntiles) {
    const uint64_t t0 = t * LI_T;
    const uint64_t last = (t0 + LI_T <= N + 1 ? t0 + LI_T : N + 1) - 1;
    int64_t steps = 0;
    uint64_t c = last;
    uint32_t xc = X[c];
    LiAffine f{0, 0};
    while (xc > 0) {
      steps++;
      const uint64_t p = li_pl(T, X, pld, c, xc);
      const uint32_t xp = X[p];
      if (p < t0 && xp > 0) {
        f.a = steps - li_bindex(T, X, pld, brow, bn[t], t, p);
        f.b = 1;
        break;
      }
      c = p;
      xc = xp;
    }
    if (f.b == 0) f.a = steps;
    aff[t] = f;
  }
}

// d of every row: per tile, pointer jumping in LDS over PL inside the tile;
// a chain leaving it ends on the boundary chain at index m, d = steps +
// D_t - m (Dt[t] = D_t from the scan of the affine maps)
struct LiDepthLds {
  int32_t anc[2][LI_T];                  // >= 0: tile row; -1: d known; -2 - m: exit at chain index m
  uint32_t dist[2][LI_T];
  uint64_t brow[LI_BD];                  // the tile's boundary chain: rows, X
  uint32_t bx[LI_BD];
};

__global__ void __launch_bounds__(LI_TPB) li_depth_kernel(LiTree T, const uint32_t *X, const uint32_t *pld,
                                                          const uint8_t *eb, uint64_t N, uint64_t ntiles,
                                                          const uint64_t *brow, const uint32_t *bx,
                                                          const uint32_t *bn, const LiAffine *scan,
                                                          uint32_t *dep, uint32_t *cnt) {
  __shared__ LiDepthLds S;
  const int tid = threadIdx.x;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint64_t t0 = t * LI_T;
    const int nrows = N + 1 - t0 < LI_T ? (int) (N + 1 - t0) : LI_T;
    const int64_t Dt = t == 0 ? 0 : scan[t - 1].a;
    // the tile's X and PL distances staged in the second buffers (free
    // until the first round), every load issued before the first wait; X
    // and e stay in registers for the pop counts at the end
    uint32_t xv[LI_RPT], ev[LI_RPT];
    {
      uint32_t dv[LI_RPT];
#pragma unroll
      for (int j = 0; j < LI_RPT; j++) {
        const uint64_t k = t0 + (uint64_t) (tid + LI_TPB * j);
        const uint64_t kc = k <= N ? k : N;
        xv[j] = X[kc];
        dv[j] = pld[kc];
        ev[j] = eb[kc];
      }
#pragma unroll
      for (int j = 0; j < LI_RPT; j++) {
        S.anc[1][tid + LI_TPB * j] = (int32_t) xv[j];
        S.dist[1][tid + LI_TPB * j] = dv[j];
      }
      if (tid < LI_BD) {                 // the boundary chain's held entries
        S.brow[tid] = brow[t * LI_BD + tid];
        S.bx[tid] = bx[t * LI_BD + tid];
      }
    }
    const int nb = (int) bn[t];
    __syncthreads();
    // a parent inside the tile is a row index; one before it (the tile's
    // prefix minima, a few rows) its place on the boundary chain
    for (int i = tid; i < LI_T; i += LI_TPB) {
      const uint64_t k = t0 + (uint64_t) i;
      int32_t anc = -1;
      uint32_t dist = 0;
      if (i < nrows) {
        const uint32_t v = (uint32_t) S.anc[1][i], d = S.dist[1][i];
        if (v > 0) {
          const uint64_t p = d != LI_ESC ? k - d : li_search_prev<false>(T, X, pld, k, v, true);
          dist = 1;
          if (p >= t0) {
            anc = (int32_t) (p - t0);
          } else {
            // p is on the boundary chain: its index by a binary search of
            // the held entries in LDS (rows strictly decreasing), X beside
            // it; past them the chain is followed in HBM (li_bindex_far)
            int lo = 0, hi = nb - 1, m = -1;
            while (lo <= hi) {
              const int mid = (lo + hi) >> 1;
              const uint64_t r = S.brow[mid];
              if (r == p) { m = mid; break; }
              if (r > p) lo = mid + 1; else hi = mid - 1;
            }
            if (m >= 0) {
              if (S.bx[m] > 0) anc = (int32_t) (-2 - m);
            } else if (X[p] > 0) {
              anc = (int32_t) (-2 - li_bindex_far(T, X, pld, brow, t, p));
            }
          }
        }
      }
      S.anc[0][i] = anc;
      S.dist[0][i] = dist;
    }
    __syncthreads();
    // (at most 11 rounds: 2^11 = LI_T; a tile's chains are short, so the
    // rounds stop once no row points inside the tile any more)
    int cur = 0;
    for (int round = 0; round < 12; round++) {
      int open = 0;
      for (int i = tid; i < LI_T; i += LI_TPB) {
        int32_t a = S.anc[cur][i];
        uint32_t d = S.dist[cur][i];
        if (a >= 0) {
          d += S.dist[cur][a];
          a = S.anc[cur][a];
        }
        open |= a >= 0;
        S.anc[cur ^ 1][i] = a;
        S.dist[cur ^ 1][i] = d;
      }
      cur ^= 1;
      if (!__syncthreads_or(open)) break;
    }
    for (int i = tid; i < nrows; i += LI_TPB) {
      const int32_t a = S.anc[cur][i];
      int64_t d = S.dist[cur][i];
      if (a <= -2) d += Dt - (int64_t) (-2 - a);
      dep[t0 + i] = (uint32_t) d;
      S.dist[cur ^ 1][i] = (uint32_t) d;   // (the other buffer is free)
    }
    __syncthreads();
    // pops of row r = t0 + i - 1 (the row before the tile: its d is D_t):
    // cnt(r) = d(r) when X[r+1] = 0, else d(r) - d(r+1) + e(r+1) -- the
    // scan's input, so that it reads one word per row
#pragma unroll
    for (int j = 0; j < LI_RPT; j++) {
      const int i = tid + LI_TPB * j;
      const uint64_t r1 = t0 + (uint64_t) i;
      if (i >= nrows) break;
      if (r1 == N) cnt[N] = 0;
      if (r1 == 0) continue;
      const uint32_t d1 = S.dist[cur ^ 1][i];
      const uint32_t d0 = i > 0 ? S.dist[cur ^ 1][i - 1] : (uint32_t) Dt;
      cnt[r1 - 1] = xv[j] == 0 ? d0 : d0 - d1 + ev[j];
    }
    __syncthreads();
  }
}

// the interval records (lcp, lb, rb, father lcp, father lb) in pop order,
// one per rightmost l-index; and the stream position of the first edge to
// the root (the reference's firstedgefromroot, esa-bottomup.c:134-141)
// a chain element of the tile's rows: its row, X, and where it lies -- in
// the tile (m < 0, !far), on the boundary chain's held entries (m >= 0), or
// past them (far: followed in HBM)
struct LiElem {
  uint64_t row;
  uint32_t x;
  int m;
  bool far;
};

struct LiItvLds {
  uint32_t x[LI_T + 1];                  // X of the tile's rows and the row after
  uint32_t d[LI_T];                      // their PL distances
  uint64_t brow[LI_BD];                  // the boundary chain's held entries
  uint32_t bx[LI_BD];
};

// PL of chain element e (X > 0)
__device__ __forceinline__ LiElem li_itv_next(const LiItvLds &S, const LiTree &T, const uint32_t *X,
                                              const uint32_t *pld, uint64_t t0, int nb, const LiElem &e) {
  LiElem n;
  n.m = -1;
  n.far = false;
  if (!e.far && e.m < 0) {
    const uint32_t d = S.d[e.row - t0];
    n.row = d != LI_ESC ? e.row - d : li_search_prev<false>(T, X, pld, e.row, e.x, true);
    if (n.row >= t0) {
      n.x = S.x[n.row - t0];
      return n;
    }
    int lo = 0, hi = nb - 1;             // rows strictly decreasing
    while (lo <= hi) {
      const int mid = (lo + hi) >> 1;
      const uint64_t r = S.brow[mid];
      if (r == n.row) { n.m = mid; break; }
      if (r > n.row) lo = mid + 1; else hi = mid - 1;
    }
    if (n.m >= 0) n.x = S.bx[n.m];
    else { n.far = true; n.x = X[n.row]; }
    return n;
  }
  if (!e.far && e.m + 1 < nb) {
    n.m = e.m + 1;
    n.row = S.brow[n.m];
    n.x = S.bx[n.m];
    return n;
  }
  n.far = true;
  n.row = li_pl(T, X, pld, e.row, e.x);
  n.x = X[n.row];
  return n;
}

// The interval records by pop row, a tile per workgroup: row r pops the
// first elements of its PL chain r, PL(r), ... -- exactly those with X >
// X[r+1] (every row between a chain element c and r is above X[c], so
// NSE(c) = r + 1) -- deepest first, records P(r), P(r) + 1, ...; the
// interval of element c is [PL(c), r], PL(c) the chain's next element.  The
// tile's X and PL distances and its boundary chain (the chain every row of
// the tile continues on once it leaves the tile: t0 - 1, PL(t0 - 1), ...)
// are in LDS, so a chain step is an LDS read, and neighbouring lanes write
// neighbouring records.  (One thread per rightmost l-index, each record's
// position from P and the depths: 1.3 ms at C2, its 40-byte records
// scattered; the same pop-row walk over HBM: 1.85 ms.)
template <typename PT>
__global__ void __launch_bounds__(LI_TPB) li_itv_kernel(LiTree T, const uint32_t *X, const uint32_t *pld,
                                                        const PT *P, uint64_t N, uint64_t t_base,
                                                        const uint64_t *brow, const uint32_t *bx,
                                                        const uint32_t *bn, uint64_t *itv,
                                                        unsigned long long *first) {
  __shared__ LiItvLds S;
  const int tid = threadIdx.x;
  const uint64_t t = t_base + blockIdx.x, t0 = t * LI_T;
  uint64_t pv[LI_RPT];                   // P of the thread's rows (loaded with X and PL)
  {
    uint32_t xv[LI_RPT], dv[LI_RPT];
#pragma unroll
    for (int j = 0; j < LI_RPT; j++) {
      const uint64_t k = t0 + (uint64_t) (tid + LI_TPB * j);
      const uint64_t kc = k <= N ? k : N;
      xv[j] = X[kc];
      dv[j] = pld[kc];
      pv[j] = (uint64_t) P[kc];
    }
#pragma unroll
    for (int j = 0; j < LI_RPT; j++) {
      const int i = tid + LI_TPB * j;
      S.x[i] = t0 + (uint64_t) i <= N ? xv[j] : 0u;
      S.d[i] = dv[j];
    }
    if (tid == 0) S.x[LI_T] = t0 + LI_T <= N ? X[t0 + LI_T] : 0u;
    if (tid < LI_BD) {
      S.brow[tid] = brow[t * LI_BD + tid];
      S.bx[tid] = bx[t * LI_BD + tid];
    }
  }
  const int nb = (int) bn[t];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < LI_RPT; j++) {
    const int i = tid + LI_TPB * j;
    const uint64_t r = t0 + (uint64_t) i;
    if (r >= N) break;
    const uint32_t xr = S.x[i], x1 = S.x[i + 1];
    const uint64_t pr = pv[j];
    if (xr == 0) {
      if (x1 == 0) atomicMin(first, (unsigned long long) (r + 2 * pr));
      continue;
    }
    LiElem c;
    c.row = r;
    c.x = xr;
    c.m = -1;
    c.far = false;
    uint64_t *w = itv + 5 * pr;
    for (uint64_t q = 0; c.x > x1; q++) {
      const LiElem lb = li_itv_next(S, T, X, pld, t0, nb, c);
      const uint32_t fd = lb.x > x1 ? lb.x : x1;
      uint64_t flb = lb.row;
      if (fd == 0) flb = 0;
      else if (lb.x >= x1) flb = li_itv_next(S, T, X, pld, t0, nb, lb).row;
      w[0] = c.x;
      w[1] = lb.row;
      w[2] = r;
      w[3] = fd;
      w[4] = flb;
      w += 5;
      if (fd == 0) atomicMin(first, (unsigned long long) (r + 2 * pr + 2 + 2 * q));
      c = lb;
    }
  }
}

// the gt_esa_bottomup event stream, every event at its position in the
// reference's order: per row its leaf edge, then per pop its lcp-interval
// and branching-edge events
//   (0, firstsucc, fd, flb, leafnumber, 0, 0)   visit_leaf_edge
//   (2, 0, lcp, lb, rb, 0, 0)                   visit_lcp_interval
//   (1, firstsucc, fd, flb, sd, slb, srb)       visit_branching_edge
// A workgroup takes 256 rows at a time: the rows' leaf data and the
// chunk's interval records (P(r0) .. P(r0 + 256), consecutive) are read
// coalesced and staged as one 4-word descriptor per event (the branching
// edge takes sd, slb, srb from the lcp-interval event before it), then the
// chunk's 7-word records are stored as aligned 16-byte pieces; events past
// the stage go straight to memory.
#define LI_EV_STAGE 16384               // event staging bytes per workgroup

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

template <typename PT, typename SufT, typename DT>
__global__ void __launch_bounds__(256, 8) li_events_kernel(LiTree T, const uint32_t *X, const uint32_t *pld,
                                                        const PT *P, const uint64_t *itv, uint64_t N,
                                                        const SufT *suf, const unsigned long long *firstp,
                                                        uint64_t *ev) {
  __shared__ __attribute__((aligned(16))) unsigned char stage_bytes[LI_EV_STAGE];
  __shared__ uint64_t sP[2];
  LiDesc<DT> *stage = reinterpret_cast<LiDesc<DT> *>(stage_bytes);
  constexpr uint32_t cap = LI_EV_STAGE / sizeof (LiDesc<DT>);
  const uint64_t first = *firstp;
  const uint64_t nchunks = (N + 255) / 256;
  for (uint64_t ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    const uint64_t r0 = ch * 256;
    const uint64_t r = r0 + threadIdx.x;
    const bool row = r < N;
    // the row's data and the chunk's record range
    uint64_t Pr = 0, leaf = 0, flb = 0;
    uint32_t xr = 0, y = 0;
    if (row) {
      Pr = P[r];
      xr = X[r];
      y = X[r + 1];
      leaf = suf != nullptr ? (uint64_t) suf[r] : 0u;
      if (y <= xr && xr > 0) flb = li_pl(T, X, pld, r, xr);
    }
    if (threadIdx.x == 0) {
      sP[0] = P[r0];
      sP[1] = P[r0 + 256 <= N ? r0 + 256 : N];
    }
    __syncthreads();
    const uint64_t k0 = sP[0], k1 = sP[1];
    const uint64_t nrows = N - r0 < 256 ? N - r0 : 256;
    const uint64_t E = nrows + 2 * (k1 - k0);     // the chunk's events
    const uint64_t ebase = r0 + 2 * k0;           // stream position of its first
    if (row) {
      const uint64_t off = (r - r0) + 2 * (Pr - k0);
      uint64_t fs, fd, fl;
      if (y <= xr) {
        fs = (xr == 0 && ebase + off == first) ? 1u : 0u;
        fd = xr;
        fl = flb;
      } else {
        fs = 1;
        fd = y;
        fl = r;
      }
      if (off < cap) {
        stage[off] = LiDesc<DT>{(DT) (fs << 2), (DT) fd, (DT) fl, (DT) leaf};
      } else {
        uint64_t *w = ev + 7 * (ebase + off);
        w[0] = 0; w[1] = fs; w[2] = fd; w[3] = fl; w[4] = leaf; w[5] = 0; w[6] = 0;
      }
    }
    for (uint64_t k = k0 + threadIdx.x; k < k1; k += 256) {
      const uint64_t *rec = itv + 5 * k;
      const uint64_t lcp = rec[0], lb = rec[1], rb = rec[2], fd = rec[3], fl = rec[4];
      const uint64_t slot = (rb - r0) + 2 * (k - k0) + 1;
      const bool newfather = fd > 0 && fl == lb;
      const uint64_t bfs = newfather ? 1u : (fd == 0 && ebase + slot + 1 == first) ? 1u : 0u;
      if (slot < cap) stage[slot] = LiDesc<DT>{(DT) 2, (DT) lcp, (DT) lb, (DT) rb};
      if (slot + 1 < cap) {
        stage[slot + 1] = LiDesc<DT>{(DT) (1u | (bfs << 2)), (DT) fd, (DT) fl, (DT) 0};
      } else {
        uint64_t *w = ev + 7 * (ebase + slot);
        if (slot >= cap) { w[0] = 2; w[1] = 0; w[2] = lcp; w[3] = lb; w[4] = rb; w[5] = 0; w[6] = 0; }
        w[7] = 1; w[8] = bfs; w[9] = fd; w[10] = fl; w[11] = lcp; w[12] = lb; w[13] = rb;
      }
    }
    __syncthreads();
    const uint64_t staged = E < cap ? E : cap;
    const uint64_t w0 = 7 * ebase, w1 = 7 * (ebase + staged);
    for (uint64_t q = (w0 >> 1) + threadIdx.x; 2 * q < w1; q += 256) {
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
    __syncthreads();
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
  bool wide;                     // rows past 2^32: 64-bit P
  uint64_t ntiles;
  uint32_t *X;                   // exact LCP, rows 0..N
  uint32_t *pld, *dep;           // PL distances, chain depths
  uint8_t *eb;                   // e (row opens an interval)
  uint32_t *tlev[LI_MAXLEV];     // tile minima and their 64-ary hierarchy
  uint32_t *sch;                 // the tiles' suffix-minimum chains
  LiTree T;                      // the searches' view of them
  void *P;                       // pops before each row (u32, u64 when wide), N + 1
  uint64_t nitv;
  uint64_t *itv;                 // 5 * nitv, pop order
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
  void *bufs[] = {p->X, p->pld, p->dep, p->eb, p->P, p->itv, p->first, p->sch};
  for (size_t i = 0; i < sizeof bufs / sizeof bufs[0]; i++) smax_dev_free_fenced(bufs[i], fence);
  for (int l = 0; l < LI_MAXLEV; l++) smax_dev_free_fenced(p->tlev[l], fence);
  smax_fence_release(fence);
  free(p);
}

template <typename PT>
static hipError_t li_scan_pops(GtLcpitvPlan *p, const uint32_t *cnt_in, hipStream_t s, void **tmp,
                               size_t *tmp_bytes) {
  const uint64_t N = p->in.nonspecials;
  const uint32_t *cnt = cnt_in;         // pops per row (li_depth_kernel), cnt[N] = 0
  size_t b = 0;
  hipError_t e = rocprim::exclusive_scan(nullptr, b, cnt, (PT *) p->P, (PT) 0, (size_t) (N + 1),
                                         rocprim::plus<PT>(), s);
  if (e != hipSuccess) return e;
  if (b > *tmp_bytes) {
    if (*tmp) {
      e = hipStreamSynchronize(s);
      if (e != hipSuccess) return e;
      smax_dev_free(*tmp);
      *tmp = NULL;
    }
    e = smax_dev_alloc(tmp, b);
    if (e != hipSuccess) return e;
    *tmp_bytes = b;
  }
  return rocprim::exclusive_scan(*tmp, b, cnt, (PT *) p->P, (PT) 0, (size_t) (N + 1),
                                 rocprim::plus<PT>(), s);
}

extern "C" int gt_lcpitv_plan_create_stream(GtLcpitvPlan **planp, const GtLcpitvDevInput *in,
                                            void *stream, char *errbuf, size_t errlen) {
  GtLcpitvPlan *p = NULL;
  hipStream_t s = (hipStream_t) stream;
  uint32_t *derr = NULL, herr = 0, *bx = NULL, *bn = NULL, nitv32 = 0;
  uint16_t *ulist = NULL;
  uint32_t *ucount = NULL, *cnt = NULL, *uoff = NULL, *ntot = NULL;
  uint64_t *dense = NULL;
  void *stmp = NULL;                   // the slot-count scan's temporary
  uint64_t *brow = NULL;
  LiAffine *aff = NULL, *affs = NULL;
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
  p->ntiles = (N + 1 + LI_T - 1) / LI_T;     // rows 0..N
  LICHK(hipSetDevice(in->device));
  LICHK(smax_dev_alloc((void **) &derr, sizeof (uint32_t)));
  LICHK(hipMemsetAsync(derr, 0, sizeof (uint32_t), s));
  LICHK(smax_dev_alloc((void **) &p->first, sizeof (unsigned long long)));
  LICHK(hipMemcpyAsync(p->first, &none, sizeof none, hipMemcpyHostToDevice, s));
  // exact LCP
  LICHK(smax_dev_alloc((void **) &p->X, sizeof (uint32_t) * (N + 1 + LI_PAD)));
  hipLaunchKernelGGL(li_expand_kernel, dim3(li_blocks((N + 16) / 16)), dim3(256), 0, s, in->lcp_dev, N, p->X);
  LICHK(hipGetLastError());
  if (in->numllv > 0) {
    hipLaunchKernelGGL(li_llv_kernel, dim3(li_blocks(in->numllv)), dim3(256), 0, s, in->llv_dev,
                       in->numllv, in->lcp_dev, N, p->X, derr);
    LICHK(hipGetLastError());
  }
  // pass A: PL and e inside the tiles; the tile minima and their hierarchy
  LICHK(smax_dev_alloc((void **) &p->pld, sizeof (uint32_t) * (N + 1)));
  LICHK(smax_dev_alloc((void **) &p->eb, N + 1));
  p->T.TL.n[0] = p->ntiles;
  LICHK(smax_dev_alloc((void **) &p->tlev[0], sizeof (uint32_t) * (p->ntiles + LI_PAD)));
  LICHK(smax_dev_alloc((void **) &p->sch, sizeof (uint32_t) * LI_CHW * p->ntiles));
  LICHK(smax_dev_alloc((void **) &ulist, sizeof (uint16_t) * LI_UCAP * p->ntiles));
  LICHK(smax_dev_alloc((void **) &ucount, sizeof (uint32_t) * p->ntiles));
  LICHK(smax_dev_alloc((void **) &uoff, sizeof (uint32_t) * p->ntiles));
  LICHK(smax_dev_alloc((void **) &dense, sizeof (uint64_t) * LI_UCAP * p->ntiles));
  LICHK(smax_dev_alloc((void **) &ntot, sizeof (uint32_t)));
  for (uint64_t tb = 0; tb < p->ntiles; tb += LI_MAX_BLOCKS) {
    const uint64_t nb = p->ntiles - tb < LI_MAX_BLOCKS ? p->ntiles - tb : LI_MAX_BLOCKS;
    hipLaunchKernelGGL(li_ansv_kernel, dim3((unsigned) nb), dim3(LI_TPB), 0, s, p->X, N, tb, p->pld,
                       p->eb, p->tlev[0], p->sch, ulist, ucount);
    LICHK(hipGetLastError());
  }
  p->T.TL.nlev = 1;
  while (p->T.TL.n[p->T.TL.nlev - 1] > 1 && p->T.TL.nlev < LI_MAXLEV) {
    const int l = p->T.TL.nlev;
    p->T.TL.n[l] = (p->T.TL.n[l - 1] + 63) / 64;
    LICHK(smax_dev_alloc((void **) &p->tlev[l], sizeof (uint32_t) * (p->T.TL.n[l] + LI_PAD)));
    hipLaunchKernelGGL(li_min64_kernel, dim3(li_blocks(p->T.TL.n[l])), dim3(256), 0, s, p->tlev[l - 1],
                       p->T.TL.n[l - 1], p->tlev[l], p->T.TL.n[l]);
    LICHK(hipGetLastError());
    p->T.TL.nlev++;
  }
  if (p->T.TL.n[p->T.TL.nlev - 1] > 1) {
    li_seterr(errbuf, errlen, "too many suffixes for the minimum hierarchy");
    goto fail;
  }
  for (int l = 0; l < p->T.TL.nlev; l++) p->T.TL.lv[l] = p->tlev[l];
  p->T.sch = p->sch;
  // pass B
  {
    auto lens = rocprim::make_transform_iterator(rocprim::make_counting_iterator<uint64_t>(0),
                                                 LiSlotLen{ucount});
    size_t b = 0;
    LICHK(rocprim::exclusive_scan(nullptr, b, lens, uoff, 0u, (size_t) p->ntiles, rocprim::plus<uint32_t>(), s));
    LICHK(smax_dev_alloc(&stmp, b ? b : 16));
    LICHK(rocprim::exclusive_scan(stmp, b, lens, uoff, 0u, (size_t) p->ntiles, rocprim::plus<uint32_t>(), s));
    hipLaunchKernelGGL(li_compact_slots_kernel, dim3(li_tile_grid((p->ntiles + 3) / 4)), dim3(256), 0, s,
                       p->T, p->X, N, p->ntiles, ulist, ucount, uoff, dense, ntot, p->pld, p->eb);
    LICHK(hipGetLastError());
    hipLaunchKernelGGL(li_resolve_list_kernel, dim3(li_blocks(32 * p->ntiles)), dim3(256), 0, s, p->T, p->X,
                       dense, ntot, p->pld, p->eb);
    LICHK(hipGetLastError());
  }
  LICHK(hipGetLastError());
  // depths: boundary chains, the tiles' affine maps and their scan, d
  LICHK(smax_dev_alloc((void **) &brow, sizeof (uint64_t) * LI_BD * p->ntiles));
  LICHK(smax_dev_alloc((void **) &bx, sizeof (uint32_t) * LI_BD * p->ntiles));
  LICHK(smax_dev_alloc((void **) &bn, sizeof (uint32_t) * p->ntiles));
  LICHK(smax_dev_alloc((void **) &aff, sizeof (LiAffine) * p->ntiles));
  LICHK(smax_dev_alloc((void **) &affs, sizeof (LiAffine) * p->ntiles));
  LICHK(smax_dev_alloc((void **) &p->dep, sizeof (uint32_t) * (N + 1)));
  hipLaunchKernelGGL(li_bchain_kernel, dim3(li_blocks(p->ntiles)), dim3(256), 0, s, p->T, p->X, p->pld, N,
                     p->ntiles, brow, bx, bn);
  LICHK(hipGetLastError());
  hipLaunchKernelGGL(li_tail_kernel, dim3(li_blocks(p->ntiles)), dim3(256), 0, s, p->T, p->X, p->pld, N,
                     p->ntiles, brow, bn, aff);
  LICHK(hipGetLastError());
  {
    size_t b = 0;
    LICHK(rocprim::inclusive_scan(nullptr, b, aff, affs, (size_t) p->ntiles, LiAffineCompose(), s));
    LICHK(smax_dev_alloc(&tmp, b ? b : 16));
    tmp_bytes = b ? b : 16;
    LICHK(rocprim::inclusive_scan(tmp, b, aff, affs, (size_t) p->ntiles, LiAffineCompose(), s));
  }
  LICHK(smax_dev_alloc((void **) &cnt, sizeof (uint32_t) * (N + 1)));
  hipLaunchKernelGGL(li_depth_kernel, dim3(li_tile_grid(p->ntiles)), dim3(LI_TPB), 0, s, p->T, p->X, p->pld,
                     p->eb, N, p->ntiles, brow, bx, bn, affs, p->dep, cnt);
  LICHK(hipGetLastError());
  // pops per row, their exclusive scan P (P[N] = intervals), the records
  LICHK(smax_dev_alloc(&p->P, (p->wide ? 8 : 4) * (N + 1)));
  LICHK(p->wide ? li_scan_pops<uint64_t>(p, cnt, s, &tmp, &tmp_bytes)
                : li_scan_pops<uint32_t>(p, cnt, s, &tmp, &tmp_bytes));
  if (p->wide)
    LICHK(hipMemcpyAsync(&p->nitv, (uint64_t *) p->P + N, sizeof (uint64_t), hipMemcpyDeviceToHost, s));
  else
    LICHK(hipMemcpyAsync(&nitv32, (uint32_t *) p->P + N, sizeof (uint32_t), hipMemcpyDeviceToHost, s));
  LICHK(hipMemcpyAsync(&herr, derr, sizeof herr, hipMemcpyDeviceToHost, s));
  LICHK(hipStreamSynchronize(s));      // the interval count sizes the records
  if (!p->wide) p->nitv = nitv32;
  if (herr & 1u) { li_seterr(errbuf, errlen, "lcp value >= 2^32-1 in .llv"); goto fail; }
  if (herr & 2u) { li_seterr(errbuf, errlen, "inconsistent .llv entry (lcp byte is not 255)"); goto fail; }
  LICHK(smax_dev_alloc((void **) &p->itv, sizeof (uint64_t) * 5 * (p->nitv ? p->nitv : 1)));
  if (N > 0) {
    for (uint64_t tb = 0; tb < p->ntiles; tb += LI_MAX_BLOCKS) {
      const uint64_t nb = p->ntiles - tb < LI_MAX_BLOCKS ? p->ntiles - tb : LI_MAX_BLOCKS;
      if (p->wide)
        hipLaunchKernelGGL(li_itv_kernel<uint64_t>, dim3((unsigned) nb), dim3(LI_TPB), 0, s, p->T, p->X,
                           p->pld, (const uint64_t *) p->P, N, tb, brow, bx, bn, p->itv, p->first);
      else
        hipLaunchKernelGGL(li_itv_kernel<uint32_t>, dim3((unsigned) nb), dim3(LI_TPB), 0, s, p->T, p->X,
                           p->pld, (const uint32_t *) p->P, N, tb, brow, bx, bn, p->itv, p->first);
      LICHK(hipGetLastError());
    }
  }
  smax_marks_record(&p->marks, s);
  {
    // the scratch buffers go back behind the plan's work on s (the tree
    // keeps X, PL, P and the records for the events pass)
    SmaxStreamMarks m;
    smax_marks_init(&m);
    smax_marks_record(&m, s);
    SmaxFence *f = smax_marks_fence(&m);
    void *bufs[] = {derr, brow, bx, bn, aff, affs, tmp, ulist, ucount, cnt, uoff, dense, ntot, stmp, p->dep, p->eb};
    for (size_t i = 0; i < sizeof bufs / sizeof bufs[0]; i++) smax_dev_free_fenced(bufs[i], f);
    smax_fence_release(f);
    p->dep = NULL;
    p->eb = NULL;
  }
  *planp = p;
  return 0;
fail:
  {
    (void) hipStreamSynchronize(s);    // nothing queued may still use a cached block
    void *bufs[] = {derr, brow, bx, bn, aff, affs, tmp, ulist, ucount, cnt, uoff, dense, ntot, stmp};
    for (size_t i = 0; i < sizeof bufs / sizeof bufs[0]; i++) smax_dev_free(bufs[i]);
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

template <typename PT, typename SufT>
static void li_launch_events(GtLcpitvPlan *p, hipStream_t s, const SufT *suf, uint64_t *ev) {
  using DT = typename std::conditional<(sizeof (PT) >= sizeof (SufT)), PT, SufT>::type;
  const uint64_t N = p->in.nonspecials;
  hipLaunchKernelGGL((li_events_kernel<PT, SufT, DT>), dim3(li_blocks(N)), dim3(256), 0, s, p->T, p->X,
                     p->pld, (const PT *) p->P, p->itv, N, suf, p->first, ev);
}

extern "C" int gt_lcpitv_plan_events(GtLcpitvPlan *p, uint64_t *events_dev, void *stream) {
  hipStream_t s = (hipStream_t) stream;
  const uint64_t N = p->in.nonspecials;
  if (((uintptr_t) events_dev & 15) != 0) return -1;   // 16-byte pieces
  if (hipSetDevice(p->in.device) != hipSuccess) return -1;
  if (N == 0) return 0;
  // the tree (plan create, maybe on another stream) before the events
  if (smax_marks_wait(&p->marks, s) != hipSuccess) return -1;
  const bool s4 = p->in.suf_dev != nullptr && p->in.suf_bytes == 4;
  const uint32_t *suf4 = s4 ? (const uint32_t *) p->in.suf_dev : nullptr;
  const uint64_t *suf8 = !s4 ? (const uint64_t *) p->in.suf_dev : nullptr;
  if (p->wide) {
    if (s4) li_launch_events<uint64_t, uint32_t>(p, s, suf4, events_dev);
    else li_launch_events<uint64_t, uint64_t>(p, s, suf8, events_dev);
  } else {
    if (s4) li_launch_events<uint32_t, uint32_t>(p, s, suf4, events_dev);
    else li_launch_events<uint32_t, uint64_t>(p, s, suf8, events_dev);
  }
  smax_marks_record(&p->marks, s);
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
