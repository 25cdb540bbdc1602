// maxpairs.hip -- maximal pairs (`gt repfind -l N`) and
// on-device sequence/position mapping of position pairs (§8(f) F4), gfx950.
//
// The reference enumerates maximal pairs with the stack-based bottom-up
// traversal of src/match/esa-bottomup-maxpairs.inc:136-264: per lcp-interval
// of depth >= minlen it keeps per-left-symbol position lists and emits the
// cartesian products between a new child (leaf or branching edge) and the
// interval's earlier children whose left symbols differ
// (src/match/esa-maxpairs.c:181-360).  A pair of suffix-array rows i < j is
// therefore emitted exactly once, at their lowest common interval, of depth
// L = min LCP[i+1..j], when L >= minlen and their left contexts differ
// (BWT >= 254 -- wildcard, separator, position 0's INITIALCHAR -- differs
// from everything, ISLEFTDIVERSE, src/match/esa-maxpairs.c:24-31).
//
// Data-parallel form used here: every row j walks back over the rows of its
// "block" (the maximal run with LCP >= minlen) keeping the running minimum
// of LCP, i.e. the depth of the lowest common interval with row i, and
// counts (pass 1) or writes (pass 2) the pairs whose left contexts differ.
// The rows with LCP[j] >= minlen (the only ones with a non-empty walk) are
// listed first (16 rows per thread per 16-byte load, per-workgroup counts,
// scan, ordered write); then one lane per listed row counts its pairs, an
// exclusive scan of the counts gives every row its output offset, and the
// emission pass writes the pairs without atomics.  The walk reads X (exact LCP,
// u32) and BWT 8 rows per step (neighbouring lanes walk neighbouring rows:
// each step of a wave is one contiguous segment), so the loop-carried
// minimum never waits on a single load.
//
// Integer/byte work; bound by the number of (row, earlier row in block)
// candidates, i.e. by the output size.  No MFMA.
//
// Reference emission order (gt_maxpairs_plan_emit_ordered, the host entry
// points): the traversal calls GtProcessmaxpairs at "events" -- a leaf
// joining its interval (processleafedge, src/match/esa-maxpairs.c:181-240)
// or a finished child interval merging into its father (processbranchingedge,
// :242-360) -- in iteration order, and within an iteration the leaf first,
// then the pops from the deepest.  A pair of rows x < y of depth L is
// emitted at the event that brings y's unit (y itself, or the child of the
// depth-L interval holding y) into that interval; its iteration is
// t = min{k >= y : LCP[k+1] <= L}, and (t, -L) orders the events.  Inside an
// event the cartesian loops order the pairs by left-symbol class (symbols,
// then "unique" >= 254 last) and by row, since every per-symbol position
// list is a contiguous slice filled in row order:
//   leaf event (max(LCP[y], LCP[y+1]) == L):  (class x, x)
//   branch event, x in the father, y in the child:
//     class x, class y < 254:  (class x, class y, x, y)
//     class x < 254, y unique: (class x, 254, y, x)
//     x unique:                (254, x, class y, y)
// The emission pass writes these keys beside the triples and three or four
// stable LSD radix sorts give the permutation.  t comes from a 64-ary
// minimum hierarchy over the exact LCP (one "next value <= L" search per
// distinct depth of a walk).
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_reduce.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_scan_by_key.hpp>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gt_maxpairs_hip.h"
#include "smax_internal.h"

static void mp_seterr(char *errbuf, size_t errlen, const char *fmt, ...) {
  if (errbuf == NULL || errlen == 0) return;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(errbuf, errlen, fmt, ap);
  va_end(ap);
}

#define MPCHK(call)                                                          \
  do {                                                                       \
    hipError_t e_ = (call);                                                  \
    if (e_ != hipSuccess) {                                                  \
      mp_seterr(errbuf, errlen, "%s: %s (%s:%d)", #call, hipGetErrorString(e_), \
                __FILE__, __LINE__);                                         \
      goto fail;                                                             \
    }                                                                        \
  } while (0)

#define MP_STEP 8     // rows per walk step

// grid-stride loop over [0, n) of a 1-D launch (mp_blocks caps the grid)
#define MP_FOR(i, n)                                                          \
  for (uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x,         \
                i##_stride = (uint64_t) gridDim.x * blockDim.x;               \
       i < (n); i += i##_stride)
#define MP_MAX_BLOCKS (1ull << 22)   // 2^30 work-items: fills the chip many times

// ------------------------------------------------------------ kernels

// X[k] = exact LCP[k] for k in [0, N] (0 at k = 0 and k = N; the 255 bytes
// are overwritten by mp_llv_kernel).  A3 decoding, src/match/esa-seqread.h:96-215.
__global__ void __launch_bounds__(256) mp_expand_kernel(const uint8_t *lcp, uint64_t N,
                                                        uint32_t *X) {
  // 255 bytes are marked until their .llv value arrives (mp_llv_kernel)
  MP_FOR(k, N + 1)
    X[k] = (k == 0 || k == N) ? 0u : (lcp[k] == 255 ? 0xffffffffu : (uint32_t) lcp[k]);
}

// .llv values over their 255 bytes; err bit 1: value >= 2^32, bit 2: a
// position whose byte is not 255 (inconsistent index)
__global__ void __launch_bounds__(256) mp_llv_kernel(const GtSmaxLlv *llv, uint64_t numllv,
                                                     const uint8_t *lcp, uint64_t N, uint32_t *X,
                                                     uint32_t *err) {
  MP_FOR(e, numllv) {
    const uint64_t pos = llv[e].position, v = llv[e].value;
    if (pos < 1 || pos >= N) continue;
    if (v >= 0xffffffffull) atomicOr(err, 1u);
    if (lcp[pos] != 255) atomicOr(err, 2u);
    X[pos] = (uint32_t) v;
  }
}

// heads of the runs of equal BWT symbols (specials >= 254 are runs of one:
// they differ from every symbol) for a max-scan to the run start
__global__ void __launch_bounds__(256) mp_run_heads_kernel(const uint8_t *B, uint64_t N,
                                                           uint64_t *hv) {
  MP_FOR(r, N + 1) {
    const uint32_t b = B[r];
    hv[r] = (r == 0 || b >= 254u || B[r - 1] != b) ? r : 0;
  }
}

// RO[r] = r - (first row of r's run), from the scanned run starts
__global__ void __launch_bounds__(256) mp_run_off_kernel(const uint64_t *rs, uint64_t N,
                                                         uint32_t *RO) {
  MP_FOR(r, N + 1) {
    const uint64_t d = r - rs[r];
    RO[r] = d > 0xffffffffull ? 0xffffffffu : (uint32_t) d;
  }
}

// a .lcp byte 255 whose row no .llv entry overwrote (X still holds the mark)
__global__ void __launch_bounds__(256) mp_llv_check_kernel(const uint32_t *X, uint64_t N,
                                                           uint32_t *err) {
  MP_FOR(k, N)
    if (X[k] == 0xffffffffu) atomicOr(err, 4u);
}

template <typename SufT>
__device__ __forceinline__ uint64_t suf_at(const void *S, uint64_t k) {
  return (uint64_t) reinterpret_cast<const SufT *>(S)[k];
}

// 64-ary minimum hierarchy over X[0..N]: lv[0] = X, lv[l][i] = min of
// lv[l-1][64i .. 64i+63]; the top level has <= 64 entries.
#define MP_HMAX 8
struct MpHier {
  const uint32_t *lv[MP_HMAX];
  uint64_t n[MP_HMAX];
  int levels;
};

// first k >= a with X[k] <= v (X[N] == 0: always found for a <= N)
__device__ uint64_t mp_next_le(const MpHier &h, uint64_t a, uint32_t v) {
  uint64_t idx = a;
  int l = 0;
  for (;;) {
    const uint64_t g = ((idx >> 6) + 1) << 6;
    const uint64_t end = g < h.n[l] ? g : h.n[l];
    uint64_t k = idx;
    while (k < end && h.lv[l][k] > v) k++;
    if (k < end) { idx = k; break; }
    if (l + 1 >= h.levels) return h.n[0] - 1;     // unreachable for valid tables
    idx = (idx >> 6) + 1;
    l++;
  }
  while (l > 0) {
    l--;
    uint64_t k = idx << 6;
    while (h.lv[l][k] > v) k++;                    // a child holds the minimum
    idx = k;
  }
  return idx;
}

// sort keys of the reference emission order (see the header), per pair
struct MpKeys {
  uint64_t *k1, *k2, *k3, *k4;   // r2 | (classes, r1) | event | t (split)
  int rowbits, lbits;            // rows < 2^rowbits, depths < 2^lbits
  int split;                     // rowbits + lbits > 64: t in k4, depth in k3
  uint32_t *rank0;               // when set: zeroed beside the keys (mp_rank_kernel's counts)
};

// Walk of row j: counts (EMIT = false) or writes at out[o..] (EMIT = true)
// the maximal pairs (i, j), i < j.  The early exit reads the LCP byte only
// (exact below 255), so rows outside blocks cost one byte.  A run of >= 8
// earlier rows sharing j's left symbol (no pairs with j) is skipped in one
// step: RO[r] = rows between r and the first row of its run of equal BWT
// symbols, RM[r] = min X over that run up to r -- so a walk costs its pairs
// plus one step per run, not the rows of its block (a homopolymer block of
// L rows with one left symbol: O(L) instead of O(L^2)).
template <bool EMIT, typename SufT, bool ORD = false>
__device__ __forceinline__ uint32_t mp_walk(const uint8_t *lcp, const uint32_t *X, const uint8_t *B,
                                            const uint32_t *RM, const uint32_t *RO,
                                            const void *S, uint64_t j, uint32_t minlen,
                                            uint64_t o, uint64_t *out, uint64_t capacity,
                                            const MpHier *h = nullptr, const MpKeys *K = nullptr) {
  const uint32_t m8 = lcp[j];
  if (j == 0 || (m8 < 255u && m8 < minlen)) return 0;
  uint32_t m = X[j];                       // depth of the pair (j-1, j)
  if (m < minlen) return 0;
  uint32_t c = 0;
  const uint32_t bj = B[j];
  const bool uj = bj >= 254u;              // unique left context
  const uint64_t sj = EMIT ? suf_at<SufT>(S, j) : 0;
  // ORD: event of the current depth (recomputed when the depth drops)
  const uint32_t xj = m, xj1 = ORD ? X[j + 1] : 0u;
  const uint64_t cy = uj ? 254u : bj;
  uint32_t ev_l = 0xffffffffu;
  uint64_t ev_k = j + 1, ev_key3 = 0, ev_key4 = 0;
  bool ev_leaf = false;
  int64_t i = (int64_t) j - 1;
  bool more = true;
  while (more) {
    uint32_t xi[MP_STEP], bi[MP_STEP];
    uint64_t si[MP_STEP];
#pragma unroll
    for (int q = 0; q < MP_STEP; q++) {
      const int64_t r = i - q;
      xi[q] = r >= 0 ? X[r] : 0u;
      bi[q] = r >= 0 ? (uint32_t) B[r] : 0u;
      si[q] = (EMIT && r >= 0) ? suf_at<SufT>(S, (uint64_t) r) : 0;
    }
    int64_t inext = i - MP_STEP;
#pragma unroll
    for (int q = 0; q < MP_STEP; q++) {
      if (!more) break;
      // row i-q pairs with j at depth m = min LCP[i-q+1 .. j]
      if (uj || bi[q] != bj) {
        if (EMIT && o + c < capacity) {
          uint64_t *w = out + 3 * (o + c);
          w[0] = m;
          if (!ORD) {                      // row-order pass: (len, pos1 < pos2)
            w[1] = si[q] < sj ? si[q] : sj;
            w[2] = si[q] < sj ? sj : si[q];
          }
          if (ORD) {
            if (m != ev_l) {
              ev_l = m;
              ev_k = mp_next_le(*h, ev_k, m);          // t = ev_k - 1
              ev_leaf = (xj > xj1 ? xj : xj1) == m;
              const uint64_t t = ev_k - 1;
              const uint64_t ld = ((1ull << K->lbits) - 1) - m;   // deeper first
              if (K->split) { ev_key3 = ld; ev_key4 = t; }
              else { ev_key3 = (t << K->lbits) | ld; }
            }
            const uint64_t x = (uint64_t) (i - q), y = j, rb = (uint64_t) K->rowbits;
            const uint64_t cx = bi[q] >= 254u ? 254u : bi[q];
            uint64_t cls, r1, r2;
            if (ev_leaf) { cls = cx << 8; r1 = x; r2 = 0; }
            else if (cx < 254u && cy < 254u) { cls = (cx << 8) | cy; r1 = x; r2 = y; }
            else if (cx < 254u) { cls = (cx << 8) | 254u; r1 = y; r2 = x; }
            else { cls = 254u << 8; r1 = x; r2 = (cy << rb) | y; }
            // the argument order of the reference's GtProcessmaxpairs call:
            // a leaf edge passes (new leaf, earlier position)
            // (src/match/esa-maxpairs.c:128,261), a branching edge (father's
            // position, son's) except when the son's position has a unique
            // left symbol and the father's not (cartproduct1 with the son's
            // position as the "leaf", :128 via :307-312)
            const bool later_first = ev_leaf || (cx < 254u && cy >= 254u);
            w[1] = later_first ? sj : si[q];
            w[2] = later_first ? si[q] : sj;
            const uint64_t e = o + c;
            K->k1[e] = r2;
            K->k2[e] = (cls << rb) | r1;
            K->k3[e] = ev_key3;
            if (K->split) K->k4[e] = ev_key4;
            if (K->rank0) K->rank0[e] = 0;
          }
        }
        c++;
      } else if (i - q >= 0) {
        const uint64_t r = (uint64_t) (i - q);
        const uint32_t ro = RO[r];
        if (ro >= MP_STEP) {               // long run of j's left symbol: jump over it
          const uint32_t rm = RM[r];
          m = rm < m ? rm : m;
          if (m < minlen) more = false;
          inext = (int64_t) (r - ro) - 1;
          break;
        }
      }
      m = xi[q] < m ? xi[q] : m;           // X[0] == 0 ends every walk
      if (m < minlen) more = false;
    }
    i = inext;
    if (i < 0) more = false;
  }
  return c;
}

// workgroup-wide exclusive prefix (u64) of one value per thread; *total = sum
__device__ __forceinline__ uint64_t mp_block_excl(uint64_t v, uint64_t *total) {
  __shared__ uint64_t sW[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t o = __shfl_up(incl, d, 64);
    if (lane >= d) incl += o;
  }
  if (lane == 63) sW[wave] = incl;
  __syncthreads();
  uint64_t wo = 0;
  for (int w = 0; w < wave; w++) wo += sW[w];
  *total = sW[0] + sW[1] + sW[2] + sW[3];
  return wo + incl - v;
}

// Candidate rows (LCP[j] >= minlen, j >= 1: rows whose walk is not empty),
// found per workgroup of MP_WG_ROWS rows: every thread tests 16 consecutive
// rows with one 16-byte LCP load (byte >= min(minlen, 255), exact below
// 255).  Pass A counts them per workgroup, pass B (after a scan of those
// counts) writes them to one global list in row order.  The walks then run
// one lane per candidate row (passes C and D), so neighbouring lanes walk
// neighbouring rows (coalesced) and a long block spreads over the device.
#define MP_ROWS 16
#define MP_WG_ROWS (256 * MP_ROWS)

__device__ __forceinline__ uint32_t mp_candidates(const uint8_t *lcp, uint64_t j0, uint64_t N,
                                                  uint32_t mf) {
  uint4 v = make_uint4(0, 0, 0, 0);
  if (j0 + MP_ROWS <= N) {
    v = *reinterpret_cast<const uint4 *>(lcp + j0);
  } else {
    for (int q = 0; q < MP_ROWS; q++)
      if (j0 + q < N) reinterpret_cast<uint8_t *>(&v)[q] = lcp[j0 + q];
  }
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t m = 0;
#pragma unroll
  for (int q = 0; q < MP_ROWS; q++)
    m |= (((w[q >> 2] >> (8 * (q & 3))) & 0xffu) >= mf ? 1u : 0u) << q;
  if (j0 == 0) m &= ~1u;                   // row 0 has no earlier row
  return m;
}

__global__ void __launch_bounds__(256)
mp_cand_count_kernel(const uint8_t *lcp, uint64_t N, uint32_t mf, uint64_t *wg_cand,
                     uint16_t *masks) {
  const uint64_t j0 = blockIdx.x * (uint64_t) MP_WG_ROWS + threadIdx.x * (uint64_t) MP_ROWS;
  const uint32_t m = mp_candidates(lcp, j0, N, mf);
  masks[blockIdx.x * (uint64_t) 256 + threadIdx.x] = (uint16_t) m;
  uint64_t tot;
  (void) mp_block_excl((uint64_t) __popc(m), &tot);
  if (threadIdx.x == 0) wg_cand[blockIdx.x] = tot;
}

// pass B reads pass A's 16-row masks (2 B per 16 rows), not the LCP bytes;
// one workgroup per MP_WR_GROUP of pass A's workgroups, 4 masks (64 rows)
// per thread: one 8-byte load each (a workgroup per pass-A workgroup, one
// mask per thread: 15.5 us for C2's 12.5 MB)
#define MP_WR_GROUP 4
__global__ void __launch_bounds__(256)
mp_cand_write_kernel(const uint16_t *masks, const uint64_t *wg_cand_off, uint64_t *list) {
  const uint64_t k0 = (uint64_t) blockIdx.x * (256 * MP_WR_GROUP) + 4u * threadIdx.x;
  uint64_t m = *reinterpret_cast<const uint64_t *>(masks + k0);
  uint64_t tot;
  uint64_t pos = wg_cand_off[(uint64_t) blockIdx.x * MP_WR_GROUP] +
                 mp_block_excl((uint64_t) __popcll(m), &tot);
  const uint64_t j0 = k0 * MP_ROWS;
  while (m) {
    const int q = __builtin_ctzll(m);
    m &= m - 1;
    list[pos++] = j0 + q;
  }
}

// Single-pass pass C + scan (small candidate lists): each workgroup
// publishes its total in a status word, then looks back over its
// predecessors' words for the nearest inclusive prefix, adding the
// aggregates before it, and publishes its own inclusive prefix (decoupled
// look-back); the whole workgroup looks back, 1024 words per round trip.  A
// status word is [tag:16 | flag:2 | value:46], the tag the pass's number, so
// no pass clears the words of the last.  Used only where every workgroup of
// the grid looks back within one window (mp_count_grid <= MP_LB_MAX_WG): for
// the 6,104-workgroup candidate list of C2 the same look-back cost 66-78 us
// on top of the 25 us stream, even with no waiting at all (the status
// loads and write-through stores themselves; profiles/s7/f2_lookback.txt),
// against 5 us for rocprim's scan between two passes.
#define MP_ST_AGG (1ull << 46)
#define MP_ST_INC (2ull << 46)
#define MP_ST_VAL (MP_ST_AGG - 1)
#define MP_LB_PER 4   // status words per thread per look-back step
#define MP_LB_MAX_WG 64   // (measured at C2's 18 workgroups: 8.9-11.6 us against 16.1)

// all 256 threads of workgroup bid: the exclusive prefix of its total tot
__device__ uint64_t mp_lookback(uint64_t *status, uint64_t bid, uint64_t tot, uint64_t tag) {
  __shared__ uint32_t sNear;
  const uint64_t tg = tag << 48;
  if (bid == 0) {
    if (threadIdx.x == 0)
      __hip_atomic_store(&status[0], tg | MP_ST_INC | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return 0;
  }
  if (threadIdx.x == 0)
    __hip_atomic_store(&status[bid], tg | MP_ST_AGG | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint64_t excl = 0;
  int64_t base = (int64_t) bid;
  for (;;) {
    // one poller per workgroup, backing off, on the nearest word of the
    // window before the window's 1024 loads (every thread of ~2000 resident
    // workgroups re-polling its words saturated the L2s: 103 us)
    if (threadIdx.x == 0) {
      uint32_t nap = 1;
      while ((__hip_atomic_load(&status[base - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 48) != tag) {
        for (uint32_t z = 0; z < nap; z++) __builtin_amdgcn_s_sleep(8);
        nap = nap < 32 ? 2 * nap : 32;
      }
    }
    __syncthreads();
    uint64_t st[MP_LB_PER];
#pragma unroll
    for (int u = 0; u < MP_LB_PER; u++) {   // word u of thread t: predecessor base-1-(t*PER+u)
      const int64_t idx = base - 1 - (int64_t) (threadIdx.x * MP_LB_PER + u);
      st[u] = idx >= 0 ? __hip_atomic_load(&status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                       : (tg | MP_ST_INC);
    }
#pragma unroll
    for (int u = 0; u < MP_LB_PER; u++) {
      const int64_t idx = base - 1 - (int64_t) (threadIdx.x * MP_LB_PER + u);
      uint32_t nap = 1;
      while ((st[u] >> 48) != tag) {
        for (uint32_t z = 0; z < nap; z++) __builtin_amdgcn_s_sleep(8);
        nap = nap < 32 ? 2 * nap : 32;
        st[u] = __hip_atomic_load(&status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    uint32_t near = 0xffffffffu;   // this thread's nearest inclusive word
#pragma unroll
    for (int u = MP_LB_PER - 1; u >= 0; u--)
      if (st[u] & MP_ST_INC) near = threadIdx.x * MP_LB_PER + u;
    if (threadIdx.x == 0) sNear = 0xffffffffu;
    __syncthreads();
    if (near != 0xffffffffu) atomicMin(&sNear, near);
    __syncthreads();
    const uint32_t k = sNear;
    uint64_t v = 0;
#pragma unroll
    for (int u = 0; u < MP_LB_PER; u++)
      if (threadIdx.x * MP_LB_PER + u <= k) v += st[u] & MP_ST_VAL;
    uint64_t sum;
    (void) mp_block_excl(v, &sum);
    excl += sum;
    __syncthreads();   // sNear and mp_block_excl's LDS before the next step
    if (k != 0xffffffffu) break;
    base -= 256 * MP_LB_PER;
  }
  if (threadIdx.x == 0)
    __hip_atomic_store(&status[bid], tg | MP_ST_INC | (excl + tot), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  return excl;
}

// Pass C: pairs per candidate row.
template <typename SufT>
__global__ void __launch_bounds__(256)
mp_count_kernel(const uint8_t *lcp, const uint32_t *X, const uint8_t *B, const uint32_t *RM,
                const uint32_t *RO, const uint64_t *list, uint64_t ncand, uint32_t minlen,
                uint32_t *cnt) {
  MP_FOR(e, ncand)
    cnt[e] = mp_walk<false, SufT>(lcp, X, B, RM, RO, nullptr, list[e], minlen, 0, nullptr, 0);
}

// passes C + scan + total in one: workgroup b owns candidates
// [b * 256 * R, (b + 1) * 256 * R) (R > 1 only past 2^30 candidates, the grid
// cap), their counts, exclusive offsets and, from the last workgroup, the
// total
template <typename SufT>
__global__ void __launch_bounds__(256)
mp_count_scan_kernel(const uint8_t *lcp, const uint32_t *X, const uint8_t *B, const uint32_t *RM,
                     const uint32_t *RO, const uint64_t *list, uint64_t ncand, uint32_t minlen,
                     uint32_t R, uint64_t *status, uint64_t tag, uint32_t *cnt, uint64_t *off,
                     uint64_t *total) {
  const uint64_t e0 = (uint64_t) blockIdx.x * 256u * R;
  uint64_t run = 0, loc0 = 0;
  uint32_t c0 = 0;
  for (uint32_t r = 0; r < R; r++) {   // the first 256 stay in registers
    const uint64_t e = e0 + (uint64_t) r * 256u + threadIdx.x;
    const uint32_t c = e < ncand ? mp_walk<false, SufT>(lcp, X, B, RM, RO, nullptr, list[e], minlen, 0,
                                                        nullptr, 0)
                                 : 0u;
    uint64_t t;
    const uint64_t loc = mp_block_excl((uint64_t) c, &t);
    if (r == 0) {
      c0 = c;
      loc0 = loc;
    } else if (e < ncand) {
      cnt[e] = c;
      off[e] = run + loc;
    }
    run += t;
    __syncthreads();   // mp_block_excl's LDS before its next use
  }
  const uint64_t pre = mp_lookback(status, blockIdx.x, run, tag);
  if (threadIdx.x == 0 && blockIdx.x == gridDim.x - 1) *total = pre + run;
  if (e0 + threadIdx.x < ncand) {
    cnt[e0 + threadIdx.x] = c0;
    off[e0 + threadIdx.x] = pre + loc0;
  }
  if (pre)
    for (uint32_t r = 1; r < R; r++) {
      const uint64_t e = e0 + (uint64_t) r * 256u + threadIdx.x;
      if (e < ncand) off[e] += pre;
    }
}

// Pass D: the pairs of every candidate row at its scanned offset,
// (len, pos1 < pos2).
template <typename SufT>
__global__ void __launch_bounds__(256)
mp_emit_kernel(const uint8_t *lcp, const uint32_t *X, const uint8_t *B, const uint32_t *RM,
               const uint32_t *RO, const void *S, const uint64_t *list, uint64_t ncand,
               uint32_t minlen, const uint32_t *cnt, const uint64_t *off, uint64_t *out,
               uint64_t capacity) {
  MP_FOR(e, ncand) {
    if (cnt[e] == 0) continue;
    (void) mp_walk<true, SufT>(lcp, X, B, RM, RO, S, list[e], minlen, off[e], out, capacity);
  }
}

// Pass D with the emission-order keys of every pair
template <typename SufT>
__global__ void __launch_bounds__(256)
mp_emit_ord_kernel(const uint8_t *lcp, const uint32_t *X, const uint8_t *B, const uint32_t *RM,
                   const uint32_t *RO, const void *S, const uint64_t *list, uint64_t ncand,
                   uint32_t minlen, const uint32_t *cnt, const uint64_t *off, uint64_t *out,
                   uint64_t capacity, MpHier h, MpKeys K) {
  MP_FOR(e, ncand) {
    if (cnt[e] == 0) continue;
    (void) mp_walk<true, SufT, true>(lcp, X, B, RM, RO, S, list[e], minlen, off[e], out, capacity,
                                     &h, &K);
  }
}

// one hierarchy level: dst[i] = min(src[64i .. 64i+63])
__global__ void __launch_bounds__(256) mp_hier_kernel(const uint32_t *src, uint64_t nsrc,
                                                      uint32_t *dst, uint64_t ndst) {
  MP_FOR(i, ndst) {
    const uint64_t b = i << 6, e = b + 64 < nsrc ? b + 64 : nsrc;
    uint32_t m = 0xffffffffu;
    for (uint64_t k = b; k < e; k++) m = src[k] < m ? src[k] : m;
    dst[i] = m;
  }
}

__global__ void __launch_bounds__(256) mp_iota_kernel(uint64_t *p, uint64_t n) {
  MP_FOR(i, n) p[i] = i;
}

// dst[i] = src[perm[i]] (words per element: 1 for keys, 3 for triples)
template <int W>
__global__ void __launch_bounds__(256) mp_gather_kernel(const uint64_t *src, const uint64_t *perm,
                                                        uint64_t n, uint64_t *dst) {
  MP_FOR(i, n) {
    const uint64_t s = perm[i];
#pragma unroll
    for (int w = 0; w < W; w++) dst[W * i + w] = src[W * s + w];
  }
}

// The order inside each event (equal k3, after a stable sort by k3 alone):
// (k2, k1), by an insertion sort of the event's permutation entries run by
// the thread of its first entry -- events hold a few pairs (a leaf's or two
// children's cartesian product), so this replaces the two 40- and 48-bit
// LSD sorts.  An event of more than MP_SEG_MAX pairs sets *big and the pass
// sorts by all three keys instead.
#define MP_SEG_MAX 64
__global__ void __launch_bounds__(256) mp_segfix_kernel(const uint64_t *ks, const uint64_t *k1,
                                                        const uint64_t *k2, uint64_t *pa, uint64_t n,
                                                        uint32_t *big) {
  MP_FOR(i, n) {
    if (i > 0 && ks[i] == ks[i - 1]) continue;   // not an event's first entry
    uint64_t e = i + 1;
    while (e < n && e - i <= MP_SEG_MAX && ks[e] == ks[i]) e++;
    if (e - i > MP_SEG_MAX) {
      atomicOr(big, 1u);
      continue;
    }
    for (uint64_t a = i + 1; a < e; a++) {       // stable: strict comparisons
      const uint64_t v = pa[a], v2 = k2[v], v1 = k1[v];
      uint64_t b = a;
      while (b > i) {
        const uint64_t u = pa[b - 1], u2 = k2[u];
        if (u2 < v2 || (u2 == v2 && k1[u] <= v1)) break;
        pa[b] = u;
        b--;
      }
      pa[b] = v;
    }
  }
}

// Small ordered passes (T <= mp_rank_max()): the stable LSD passes below
// are one rank count instead -- the final order is the composite key
// (k_{NK-1}, ..., k_1, emission index) in lexicographic order, so an
// entry's place is the number of entries before it under that order.  Each
// workgroup counts, for 256 entries i, the entries of one MP_RANK_J-slice j
// that precede i (the slice staged in LDS, the loop unrolled so its LDS
// reads overlap) and adds them into rank[i]; one scatter moves the triples.
// At C2 (3,365 pairs) that is 14 x 53 workgroups, against three rocprim
// sorts of ~5 kernels each.
#define MP_RANK_J 64
template <int NK>
__global__ void __launch_bounds__(256) mp_rank_kernel(const uint64_t *keys, uint64_t T,
                                                      uint32_t *rank) {
  __shared__ uint64_t kj[NK][MP_RANK_J];
  const uint64_t i = (uint64_t) blockIdx.x * 256 + threadIdx.x;
  const uint64_t j0 = (uint64_t) blockIdx.y * MP_RANK_J;
  const uint32_t jn = T - j0 < MP_RANK_J ? (uint32_t) (T - j0) : MP_RANK_J;
  if (threadIdx.x < MP_RANK_J)
#pragma unroll
    for (int k = 0; k < NK; k++)   // past T: all ones, after every entry
      kj[k][threadIdx.x] = threadIdx.x < jn ? keys[(uint64_t) k * T + j0 + threadIdx.x] : ~0ull;
  uint64_t ki[NK];
#pragma unroll
  for (int k = 0; k < NK; k++) ki[k] = i < T ? keys[(uint64_t) k * T + i] : 0;
  __syncthreads();
  if (i >= T) return;
  uint32_t cnt = 0;
#pragma unroll 16
  for (uint32_t t = 0; t < MP_RANK_J; t++) {
    // lt: entry j0+t sorts before i; eq: equal keys (then emission order)
    bool lt = false, eq = true;
#pragma unroll
    for (int k = NK - 1; k >= 0; k--) {
      const uint64_t a = kj[k][t];
      lt = lt || (eq && a < ki[k]);
      eq = eq && a == ki[k];
    }
    cnt += (t < jn && (lt || (eq && j0 + t < i))) ? 1u : 0u;
  }
  if (cnt) atomicAdd(&rank[i], cnt);
}

__global__ void __launch_bounds__(256) mp_rank_scatter_kernel(const uint64_t *tri,
                                                              const uint32_t *rank, uint64_t T,
                                                              uint64_t *out) {
  MP_FOR(i, T) {
    const uint64_t r = rank[i];
#pragma unroll
    for (int w = 0; w < 3; w++) out[3 * r + w] = tri[3 * i + w];
  }
}

// largest ordered pass sorted by ranks (GT_MP_RANK_MAX overrides; 0 = never)
static uint64_t mp_rank_max() {
  const char *e = getenv("GT_MP_RANK_MAX");
  return e ? strtoull(e, NULL, 0) : (uint64_t) 16384;
}

__global__ void mp_total_kernel(const uint32_t *cnt, const uint64_t *off, uint64_t n,
                                uint64_t *total) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *total = n == 0 ? 0 : off[n - 1] + cnt[n - 1];
}

// F4: (len, pos1, pos2) -> (len, seqnum1, relpos1, seqnum2, relpos2); seqnum
// = number of separators before the position (gt_encseq_seqnum,
// src/core/encseq.c:3815-3840), relpos = position - sequence start
// (gt_encseq_seqstartpos, :3842-3885).
__global__ void __launch_bounds__(256) seqpos_map_kernel(const uint64_t *sep, uint64_t nsep,
                                                         const uint64_t *pairs, uint64_t count,
                                                         uint64_t *out) {
  MP_FOR(k, count) {
    const uint64_t len = pairs[3 * k], p[2] = {pairs[3 * k + 1], pairs[3 * k + 2]};
    uint64_t *w = out + 5 * k;
    w[0] = len;
#pragma unroll
    for (int h = 0; h < 2; h++) {
      uint64_t lo = 0, hi = nsep;
      while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (sep[mid] < p[h]) lo = mid + 1; else hi = mid;
      }
      w[1 + 2 * h] = lo;
      w[2 + 2 * h] = p[h] - (lo == 0 ? 0 : sep[lo - 1] + 1);
    }
  }
}

// ------------------------------------------------------------ plan

struct GtMaxpairsPlan {
  GtMaxpairsDevInput in;
  unsigned int minlen;
  uint32_t *X;                   // N+1 exact LCP values
  uint32_t *RM, *RO;             // N+1: runs of equal BWT symbols (mp_walk)
  uint64_t nwg;                  // candidate workgroups (MP_WG_ROWS rows)
  uint64_t *wg_cand, *wg_cand_off;
  uint64_t ncand;                // candidate rows (fixed by the tables and minlen)
  uint64_t *list;                // ncand candidate rows, row order
  uint32_t *cnt;                 // ncand pair counts
  uint64_t *off;                 // ncand exclusive offsets
  uint64_t *total;               // 1
  uint16_t *masks;               // nwg * 256 candidate masks of 16 rows (pass A -> B)
  uint64_t *st_cnt;              // look-back status words (count workgroups)
  uint32_t epoch;                // count passes so far (the status words' tag)
  void *scan_tmp;
  size_t scan_tmp_bytes;
  bool counted;
  uint32_t *hier;                // levels >= 1 of the minimum hierarchy (ordered emission)
  MpHier h;
  uint32_t xmax;                 // largest exact LCP value
  SmaxStreamMarks marks;         // streams the plan's work ran on (waits and the
                                 // delete-time fence use their events only)
};

// per-element kernels are grid-stride loops (MP_FOR) over a capped grid: a
// dispatch holds fewer than 2^32 work-items, and N + 1 rows exceed that past
// 2^32 suffixes (12 Gbp: 1.2e10 rows)
static unsigned mp_blocks(uint64_t n) {
  const uint64_t b = (n + 255) / 256;
  return (unsigned) (b > MP_MAX_BLOCKS ? MP_MAX_BLOCKS : (b ? b : 1));
}

// the single-pass count's grid: 256 * R candidates per workgroup, R > 1
// only where one per workgroup would exceed the grid cap
static uint64_t mp_count_grid(uint64_t ncand, uint32_t *R) {
  const uint64_t per = (ncand + 256u * MP_MAX_BLOCKS - 1) / (256u * MP_MAX_BLOCKS);
  const uint64_t r = per ? per : 1;
  if (R) *R = (uint32_t) r;
  const uint64_t g = (ncand + 256u * r - 1) / (256u * r);
  return g ? g : 1;
}

// GT_MP_LOOKBACK=0: pass C, its scan and the total as three kernels always
static bool mp_lookback_on() {
  const char *e = getenv("GT_MP_LOOKBACK");
  return !(e && e[0] == '0');
}

extern "C" void gt_maxpairs_plan_delete(GtMaxpairsPlan *p) {
  if (p == NULL) return;
  (void) hipSetDevice(p->in.device);
  // the buffers return to the runtime's cache behind the plan's own work
  // (events recorded where it was enqueued): nothing here waits
  void *bufs[] = {p->X, p->RM, p->RO, p->wg_cand, p->wg_cand_off, p->list, p->cnt, p->off,
                  p->total, p->scan_tmp, p->hier, p->masks, p->st_cnt};
  SmaxFence *fence = smax_marks_fence(&p->marks);
  for (size_t i = 0; i < sizeof bufs / sizeof bufs[0]; i++) smax_dev_free_fenced(bufs[i], fence);
  smax_fence_release(fence);
  free(p);
}

extern "C" int gt_maxpairs_plan_create(GtMaxpairsPlan **planp, const GtMaxpairsDevInput *in,
                                       unsigned int minlen, char *errbuf, size_t errlen) {
  return gt_maxpairs_plan_create_stream(planp, in, minlen, NULL, errbuf, errlen);
}

extern "C" int gt_maxpairs_plan_create_stream(GtMaxpairsPlan **planp, const GtMaxpairsDevInput *in,
                                              unsigned int minlen, void *stream, char *errbuf,
                                              size_t errlen) {
  GtMaxpairsPlan *p = NULL;
  hipStream_t s = (hipStream_t) stream;
  uint32_t *derr = NULL, herr = 0;
  const uint64_t N = in != NULL ? in->nonspecials : 0;
  *planp = NULL;
  if (in == NULL || in->lcp_dev == NULL || in->bwt_dev == NULL || in->suf_dev == NULL) {
    mp_seterr(errbuf, errlen, "maxpairs needs device lcptab, bwttab and suftab");
    return -1;
  }
  if (in->suf_bytes != 4 && in->suf_bytes != 8) {
    mp_seterr(errbuf, errlen, "suftab entries must be 4 or 8 bytes (got %d)", in->suf_bytes);
    return -1;
  }
  if (in->numllv > 0 && in->llv_dev == NULL) {
    mp_seterr(errbuf, errlen, "missing llvtab");
    return -1;
  }
  if (minlen < 1) {
    mp_seterr(errbuf, errlen, "minimum length must be >= 1");
    return -1;
  }
  if ((uintptr_t) in->lcp_dev & 15) {
    mp_seterr(errbuf, errlen, "device lcptab must be 16-byte aligned");
    return -1;
  }
  p = (GtMaxpairsPlan *) calloc(1, sizeof *p);
  if (p == NULL) {
    mp_seterr(errbuf, errlen, "out of memory");
    return -1;
  }
  p->in = *in;
  p->minlen = minlen;
  smax_marks_init(&p->marks);
  // every buffer from the runtime's caching allocator, every step on s
  MPCHK(hipSetDevice(in->device));
  MPCHK(smax_dev_alloc((void **) &p->X, sizeof (uint32_t) * (N + 1)));
  p->nwg = (N + MP_WG_ROWS - 1) / MP_WG_ROWS;
  MPCHK(smax_dev_alloc((void **) &p->wg_cand, sizeof (uint64_t) * (p->nwg + 1)));
  MPCHK(smax_dev_alloc((void **) &p->wg_cand_off, sizeof (uint64_t) * (p->nwg + 1)));
  // whole groups of MP_WR_GROUP pass-A workgroups; the masks past the last
  // one stay zero
  MPCHK(smax_dev_alloc((void **) &p->masks, sizeof (uint16_t) * 256 * (p->nwg + MP_WR_GROUP)));
  MPCHK(hipMemsetAsync(p->masks, 0, sizeof (uint16_t) * 256 * (p->nwg + MP_WR_GROUP), s));
  MPCHK(smax_dev_alloc((void **) &p->total, sizeof (uint64_t)));
  MPCHK(hipMemsetAsync(p->total, 0, sizeof (uint64_t), s));
  MPCHK(smax_dev_alloc((void **) &derr, sizeof (uint32_t)));
  MPCHK(hipMemsetAsync(derr, 0, sizeof (uint32_t), s));
  hipLaunchKernelGGL(mp_expand_kernel, dim3(mp_blocks(N + 1)), dim3(256), 0, s, in->lcp_dev, N,
                     p->X);
  MPCHK(hipGetLastError());
  if (in->numllv > 0) {
    hipLaunchKernelGGL(mp_llv_kernel, dim3(mp_blocks(in->numllv)), dim3(256), 0, s, in->llv_dev,
                       in->numllv, in->lcp_dev, N, p->X, derr);
    MPCHK(hipGetLastError());
  }
  hipLaunchKernelGGL(mp_llv_check_kernel, dim3(mp_blocks(N)), dim3(256), 0, s, p->X, N, derr);
  MPCHK(hipGetLastError());
  // runs of equal BWT symbols: start offsets and running LCP minima
  {
    uint64_t *hv = NULL, *rs = NULL;
    void *tmp = NULL;
    size_t b1 = 0, b2 = 0;
    hipError_t e = smax_dev_alloc((void **) &p->RM, sizeof (uint32_t) * (N + 1));
    if (e == hipSuccess) e = smax_dev_alloc((void **) &p->RO, sizeof (uint32_t) * (N + 1));
    if (e == hipSuccess) e = smax_dev_alloc((void **) &hv, sizeof (uint64_t) * (N + 1));
    if (e == hipSuccess) e = smax_dev_alloc((void **) &rs, sizeof (uint64_t) * (N + 1));
    if (e == hipSuccess) {
      hipLaunchKernelGGL(mp_run_heads_kernel, dim3(mp_blocks(N + 1)), dim3(256), 0, s,
                         in->bwt_dev, N, hv);
      e = rocprim::inclusive_scan(nullptr, b1, hv, rs, (size_t) (N + 1), rocprim::maximum<uint64_t>(),
                                  s);
    }
    if (e == hipSuccess)
      e = rocprim::inclusive_scan_by_key(nullptr, b2, rs, p->X, p->RM, (size_t) (N + 1),
                                         rocprim::minimum<uint32_t>(), rocprim::equal_to<uint64_t>(), s);
    if (e == hipSuccess) e = smax_dev_alloc(&tmp, b1 > b2 ? b1 : b2);
    if (e == hipSuccess)
      e = rocprim::inclusive_scan(tmp, b1, hv, rs, (size_t) (N + 1), rocprim::maximum<uint64_t>(), s);
    if (e == hipSuccess)
      e = rocprim::inclusive_scan_by_key(tmp, b2, rs, p->X, p->RM, (size_t) (N + 1),
                                         rocprim::minimum<uint32_t>(), rocprim::equal_to<uint64_t>(), s);
    if (e == hipSuccess) {
      hipLaunchKernelGGL(mp_run_off_kernel, dim3(mp_blocks(N + 1)), dim3(256), 0, s, rs, N, p->RO);
      e = hipGetLastError();
    }
    {
      // the temporaries go back behind the work on s, nothing waits here
      SmaxStreamMarks m;
      smax_marks_init(&m);
      smax_marks_record(&m, s);
      SmaxFence *f = smax_marks_fence(&m);
      smax_dev_free_fenced(hv, f);
      smax_dev_free_fenced(rs, f);
      smax_dev_free_fenced(tmp, f);
      smax_fence_release(f);
    }
    MPCHK(e);
  }
  // candidate rows: their number sizes the per-candidate buffers (the tables
  // are immutable for the plan's life; every count pass rebuilds the list)
  if (N > 0) {
    size_t b1 = 0;
    MPCHK(rocprim::exclusive_scan(nullptr, b1, p->wg_cand, p->wg_cand_off, (uint64_t) 0,
                                  (size_t) p->nwg, rocprim::plus<uint64_t>(), s));
    p->scan_tmp_bytes = b1;
    hipLaunchKernelGGL(mp_cand_count_kernel, dim3((unsigned) p->nwg), dim3(256), 0, s, in->lcp_dev,
                       N, minlen < 255u ? minlen : 255u, p->wg_cand, p->masks);
    MPCHK(hipGetLastError());
    MPCHK(smax_dev_alloc(&p->scan_tmp, b1 ? b1 : 16));
    MPCHK(rocprim::exclusive_scan(p->scan_tmp, b1, p->wg_cand, p->wg_cand_off, (uint64_t) 0,
                                  (size_t) p->nwg, rocprim::plus<uint64_t>(), s));
    uint64_t last[2];
    MPCHK(hipMemcpyAsync(&last[0], p->wg_cand + p->nwg - 1, sizeof (uint64_t), hipMemcpyDeviceToHost, s));
    MPCHK(hipMemcpyAsync(&last[1], p->wg_cand_off + p->nwg - 1, sizeof (uint64_t), hipMemcpyDeviceToHost,
                         s));
    MPCHK(hipStreamSynchronize(s));    // the candidate count sizes the lists
    p->ncand = last[0] + last[1];
  }
  MPCHK(smax_dev_alloc((void **) &p->list, sizeof (uint64_t) * (p->ncand + 1)));
  MPCHK(smax_dev_alloc((void **) &p->cnt, sizeof (uint32_t) * (p->ncand + 1)));
  MPCHK(smax_dev_alloc((void **) &p->off, sizeof (uint64_t) * (p->ncand + 1)));
  MPCHK(smax_dev_alloc((void **) &p->st_cnt, sizeof (uint64_t) * (MP_LB_MAX_WG + 1)));
  MPCHK(hipMemsetAsync(p->st_cnt, 0, sizeof (uint64_t) * (MP_LB_MAX_WG + 1), s));
  if (p->ncand > 0) {
    size_t b2 = 0;
    MPCHK(rocprim::exclusive_scan(nullptr, b2, p->cnt, p->off, (uint64_t) 0, (size_t) p->ncand,
                                  rocprim::plus<uint64_t>(), s));
    if (b2 > p->scan_tmp_bytes) {
      MPCHK(hipStreamSynchronize(s));   // the candidate scan is done with it
      smax_dev_free(p->scan_tmp);
      p->scan_tmp = NULL;
      MPCHK(smax_dev_alloc(&p->scan_tmp, b2));
      p->scan_tmp_bytes = b2;
    }
  }
  if (p->scan_tmp == NULL) MPCHK(smax_dev_alloc(&p->scan_tmp, 16));
  MPCHK(hipMemcpyAsync(&herr, derr, sizeof herr, hipMemcpyDeviceToHost, s));
  MPCHK(hipStreamSynchronize(s));
  if (herr & 1u) { mp_seterr(errbuf, errlen, "lcp value >= 2^32 in .llv"); goto fail; }
  if (herr & 2u) { mp_seterr(errbuf, errlen, "inconsistent .llv entry (lcp byte is not 255)"); goto fail; }
  if (herr & 4u) { mp_seterr(errbuf, errlen, "inconsistent index: a .lcp byte 255 without its .llv entry"); goto fail; }
  smax_dev_free(derr);
  smax_marks_record(&p->marks, s);
  *planp = p;
  return 0;
fail:
  (void) hipStreamSynchronize(s);
  smax_dev_free(derr);
  smax_marks_record(&p->marks, s);
  gt_maxpairs_plan_delete(p);
  return -1;
}

extern "C" int gt_maxpairs_plan_count(GtMaxpairsPlan *p, void *stream) {
  char *errbuf = NULL;
  size_t errlen = 0;
  hipStream_t s = (hipStream_t) stream;
  const uint64_t N = p->in.nonspecials, nc = p->ncand;
  const uint32_t mf = p->minlen < 255u ? p->minlen : 255u;
  MPCHK(hipSetDevice(p->in.device));
  MPCHK(smax_marks_wait(&p->marks, s));   // the plan's earlier work on other streams
  if (nc == 0) {
    MPCHK(hipMemsetAsync(p->total, 0, sizeof (uint64_t), s));
  } else {
    size_t bytes = p->scan_tmp_bytes;
    hipLaunchKernelGGL(mp_cand_count_kernel, dim3((unsigned) p->nwg), dim3(256), 0, s,
                       p->in.lcp_dev, N, mf, p->wg_cand, p->masks);
    MPCHK(hipGetLastError());
    // (one 1024-thread workgroup scanning the 24,414 counts of C2 took 34.8 us)
    MPCHK(rocprim::exclusive_scan(p->scan_tmp, bytes, p->wg_cand, p->wg_cand_off, (uint64_t) 0,
                                  (size_t) p->nwg, rocprim::plus<uint64_t>(), s));
    hipLaunchKernelGGL(mp_cand_write_kernel, dim3((unsigned) ((p->nwg + MP_WR_GROUP - 1) / MP_WR_GROUP)),
                       dim3(256), 0, s, p->masks, p->wg_cand_off, p->list);
    MPCHK(hipGetLastError());
    uint32_t R = 1;
    const uint64_t g = mp_count_grid(nc, &R);
    if (g <= MP_LB_MAX_WG && mp_lookback_on()) {
      p->epoch = p->epoch % 0xffffu + 1u;   // tags 1 .. 65535: never the last pass's
      hipLaunchKernelGGL((mp_count_scan_kernel<uint32_t>), dim3((unsigned) g), dim3(256), 0, s,
                         p->in.lcp_dev, p->X, p->in.bwt_dev, p->RM, p->RO, p->list, nc, p->minlen, R,
                         p->st_cnt, (uint64_t) p->epoch, p->cnt, p->off, p->total);
      MPCHK(hipGetLastError());
    } else {
      hipLaunchKernelGGL((mp_count_kernel<uint32_t>), dim3(mp_blocks(nc)), dim3(256), 0, s,
                         p->in.lcp_dev, p->X, p->in.bwt_dev, p->RM, p->RO, p->list, nc, p->minlen,
                         p->cnt);
      MPCHK(hipGetLastError());
      bytes = p->scan_tmp_bytes;
      MPCHK(rocprim::exclusive_scan(p->scan_tmp, bytes, p->cnt, p->off, (uint64_t) 0, (size_t) nc,
                                    rocprim::plus<uint64_t>(), s));
      hipLaunchKernelGGL(mp_total_kernel, dim3(1), dim3(64), 0, s, p->cnt, p->off, nc, p->total);
      MPCHK(hipGetLastError());
    }
  }
  smax_marks_record(&p->marks, s);
  p->counted = true;
  return 0;
fail:
  smax_marks_record(&p->marks, s);
  return -1;
}

extern "C" int gt_maxpairs_plan_total(GtMaxpairsPlan *p, uint64_t *total) {
  char *errbuf = NULL;
  size_t errlen = 0;
  MPCHK(hipSetDevice(p->in.device));
  MPCHK(smax_marks_sync(&p->marks));     // the plan's own work, not the device
  MPCHK(hipMemcpy(total, p->total, sizeof (uint64_t), hipMemcpyDeviceToHost));
  return 0;
fail:
  return -1;
}

extern "C" uint64_t gt_maxpairs_plan_candidates(const GtMaxpairsPlan *p) { return p->ncand; }

extern "C" int gt_maxpairs_plan_emit(GtMaxpairsPlan *p, uint64_t *out_dev, uint64_t capacity,
                                     void *stream) {
  char *errbuf = NULL;
  size_t errlen = 0;
  hipStream_t s = (hipStream_t) stream;
  const uint64_t nc = p->ncand;
  if (!p->counted) return -1;
  MPCHK(hipSetDevice(p->in.device));
  if (nc == 0 || capacity == 0) return 0;
  MPCHK(smax_marks_wait(&p->marks, s));
  if (p->in.suf_bytes == 8)
    hipLaunchKernelGGL((mp_emit_kernel<uint64_t>), dim3(mp_blocks(nc)), dim3(256), 0, s,
                       p->in.lcp_dev, p->X, p->in.bwt_dev, p->RM, p->RO, p->in.suf_dev, p->list, nc,
                       p->minlen, p->cnt, p->off, out_dev, capacity);
  else
    hipLaunchKernelGGL((mp_emit_kernel<uint32_t>), dim3(mp_blocks(nc)), dim3(256), 0, s,
                       p->in.lcp_dev, p->X, p->in.bwt_dev, p->RM, p->RO, p->in.suf_dev, p->list, nc,
                       p->minlen, p->cnt, p->off, out_dev, capacity);
  smax_marks_record(&p->marks, s);
  MPCHK(hipGetLastError());
  return 0;
fail:
  return -1;
}

static int mp_bits(uint64_t v) { return v == 0 ? 1 : 64 - __builtin_clzll(v); }

// an ordered pass's temporaries back to the cache behind its work on s;
// the plan's mark on s stands behind the pass too
static hipError_t mp_free_behind(GtMaxpairsPlan *p, hipStream_t s, void *a, void *b, void *c, void *d,
                                 void *e, void *f) {
  SmaxStreamMarks m;
  smax_marks_init(&m);
  smax_marks_record(&m, s);
  SmaxFence *fence = smax_marks_fence(&m);
  void *bufs[] = {a, b, c, d, e, f};
  for (size_t i = 0; i < sizeof bufs / sizeof bufs[0]; i++) smax_dev_free_fenced(bufs[i], fence);
  smax_fence_release(fence);
  smax_marks_record(&p->marks, s);
  // the pass is complete when the call returns, as documented (its caller's
  // stream only, never the device)
  return hipStreamSynchronize(s);
}

// the minimum hierarchy and the largest LCP value, once per plan
static int mp_build_hier(GtMaxpairsPlan *p, hipStream_t s, char *errbuf, size_t errlen) {
  const uint64_t N = p->in.nonspecials;
  uint64_t n[MP_HMAX], off[MP_HMAX], tot = 0;
  int L = 1;
  uint32_t *dmax = NULL;
  void *tmp = NULL;
  size_t tb = 0;
  if (p->hier != NULL || p->h.levels > 0) return 0;
  n[0] = N + 1;
  while (n[L - 1] > 64) {
    if (L >= MP_HMAX) { mp_seterr(errbuf, errlen, "minimum hierarchy too deep"); return -1; }
    n[L] = (n[L - 1] + 63) / 64;
    off[L] = tot;
    tot += n[L];
    L++;
  }
  if (tot > 0) MPCHK(smax_dev_alloc((void **) &p->hier, sizeof (uint32_t) * tot));
  p->h.lv[0] = p->X;
  p->h.n[0] = n[0];
  for (int l = 1; l < L; l++) {
    p->h.lv[l] = p->hier + off[l];
    p->h.n[l] = n[l];
    hipLaunchKernelGGL(mp_hier_kernel, dim3(mp_blocks(n[l])), dim3(256), 0, s, p->h.lv[l - 1],
                       n[l - 1], (uint32_t *) p->h.lv[l], n[l]);
    MPCHK(hipGetLastError());
  }
  p->h.levels = L;
  MPCHK(smax_dev_alloc((void **) &dmax, sizeof (uint32_t)));
  MPCHK(rocprim::reduce(nullptr, tb, p->X, dmax, 0u, (size_t) (N + 1), rocprim::maximum<uint32_t>(), s));
  MPCHK(smax_dev_alloc(&tmp, tb ? tb : 16));
  MPCHK(rocprim::reduce(tmp, tb, p->X, dmax, 0u, (size_t) (N + 1), rocprim::maximum<uint32_t>(), s));
  MPCHK(hipMemcpyAsync(&p->xmax, dmax, sizeof (uint32_t), hipMemcpyDeviceToHost, s));
  MPCHK(hipStreamSynchronize(s));       // once per plan: the key widths need xmax
  smax_dev_free(dmax);
  smax_dev_free(tmp);
  return 0;
fail:
  (void) hipStreamSynchronize(s);
  smax_dev_free(dmax);
  smax_dev_free(tmp);
  return -1;
}

extern "C" int gt_maxpairs_plan_emit_ordered(GtMaxpairsPlan *p, uint64_t *out_dev, uint64_t capacity,
                                             void *stream) {
  char *errbuf = NULL;
  size_t errlen = 0;
  hipStream_t s = (hipStream_t) stream;
  const uint64_t nc = p->ncand;
  uint64_t T = 0;
  uint64_t *tri = NULL, *keys = NULL, *ktmp = NULL, *pa = NULL, *pb = NULL, *ks = NULL;
  uint32_t *big = NULL;
  void *st = NULL;
  size_t sb = 0;
  MpKeys K;
  bool by_rank = false;
  if (!p->counted) return -1;
  MPCHK(hipSetDevice(p->in.device));
  MPCHK(smax_marks_wait(&p->marks, s));
  MPCHK(hipMemcpyAsync(&T, p->total, sizeof (uint64_t), hipMemcpyDeviceToHost, s));
  MPCHK(hipStreamSynchronize(s));        // the pair count sizes the pass
  if (T == 0) return 0;
  if (capacity < T) return -1;
  if (mp_build_hier(p, s, errbuf, errlen) != 0) return -1;
  K.rowbits = mp_bits(p->in.nonspecials);
  K.lbits = mp_bits(p->xmax);
  K.split = K.rowbits + K.lbits > 64;
  if (K.rowbits > 48) return -1;
  // per-call temporaries from the runtime's caching allocator: repeated
  // passes reuse them (a hipMalloc/hipFree of each per pass was most of a
  // small table's ordered pass)
  MPCHK(smax_dev_alloc((void **) &tri, sizeof (uint64_t) * 3 * T));
  MPCHK(smax_dev_alloc((void **) &keys, sizeof (uint64_t) * (K.split ? 4 : 3) * T));
  MPCHK(smax_dev_alloc((void **) &ktmp, sizeof (uint64_t) * T));
  K.k1 = keys;
  K.k2 = keys + T;
  K.k3 = keys + 2 * T;
  K.k4 = K.split ? keys + 3 * T : nullptr;
  // small passes are ordered by rank counts (mp_rank_kernel) in ktmp
  by_rank = T <= mp_rank_max() && (T + MP_RANK_J - 1) / MP_RANK_J <= 65535;
  K.rank0 = by_rank ? (uint32_t *) ktmp : nullptr;
  if (p->in.suf_bytes == 8)
    hipLaunchKernelGGL((mp_emit_ord_kernel<uint64_t>), dim3(mp_blocks(nc)), dim3(256), 0, s,
                       p->in.lcp_dev, p->X, p->in.bwt_dev, p->RM, p->RO, p->in.suf_dev, p->list, nc,
                       p->minlen, p->cnt, p->off, tri, T, p->h, K);
  else
    hipLaunchKernelGGL((mp_emit_ord_kernel<uint32_t>), dim3(mp_blocks(nc)), dim3(256), 0, s,
                       p->in.lcp_dev, p->X, p->in.bwt_dev, p->RM, p->RO, p->in.suf_dev, p->list, nc,
                       p->minlen, p->cnt, p->off, tri, T, p->h, K);
  MPCHK(hipGetLastError());
  if (by_rank) {
    uint32_t *rank = K.rank0;   // T u64 hold T u32 ranks, zeroed by the emission
    const dim3 grid((unsigned) ((T + 255) / 256), (unsigned) ((T + MP_RANK_J - 1) / MP_RANK_J));
    if (K.split)
      hipLaunchKernelGGL(mp_rank_kernel<4>, grid, dim3(256), 0, s, keys, T, rank);
    else
      hipLaunchKernelGGL(mp_rank_kernel<3>, grid, dim3(256), 0, s, keys, T, rank);
    MPCHK(hipGetLastError());
    hipLaunchKernelGGL(mp_rank_scatter_kernel, dim3(mp_blocks(T)), dim3(256), 0, s, tri, rank, T,
                       out_dev);
    MPCHK(hipGetLastError());
    MPCHK(mp_free_behind(p, s, tri, keys, ktmp, NULL, NULL, NULL));
    return 0;
  }
  MPCHK(smax_dev_alloc((void **) &pa, sizeof (uint64_t) * T));
  MPCHK(smax_dev_alloc((void **) &pb, sizeof (uint64_t) * T));
  hipLaunchKernelGGL(mp_iota_kernel, dim3(mp_blocks(T)), dim3(256), 0, s, pa, T);
  MPCHK(hipGetLastError());
  MPCHK(rocprim::radix_sort_pairs(nullptr, sb, ktmp, ktmp, pa, pb, (size_t) T, 0, 64, s));
  MPCHK(smax_dev_alloc(&st, sb ? sb : 16));
  if (!K.split) {
    // one stable sort by the event (k3), then each event's few pairs put in
    // (k2, k1) order in place (mp_segfix_kernel): 5 radix passes instead of
    // 16 at 3 Gbp
    MPCHK(smax_dev_alloc((void **) &ks, sizeof (uint64_t) * T));
    MPCHK(smax_dev_alloc((void **) &big, sizeof (uint32_t)));
    MPCHK(hipMemsetAsync(big, 0, sizeof (uint32_t), s));
    MPCHK(hipMemcpyAsync(ktmp, K.k3, sizeof (uint64_t) * T, hipMemcpyDeviceToDevice, s));
    size_t b = sb;
    MPCHK(rocprim::radix_sort_pairs(st, b, ktmp, ks, pa, pb, (size_t) T, 0, K.rowbits + K.lbits, s));
    uint64_t *t = pa; pa = pb; pb = t;
    hipLaunchKernelGGL(mp_segfix_kernel, dim3(mp_blocks(T)), dim3(256), 0, s, ks, K.k1, K.k2, pa, T, big);
    MPCHK(hipGetLastError());
    uint32_t hbig = 0;
    MPCHK(hipMemcpyAsync(&hbig, big, sizeof hbig, hipMemcpyDeviceToHost, s));
    MPCHK(hipStreamSynchronize(s));      // an event past MP_SEG_MAX pairs: all three keys
    if (hbig == 0) {
      hipLaunchKernelGGL((mp_gather_kernel<3>), dim3(mp_blocks(T)), dim3(256), 0, s, tri, pa, T,
                         out_dev);
      MPCHK(hipGetLastError());
      smax_dev_free(ks);                 // the sync above passed their users
      smax_dev_free(big);
      ks = NULL;
      big = NULL;
      MPCHK(mp_free_behind(p, s, tri, keys, ktmp, pa, pb, st));
      return 0;
    }
    smax_dev_free(ks);
    smax_dev_free(big);
    ks = NULL;
    big = NULL;
    hipLaunchKernelGGL(mp_iota_kernel, dim3(mp_blocks(T)), dim3(256), 0, s, pa, T);
    MPCHK(hipGetLastError());
  }
  {
    // stable LSD passes: r2, then (classes, r1), then the event [depth, then t]
    const int nk = K.split ? 4 : 3;
    const int bits[4] = {K.rowbits + 8, K.rowbits + 16, K.split ? K.lbits : K.rowbits + K.lbits,
                         K.rowbits};
    for (int k = 0; k < nk; k++) {
      const uint64_t *src = keys + (uint64_t) k * T;
      if (k == 0) {
        MPCHK(hipMemcpyAsync(ktmp, src, sizeof (uint64_t) * T, hipMemcpyDeviceToDevice, s));
      } else {
        hipLaunchKernelGGL((mp_gather_kernel<1>), dim3(mp_blocks(T)), dim3(256), 0, s, src, pa, T,
                           ktmp);
        MPCHK(hipGetLastError());
      }
      // sorted keys land in k1's slot (no longer needed after the first pass)
      size_t b = sb;
      MPCHK(rocprim::radix_sort_pairs(st, b, ktmp, keys, pa, pb, (size_t) T, 0, bits[k], s));
      uint64_t *t = pa; pa = pb; pb = t;
    }
  }
  hipLaunchKernelGGL((mp_gather_kernel<3>), dim3(mp_blocks(T)), dim3(256), 0, s, tri, pa, T,
                     out_dev);
  MPCHK(hipGetLastError());
  MPCHK(mp_free_behind(p, s, tri, keys, ktmp, pa, pb, st));
  return 0;
fail:
  {
    (void) hipStreamSynchronize(s);
    void *bufs[] = {tri, keys, ktmp, pa, pb, st, ks, big};
    for (size_t i = 0; i < sizeof bufs / sizeof bufs[0]; i++) smax_dev_free(bufs[i]);
  }
  return -1;
}

extern "C" int gt_seqpos_map_dev(const uint64_t *sep_dev, uint64_t nsep, const uint64_t *pairs_dev,
                                 uint64_t count, uint64_t *out_dev, int device, void *stream) {
  char *errbuf = NULL;
  size_t errlen = 0;
  MPCHK(hipSetDevice(device));
  if (count == 0) return 0;
  hipLaunchKernelGGL(seqpos_map_kernel, dim3(mp_blocks(count)), dim3(256), 0,
                     (hipStream_t) stream, sep_dev, nsep, pairs_dev, count, out_dev);
  MPCHK(hipGetLastError());
  return 0;
fail:
  return -1;
}

// ------------------------------------------------------------ host boundary

// Host tables -> HBM, count, emit in the reference's order, D2H.  *pairs is
// malloc'd (3 * *count).  With lines != NULL the pairs stay in HBM and are
// formatted there as gt repfind lines (F4) handed to lines(ldata, ...) in
// chunks; sep[0..nsep) are the separator positions.
static int mp_host_run(const GtSmaxInput *in, unsigned int minlen, uint64_t **pairs,
                       uint64_t *count, char *errbuf, size_t errlen,
                       GtRepfindTextFunc lines = nullptr, void *ldata = nullptr,
                       const uint64_t *sep = nullptr, uint64_t nsep = 0) {
  uint64_t *dsep = NULL;
  uint8_t *lcp = NULL, *bwt = NULL;
  GtSmaxLlv *llv = NULL;
  void *suf = NULL;
  uint64_t *out = NULL, total = 0;
  GtMaxpairsPlan *plan = NULL;
  GtMaxpairsDevInput din;
  uint64_t N;
  int dev = 0;
  SmaxDeviceGuard keep;
  *pairs = NULL;
  *count = 0;
  if (in == NULL || in->lcptab == NULL || in->bwttab == NULL || in->suftab == NULL) {
    mp_seterr(errbuf, errlen, "maxpairs needs lcptab, bwttab and suftab");
    return -1;
  }
  if (in->suftab_bytes != 4 && in->suftab_bytes != 8) {
    mp_seterr(errbuf, errlen, "suftab entries must be 4 or 8 bytes (got %d)", in->suftab_bytes);
    return -1;
  }
  if (in->numllv > 0 && in->llvtab == NULL) {
    mp_seterr(errbuf, errlen, "missing llvtab");
    return -1;
  }
  if (in->nonspecials > in->totallength) {
    mp_seterr(errbuf, errlen, "nonspecials (%lu) exceeds totallength (%lu)",
              (unsigned long) in->nonspecials, (unsigned long) in->totallength);
    return -1;
  }
  N = in->nonspecials;
  // the caller's current device (restored on return); tables from the
  // runtime's caching allocator, staged through its pinned ring
  MPCHK(hipGetDevice(&dev));
  MPCHK(smax_dev_alloc((void **) &lcp, N + 1));
  MPCHK(smax_dev_alloc((void **) &bwt, N + 1));
  MPCHK(smax_dev_alloc(&suf, (size_t) in->suftab_bytes * (N + 1)));
  MPCHK(smax_stage_upload(lcp, in->lcptab, N + 1));
  MPCHK(smax_stage_upload(bwt, in->bwttab, N + 1));
  MPCHK(smax_stage_upload(suf, in->suftab, (size_t) in->suftab_bytes * (N + 1)));
  if (in->numllv > 0) {
    MPCHK(smax_dev_alloc((void **) &llv, sizeof (GtSmaxLlv) * in->numllv));
    MPCHK(smax_stage_upload(llv, in->llvtab, sizeof (GtSmaxLlv) * in->numllv));
  }
  din.lcp_dev = lcp;
  din.bwt_dev = bwt;
  din.llv_dev = llv;
  din.numllv = in->numllv;
  din.suf_dev = suf;
  din.suf_bytes = in->suftab_bytes;
  din.nonspecials = N;
  din.device = dev;
  if (gt_maxpairs_plan_create(&plan, &din, minlen, errbuf, errlen) != 0) goto fail_quiet;
  if (gt_maxpairs_plan_count(plan, NULL) != 0 || gt_maxpairs_plan_total(plan, &total) != 0) {
    mp_seterr(errbuf, errlen, "maxpairs count pass failed");
    goto fail_quiet;
  }
  if (total > 0) {
    if (lines == nullptr) *pairs = (uint64_t *) malloc(sizeof (uint64_t) * 3 * total);
    if (lines == nullptr && *pairs == NULL) {
      mp_seterr(errbuf, errlen, "out of memory (%lu pairs)", (unsigned long) total);
      goto fail_quiet;
    }
    MPCHK(smax_dev_alloc((void **) &out, sizeof (uint64_t) * 3 * total));
    if (gt_maxpairs_plan_emit_ordered(plan, out, total, NULL) != 0) {
      mp_seterr(errbuf, errlen, "maxpairs emission pass failed");
      goto fail_quiet;
    }
    if (lines != nullptr) {
      MPCHK(smax_dev_alloc((void **) &dsep, sizeof (uint64_t) * (nsep ? nsep : 1)));
      if (nsep) MPCHK(smax_stage_upload(dsep, sep, sizeof (uint64_t) * nsep));
      if (gt_repfind_pairs_lines_dev(out, total, dsep, nsep, dev, lines, ldata, errbuf, errlen) != 0)
        goto fail_quiet;
    } else {
      MPCHK(smax_stage_download(*pairs, out, sizeof (uint64_t) * 3 * total));
    }
  }
  *count = total;
  gt_maxpairs_plan_delete(plan);
  {
    void *bufs[] = {lcp, bwt, suf, llv, out, dsep};
    (void) hipStreamSynchronize(nullptr);   // the plan's kernels (null stream) are done
    for (size_t i = 0; i < sizeof bufs / sizeof bufs[0]; i++) smax_dev_free(bufs[i]);
  }
  return 0;
fail:
fail_quiet:
  gt_maxpairs_plan_delete(plan);
  {
    void *bufs[] = {lcp, bwt, suf, llv, out, dsep};
    (void) hipStreamSynchronize(nullptr);   // the plan's kernels (null stream) are done
    for (size_t i = 0; i < sizeof bufs / sizeof bufs[0]; i++) smax_dev_free(bufs[i]);
  }
  free(*pairs);
  *pairs = NULL;
  return -1;
}

extern "C" int gt_maxpairs_hip_enumerate_to_buffer(const GtSmaxInput *in, unsigned int minlen,
                                                   uint64_t **len_pos1_pos2, uint64_t *count,
                                                   char *errbuf, size_t errlen) {
  return mp_host_run(in, minlen, len_pos1_pos2, count, errbuf, errlen);
}

extern "C" int gt_maxpairs_hip_enumerate(const GtSmaxInput *in, unsigned int minlen,
                                         GtMaxpairsFunc cb, void *data, char *errbuf,
                                         size_t errlen) {
  uint64_t *pairs = NULL, count = 0;
  if (mp_host_run(in, minlen, &pairs, &count, errbuf, errlen) != 0) return -1;
  for (uint64_t k = 0; k < count; k++) {
    if (cb(data, pairs[3 * k], pairs[3 * k + 1], pairs[3 * k + 2]) != 0) {
      mp_seterr(errbuf, errlen, "maxpairs callback returned non-zero");
      free(pairs);
      return -1;
    }
  }
  free(pairs);
  return 0;
}

extern "C" int gt_repfind_maxpairs_lines(const GtSmaxInput *in, unsigned int minlen,
                                         const uint64_t *sep, uint64_t nsep, GtRepfindTextFunc cb,
                                         void *data, char *errbuf, size_t errlen) {
  uint64_t *pairs = NULL, count = 0;
  if (cb == NULL) {
    mp_seterr(errbuf, errlen, "no output function");
    return -1;
  }
  return mp_host_run(in, minlen, &pairs, &count, errbuf, errlen, cb, data, sep, nsep);
}
