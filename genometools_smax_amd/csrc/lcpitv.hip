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
// One thread per row; the intervals are compacted, radix-sorted into pop
// order (rb ascending, depth descending) and the host replays the visitor
// events in the reference's exact order from them (the replay is a merge,
// no stack: which callback comes when is decided by LCP[idx], LCP[idx+1]
// and whether a father shares its child's lb).
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gt_lcpitv_hip.h"

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

__global__ void __launch_bounds__(256) li_expand_kernel(const uint8_t *lcp, uint64_t N,
                                                        uint32_t *X) {
  const uint64_t k = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (k > N) return;
  X[k] = (k == 0 || k == N) ? 0u : (uint32_t) lcp[k];
}

__global__ void __launch_bounds__(256) li_llv_kernel(const GtSmaxLlv *llv, uint64_t numllv,
                                                     const uint8_t *lcp, uint64_t N, uint32_t *X,
                                                     uint32_t *err) {
  const uint64_t e = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (e >= numllv) return;
  const uint64_t pos = llv[e].position, v = llv[e].value;
  if (pos < 1 || pos >= N) return;
  if (v > 0xfffffffeull) atomicOr(err, 1u);
  if (lcp[pos] != 255) atomicOr(err, 2u);
  X[pos] = (uint32_t) v;
}

__global__ void __launch_bounds__(256) li_min64_kernel(const uint32_t *in, uint64_t n_in,
                                                       uint32_t *out, uint64_t n_out) {
  const uint64_t g = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (g >= n_out) return;
  uint32_t m = 0xffffffffu;
  const uint64_t b = g * 64, e = b + 64 < n_in ? b + 64 : n_in;
  for (uint64_t i = b; i < e; i++) m = in[i] < m ? in[i] : m;
  out[g] = m;
}

__device__ __forceinline__ bool li_ok(uint32_t x, uint32_t v, bool strict) {
  return strict ? x < v : x <= v;
}

// nearest p < k with X[p] < v (strict) / <= v; X[0] == 0 guarantees one
// for v > 0 (strict) and any v (<=)
__device__ static uint64_t li_prev(const LiLevels &L, uint64_t k, uint32_t v, bool strict) {
  uint64_t i = k, p = 0;
  int lev = 0;
  for (;;) {
    const uint64_t start = (i >> 6) << 6;
    bool found = false;
    for (uint64_t q = i; q > start;) {
      q--;
      if (li_ok(L.lv[lev][q], v, strict)) { p = q; found = true; break; }
    }
    if (found) break;
    if (lev + 1 >= L.nlev || i < 64) return 0;   // only row 0 is left
    i >>= 6;
    lev++;
  }
  while (lev > 0) {                // last child of p whose subtree qualifies
    lev--;
    const uint64_t b = p << 6;
    const uint64_t e = b + 64 < L.n[lev] ? b + 64 : L.n[lev];
    for (uint64_t c = e; c > b;) {
      c--;
      if (li_ok(L.lv[lev][c], v, strict)) { p = c; break; }
    }
  }
  return p;
}

// nearest q > k with X[q] < v (X[N] == 0 guarantees one for v > 0)
__device__ static uint64_t li_next(const LiLevels &L, uint64_t k, uint32_t v) {
  uint64_t i = k, p = 0;
  int lev = 0;
  for (;;) {
    const uint64_t end = ((i >> 6) + 1) << 6;
    const uint64_t e = end < L.n[lev] ? end : L.n[lev];
    bool found = false;
    for (uint64_t q = i + 1; q < e; q++)
      if (L.lv[lev][q] < v) { p = q; found = true; break; }
    if (found) break;
    if (lev + 1 >= L.nlev) return L.n[0] - 1;    // row N
    i >>= 6;
    lev++;
  }
  while (lev > 0) {                // first child of p whose subtree qualifies
    lev--;
    const uint64_t b = p << 6;
    const uint64_t e = b + 64 < L.n[lev] ? b + 64 : L.n[lev];
    for (uint64_t c = b; c < e; c++)
      if (L.lv[lev][c] < v) { p = c; break; }
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

__global__ void __launch_bounds__(256) li_count_kernel(LiLevels L, uint64_t N, uint32_t *wg_cnt) {
  const uint64_t k = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  uint64_t lb;
  uint32_t tot;
  (void) li_block_excl(li_leftmost(L, k, N, &lb) ? 1u : 0u, &tot);
  if (threadIdx.x == 0) wg_cnt[blockIdx.x] = tot;
}

// records (lcp, lb, rb, fatherlcp, fatherlb) in row order of their
// leftmost l-index, and the pop-order sort key rb << 32 | ~lcp
__global__ void __launch_bounds__(256) li_write_kernel(LiLevels L, uint64_t N,
                                                       const uint64_t *wg_off, uint64_t *rec,
                                                       uint64_t *key, uint32_t *idx) {
  const uint64_t k = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  uint64_t lb = 0;
  const bool open = li_leftmost(L, k, N, &lb);
  uint32_t tot;
  const uint64_t pos = wg_off[blockIdx.x] + li_block_excl(open ? 1u : 0u, &tot);
  if (!open) return;
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
  key[pos] = ((q - 1) << 32) | (uint64_t) (0xffffffffu - v);
  idx[pos] = (uint32_t) pos;
}

__global__ void __launch_bounds__(256) li_gather_kernel(const uint64_t *rec, const uint32_t *idx,
                                                        uint64_t n, uint64_t *out) {
  const uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t *r = rec + 5 * (uint64_t) idx[i];
  uint64_t *w = out + 5 * i;
#pragma unroll
  for (int f = 0; f < 5; f++) w[f] = r[f];
}

// father lb of leaf idx when it is attached in step 1 (LCP[idx+1] <= LCP[idx])
__global__ void __launch_bounds__(256) li_leaf_kernel(LiLevels L, uint64_t N, uint64_t *leaf_lb) {
  const uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (i >= N) return;
  const uint32_t xi = L.lv[0][i], xn = L.lv[0][i + 1];
  uint64_t lb = i;
  if (xn <= xi) lb = xi == 0 ? 0 : li_prev(L, i, xi, true);
  leaf_lb[i] = lb;
}

// ------------------------------------------------------------ host

static unsigned li_blocks(uint64_t n) { return (unsigned) ((n + 255) / 256); }

// Builds the tree on device 0: *itv (5 * *count, pop order) and, if
// leaf_lb != NULL, the N step-1 leaf fathers.  Host buffers are malloc'd.
static int li_build(const GtSmaxInput *in, uint64_t **itv, uint64_t *count, uint64_t **leaf_lb,
                    char *errbuf, size_t errlen) {
  uint8_t *lcp = NULL;
  GtSmaxLlv *llv = NULL;
  uint32_t *lev[LI_MAXLEV] = {NULL};
  uint32_t *derr = NULL, herr = 0, *wg_cnt = NULL, *idx_in = NULL, *idx_out = NULL;
  uint64_t *wg_off = NULL, *rec = NULL, *key_in = NULL, *key_out = NULL, *sorted = NULL,
           *dleaf = NULL;
  void *tmp = NULL;
  size_t tmp_bytes = 0;
  LiLevels L;
  uint64_t N, nwg, nitv = 0;
  memset(&L, 0, sizeof L);
  *itv = NULL;
  *count = 0;
  if (leaf_lb) *leaf_lb = NULL;
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
  if (N >= 0xffffffffull) {
    li_seterr(errbuf, errlen, "lcp-interval enumeration supports < 2^32 suffixes");
    return -1;
  }
  LICHK(hipSetDevice(0));
  LICHK(hipMalloc(&lcp, N + 1));
  LICHK(hipMemcpy(lcp, in->lcptab, N + 1, hipMemcpyHostToDevice));
  if (in->numllv > 0) {
    LICHK(hipMalloc(&llv, sizeof (GtSmaxLlv) * in->numllv));
    LICHK(hipMemcpy(llv, in->llvtab, sizeof (GtSmaxLlv) * in->numllv, hipMemcpyHostToDevice));
  }
  LICHK(hipMalloc(&derr, sizeof (uint32_t)));
  LICHK(hipMemset(derr, 0, sizeof (uint32_t)));
  // level 0: exact LCP, then 64-ary mins until one entry remains
  L.n[0] = N + 1;
  LICHK(hipMalloc(&lev[0], sizeof (uint32_t) * L.n[0]));
  hipLaunchKernelGGL(li_expand_kernel, dim3(li_blocks(N + 1)), dim3(256), 0, 0, lcp, N, lev[0]);
  LICHK(hipGetLastError());
  if (in->numllv > 0) {
    hipLaunchKernelGGL(li_llv_kernel, dim3(li_blocks(in->numllv)), dim3(256), 0, 0, llv,
                       in->numllv, lcp, N, lev[0], derr);
    LICHK(hipGetLastError());
  }
  L.nlev = 1;
  while (L.n[L.nlev - 1] > 1 && L.nlev < LI_MAXLEV) {
    const int l = L.nlev;
    L.n[l] = (L.n[l - 1] + 63) / 64;
    LICHK(hipMalloc(&lev[l], sizeof (uint32_t) * L.n[l]));
    hipLaunchKernelGGL(li_min64_kernel, dim3(li_blocks(L.n[l])), dim3(256), 0, 0, lev[l - 1],
                       L.n[l - 1], lev[l], L.n[l]);
    LICHK(hipGetLastError());
    L.nlev++;
  }
  for (int l = 0; l < L.nlev; l++) L.lv[l] = lev[l];
  LICHK(hipMemcpy(&herr, derr, sizeof herr, hipMemcpyDeviceToHost));
  if (herr & 1u) { li_seterr(errbuf, errlen, "lcp value >= 2^32-1 in .llv"); goto fail; }
  if (herr & 2u) { li_seterr(errbuf, errlen, "inconsistent .llv entry (lcp byte is not 255)"); goto fail; }
  // intervals: count per workgroup, scan, write, sort into pop order
  nwg = (N + 255) / 256;
  LICHK(hipMalloc(&wg_cnt, sizeof (uint32_t) * (nwg + 1)));
  LICHK(hipMalloc(&wg_off, sizeof (uint64_t) * (nwg + 1)));
  hipLaunchKernelGGL(li_count_kernel, dim3((unsigned) nwg), dim3(256), 0, 0, L, N, wg_cnt);
  LICHK(hipGetLastError());
  LICHK(rocprim::exclusive_scan(nullptr, tmp_bytes, wg_cnt, wg_off, (uint64_t) 0, (size_t) nwg,
                                rocprim::plus<uint64_t>(), (hipStream_t) 0));
  LICHK(hipMalloc(&tmp, tmp_bytes ? tmp_bytes : 16));
  LICHK(rocprim::exclusive_scan(tmp, tmp_bytes, wg_cnt, wg_off, (uint64_t) 0, (size_t) nwg,
                                rocprim::plus<uint64_t>(), (hipStream_t) 0));
  {
    uint64_t lo = 0;
    uint32_t lc = 0;
    LICHK(hipMemcpy(&lo, wg_off + nwg - 1, sizeof lo, hipMemcpyDeviceToHost));
    LICHK(hipMemcpy(&lc, wg_cnt + nwg - 1, sizeof lc, hipMemcpyDeviceToHost));
    nitv = lo + lc;
  }
  if (nitv > 0) {
    LICHK(hipMalloc(&rec, sizeof (uint64_t) * 5 * nitv));
    LICHK(hipMalloc(&key_in, sizeof (uint64_t) * nitv));
    LICHK(hipMalloc(&key_out, sizeof (uint64_t) * nitv));
    LICHK(hipMalloc(&idx_in, sizeof (uint32_t) * nitv));
    LICHK(hipMalloc(&idx_out, sizeof (uint32_t) * nitv));
    LICHK(hipMalloc(&sorted, sizeof (uint64_t) * 5 * nitv));
    hipLaunchKernelGGL(li_write_kernel, dim3((unsigned) nwg), dim3(256), 0, 0, L, N, wg_off, rec,
                       key_in, idx_in);
    LICHK(hipGetLastError());
    LICHK(hipFree(tmp));
    tmp = NULL;
    tmp_bytes = 0;
    LICHK(rocprim::radix_sort_pairs(nullptr, tmp_bytes, key_in, key_out, idx_in, idx_out,
                                    (size_t) nitv, 0, 64, (hipStream_t) 0));
    LICHK(hipMalloc(&tmp, tmp_bytes ? tmp_bytes : 16));
    LICHK(rocprim::radix_sort_pairs(tmp, tmp_bytes, key_in, key_out, idx_in, idx_out,
                                    (size_t) nitv, 0, 64, (hipStream_t) 0));
    hipLaunchKernelGGL(li_gather_kernel, dim3(li_blocks(nitv)), dim3(256), 0, 0, rec, idx_out,
                       nitv, sorted);
    LICHK(hipGetLastError());
    *itv = (uint64_t *) malloc(sizeof (uint64_t) * 5 * nitv);
    if (*itv == NULL) { li_seterr(errbuf, errlen, "out of memory"); goto fail; }
    LICHK(hipMemcpy(*itv, sorted, sizeof (uint64_t) * 5 * nitv, hipMemcpyDeviceToHost));
  }
  if (leaf_lb != NULL && N > 0) {
    LICHK(hipMalloc(&dleaf, sizeof (uint64_t) * N));
    hipLaunchKernelGGL(li_leaf_kernel, dim3(li_blocks(N)), dim3(256), 0, 0, L, N, dleaf);
    LICHK(hipGetLastError());
    *leaf_lb = (uint64_t *) malloc(sizeof (uint64_t) * N);
    if (*leaf_lb == NULL) { li_seterr(errbuf, errlen, "out of memory"); goto fail; }
    LICHK(hipMemcpy(*leaf_lb, dleaf, sizeof (uint64_t) * N, hipMemcpyDeviceToHost));
  }
  *count = nitv;
  {
    void *bufs[] = {lcp, llv, derr, wg_cnt, wg_off, rec, key_in, key_out, idx_in, idx_out,
                    sorted, dleaf, tmp};
    for (size_t i = 0; i < sizeof bufs / sizeof bufs[0]; i++)
      if (bufs[i]) (void) hipFree(bufs[i]);
    for (int l = 0; l < LI_MAXLEV; l++)
      if (lev[l]) (void) hipFree(lev[l]);
  }
  return 0;
fail:
  {
    void *bufs[] = {lcp, llv, derr, wg_cnt, wg_off, rec, key_in, key_out, idx_in, idx_out,
                    sorted, dleaf, tmp};
    for (size_t i = 0; i < sizeof bufs / sizeof bufs[0]; i++)
      if (bufs[i]) (void) hipFree(bufs[i]);
    for (int l = 0; l < LI_MAXLEV; l++)
      if (lev[l]) (void) hipFree(lev[l]);
  }
  free(*itv);
  *itv = NULL;
  if (leaf_lb) { free(*leaf_lb); *leaf_lb = NULL; }
  return -1;
}

extern "C" int gt_lcpitv_hip_enumerate_to_buffer(const GtSmaxInput *in, uint64_t **itv,
                                                 uint64_t *count, char *errbuf, size_t errlen) {
  return li_build(in, itv, count, NULL, errbuf, errlen);
}

// exact LCP of row k from the host tables (A3 decoding; llv cursor advances)
static inline uint64_t li_host_lcp(const GtSmaxInput *in, uint64_t k, uint64_t *cursor) {
  if (k == 0 || k >= in->nonspecials) return 0;
  const uint8_t b = in->lcptab[k];
  if (b < 255) return b;
  while (*cursor < in->numllv && in->llvtab[*cursor].position < k) (*cursor)++;
  return *cursor < in->numllv && in->llvtab[*cursor].position == k ? in->llvtab[*cursor].value
                                                                     : 255;
}

static inline uint64_t li_suffix(const GtSmaxInput *in, uint64_t k) {
  return in->suftab_bytes == 4 ? ((const uint32_t *) in->suftab)[k]
                               : ((const uint64_t *) in->suftab)[k];
}

// Replays gt_esa_bottomup's callback sequence (src/match/esa-bottomup.c:
// 131-271) from the tree: per row idx, with X = LCP[idx], Y = LCP[idx+1]:
//   Y <= X: leaf edge to the interval of depth X holding idx (lb from the GPU)
//   the intervals with rb == idx (pop order): lcp-interval callback, then
//     the branching edge to the father -- unless the father is new at idx
//     (same lb, depth Y), whose edge (firstsucc) comes after the pops
//   Y > X: leaf edge (firstsucc) to the new interval (Y, idx)
// firstsucc on an edge from the root: only the first such edge.
extern "C" int gt_esa_bottomup_hip(const GtSmaxInput *in, const GtLcpitvVisitor *v, void *data,
                                   char *errbuf, size_t errlen) {
  uint64_t *itv = NULL, *leaf_lb = NULL, count = 0, j = 0, cur2 = 0;
  int rc = 0;
  bool rootfirst = true;
  if (v == NULL) {
    li_seterr(errbuf, errlen, "missing visitor");
    return -1;
  }
  if (v->leaf_edge != NULL && (in == NULL || in->suftab == NULL ||
                               (in->suftab_bytes != 4 && in->suftab_bytes != 8))) {
    li_seterr(errbuf, errlen, "leaf edges need suftab (4 or 8 bytes per entry)");
    return -1;
  }
  if (li_build(in, &itv, &count, v->leaf_edge ? &leaf_lb : NULL, errbuf, errlen) != 0) return -1;
  const uint64_t N = in->nonspecials;
  uint64_t X = 0;
  for (uint64_t idx = 0; idx < N && rc == 0; idx++) {
    const uint64_t Y = li_host_lcp(in, idx + 1, &cur2);
    if (Y <= X && v->leaf_edge) {
      const bool first = X == 0 && rootfirst;
      if (X == 0) rootfirst = false;
      rc = v->leaf_edge(data, first, X, leaf_lb[idx], li_suffix(in, idx));
    } else if (Y <= X && X == 0) {
      rootfirst = false;
    }
    const uint64_t *last = NULL;
    while (rc == 0 && j < count && itv[5 * j + 2] == idx) {
      const uint64_t *r = itv + 5 * j++;
      if (v->lcp_interval) rc = v->lcp_interval(data, r[0], r[1], r[2]);
      if (rc != 0) break;
      if (r[3] > 0 && r[4] == r[1]) {
        last = r;                        // father pushed after the pops
      } else {
        const bool first = r[3] == 0 && rootfirst;
        if (r[3] == 0) rootfirst = false;
        if (v->branching_edge) rc = v->branching_edge(data, first, r[3], r[4], r[0], r[1], r[2]);
      }
    }
    if (rc == 0 && last != NULL) {
      if (v->branching_edge) rc = v->branching_edge(data, true, last[3], last[1], last[0], last[1],
                                                    last[2]);
    } else if (rc == 0 && Y > X && v->leaf_edge) {
      rc = v->leaf_edge(data, true, Y, idx, li_suffix(in, idx));
    }
    X = Y;
  }
  free(itv);
  free(leaf_lb);
  if (rc != 0) {
    li_seterr(errbuf, errlen, "visitor callback returned non-zero");
    return -1;
  }
  return 0;
}
