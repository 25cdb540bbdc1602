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
// Pass 1 + an exclusive scan give every row its output offset, so pass 2
// writes the pairs without atomics.  Rows outside blocks (most rows of
// non-repetitive input) exit after one load.  The walk reads X (exact LCP,
// u32) and BWT 8 rows per step (neighbouring lanes walk neighbouring rows:
// each step of a wave is one contiguous segment), so the loop-carried
// minimum never waits on a single load.
//
// Integer/byte work; bound by the number of (row, earlier row in block)
// candidates, i.e. by the output size.  No MFMA.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_scan.hpp>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gt_maxpairs_hip.h"

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

// ------------------------------------------------------------ kernels

// X[k] = exact LCP[k] for k in [0, N] (0 at k = 0 and k = N; the 255 bytes
// are overwritten by mp_llv_kernel).  A3 decoding, src/match/esa-seqread.h:96-215.
__global__ void __launch_bounds__(256) mp_expand_kernel(const uint8_t *lcp, uint64_t N,
                                                        uint32_t *X) {
  const uint64_t k = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (k > N) return;
  X[k] = (k == 0 || k == N) ? 0u : (uint32_t) lcp[k];
}

// .llv values over their 255 bytes; err bit 1: value >= 2^32, bit 2: a
// position whose byte is not 255 (inconsistent index)
__global__ void __launch_bounds__(256) mp_llv_kernel(const GtSmaxLlv *llv, uint64_t numllv,
                                                     const uint8_t *lcp, uint64_t N, uint32_t *X,
                                                     uint32_t *err) {
  const uint64_t e = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (e >= numllv) return;
  const uint64_t pos = llv[e].position, v = llv[e].value;
  if (pos < 1 || pos >= N) return;
  if (v > 0xffffffffull) atomicOr(err, 1u);
  if (lcp[pos] != 255) atomicOr(err, 2u);
  X[pos] = (uint32_t) v;
}

template <typename SufT>
__device__ __forceinline__ uint64_t suf_at(const void *S, uint64_t k) {
  return (uint64_t) reinterpret_cast<const SufT *>(S)[k];
}

// Pass 1 (EMIT = false): cnt[j] = number of maximal pairs (i, j), i < j.
// Pass 2 (EMIT = true): writes them at off[j] as (len, pos1 < pos2).
template <bool EMIT, typename SufT>
__global__ void __launch_bounds__(256)
mp_walk_kernel(const uint32_t *X, const uint8_t *B, const void *S, uint64_t N, uint32_t minlen,
               uint64_t *cnt, const uint64_t *off, uint64_t *out, uint64_t capacity) {
  const uint64_t j = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (j >= N) return;
  uint32_t m = X[j];                       // depth of the pair (j-1, j)
  uint64_t c = 0;
  if (j > 0 && m >= minlen) {
    const uint32_t bj = B[j];
    const bool uj = bj >= 254u;            // unique left context
    const uint64_t o = EMIT ? off[j] : 0;
    const uint64_t sj = EMIT ? suf_at<SufT>(S, j) : 0;
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
#pragma unroll
      for (int q = 0; q < MP_STEP; q++) {
        if (!more) break;
        // row i-q pairs with j at depth m = min LCP[i-q+1 .. j]
        if (uj || bi[q] != bj) {
          if (EMIT && o + c < capacity) {
            uint64_t *w = out + 3 * (o + c);
            w[0] = m;
            w[1] = si[q] < sj ? si[q] : sj;
            w[2] = si[q] < sj ? sj : si[q];
          }
          c++;
        }
        m = xi[q] < m ? xi[q] : m;         // X[0] == 0 ends every walk
        if (m < minlen) more = false;
      }
      i -= MP_STEP;
    }
  }
  if (!EMIT) cnt[j] = c;
}

__global__ void mp_total_kernel(const uint64_t *cnt, const uint64_t *off, uint64_t N,
                                uint64_t *total) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *total = N == 0 ? 0 : off[N - 1] + cnt[N - 1];
}

// F4: (len, pos1, pos2) -> (len, seqnum1, relpos1, seqnum2, relpos2); seqnum
// = number of separators before the position (gt_encseq_seqnum,
// src/core/encseq.c:3815-3840), relpos = position - sequence start
// (gt_encseq_seqstartpos, :3842-3885).
__global__ void __launch_bounds__(256) seqpos_map_kernel(const uint64_t *sep, uint64_t nsep,
                                                         const uint64_t *pairs, uint64_t count,
                                                         uint64_t *out) {
  const uint64_t k = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (k >= count) return;
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

// ------------------------------------------------------------ plan

struct GtMaxpairsPlan {
  GtMaxpairsDevInput in;
  unsigned int minlen;
  uint32_t *X;          // N+1 exact LCP values
  uint64_t *cnt, *off;  // N pair counts, N exclusive offsets
  uint64_t *total;      // 1
  void *scan_tmp;
  size_t scan_tmp_bytes;
  bool counted;
};

static unsigned mp_blocks(uint64_t n) { return (unsigned) ((n + 255) / 256); }

extern "C" void gt_maxpairs_plan_delete(GtMaxpairsPlan *p) {
  if (p == NULL) return;
  (void) hipSetDevice(p->in.device);
  void *bufs[] = {p->X, p->cnt, p->off, p->total, p->scan_tmp};
  for (size_t i = 0; i < sizeof bufs / sizeof bufs[0]; i++)
    if (bufs[i]) (void) hipFree(bufs[i]);
  free(p);
}

extern "C" int gt_maxpairs_plan_create(GtMaxpairsPlan **planp, const GtMaxpairsDevInput *in,
                                       unsigned int minlen, char *errbuf, size_t errlen) {
  GtMaxpairsPlan *p = NULL;
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
  p = (GtMaxpairsPlan *) calloc(1, sizeof *p);
  if (p == NULL) {
    mp_seterr(errbuf, errlen, "out of memory");
    return -1;
  }
  p->in = *in;
  p->minlen = minlen;
  MPCHK(hipSetDevice(in->device));
  MPCHK(hipMalloc(&p->X, sizeof (uint32_t) * (N + 1)));
  MPCHK(hipMalloc(&p->cnt, sizeof (uint64_t) * (N + 1)));
  MPCHK(hipMalloc(&p->off, sizeof (uint64_t) * (N + 1)));
  MPCHK(hipMalloc(&p->total, sizeof (uint64_t)));
  MPCHK(hipMemset(p->total, 0, sizeof (uint64_t)));
  MPCHK(hipMalloc(&derr, sizeof (uint32_t)));
  MPCHK(hipMemset(derr, 0, sizeof (uint32_t)));
  hipLaunchKernelGGL(mp_expand_kernel, dim3(mp_blocks(N + 1)), dim3(256), 0, 0, in->lcp_dev, N,
                     p->X);
  MPCHK(hipGetLastError());
  if (in->numllv > 0) {
    hipLaunchKernelGGL(mp_llv_kernel, dim3(mp_blocks(in->numllv)), dim3(256), 0, 0, in->llv_dev,
                       in->numllv, in->lcp_dev, N, p->X, derr);
    MPCHK(hipGetLastError());
  }
  if (N > 0) {
    MPCHK(rocprim::exclusive_scan(nullptr, p->scan_tmp_bytes, p->cnt, p->off, (uint64_t) 0,
                                  (size_t) N, rocprim::plus<uint64_t>(), (hipStream_t) 0));
  }
  MPCHK(hipMalloc(&p->scan_tmp, p->scan_tmp_bytes ? p->scan_tmp_bytes : 16));
  MPCHK(hipMemcpy(&herr, derr, sizeof herr, hipMemcpyDeviceToHost));
  if (herr & 1u) { mp_seterr(errbuf, errlen, "lcp value >= 2^32 in .llv"); goto fail; }
  if (herr & 2u) { mp_seterr(errbuf, errlen, "inconsistent .llv entry (lcp byte is not 255)"); goto fail; }
  (void) hipFree(derr);
  *planp = p;
  return 0;
fail:
  if (derr) (void) hipFree(derr);
  gt_maxpairs_plan_delete(p);
  return -1;
}

extern "C" int gt_maxpairs_plan_count(GtMaxpairsPlan *p, void *stream) {
  char *errbuf = NULL;
  size_t errlen = 0;
  hipStream_t s = (hipStream_t) stream;
  const uint64_t N = p->in.nonspecials;
  MPCHK(hipSetDevice(p->in.device));
  if (N == 0) {
    MPCHK(hipMemsetAsync(p->total, 0, sizeof (uint64_t), s));
  } else {
    if (p->in.suf_bytes == 8)
      hipLaunchKernelGGL((mp_walk_kernel<false, uint64_t>), dim3(mp_blocks(N)), dim3(256), 0, s,
                         p->X, p->in.bwt_dev, p->in.suf_dev, N, p->minlen, p->cnt, nullptr,
                         nullptr, 0);
    else
      hipLaunchKernelGGL((mp_walk_kernel<false, uint32_t>), dim3(mp_blocks(N)), dim3(256), 0, s,
                         p->X, p->in.bwt_dev, p->in.suf_dev, N, p->minlen, p->cnt, nullptr,
                         nullptr, 0);
    MPCHK(hipGetLastError());
    size_t bytes = p->scan_tmp_bytes;
    MPCHK(rocprim::exclusive_scan(p->scan_tmp, bytes, p->cnt, p->off, (uint64_t) 0, (size_t) N,
                                  rocprim::plus<uint64_t>(), s));
    hipLaunchKernelGGL(mp_total_kernel, dim3(1), dim3(64), 0, s, p->cnt, p->off, N, p->total);
    MPCHK(hipGetLastError());
  }
  p->counted = true;
  return 0;
fail:
  return -1;
}

extern "C" int gt_maxpairs_plan_total(GtMaxpairsPlan *p, uint64_t *total) {
  char *errbuf = NULL;
  size_t errlen = 0;
  MPCHK(hipSetDevice(p->in.device));
  MPCHK(hipDeviceSynchronize());
  MPCHK(hipMemcpy(total, p->total, sizeof (uint64_t), hipMemcpyDeviceToHost));
  return 0;
fail:
  return -1;
}

extern "C" int gt_maxpairs_plan_emit(GtMaxpairsPlan *p, uint64_t *out_dev, uint64_t capacity,
                                     void *stream) {
  char *errbuf = NULL;
  size_t errlen = 0;
  hipStream_t s = (hipStream_t) stream;
  const uint64_t N = p->in.nonspecials;
  if (!p->counted) return -1;
  MPCHK(hipSetDevice(p->in.device));
  if (N == 0 || capacity == 0) return 0;
  if (p->in.suf_bytes == 8)
    hipLaunchKernelGGL((mp_walk_kernel<true, uint64_t>), dim3(mp_blocks(N)), dim3(256), 0, s,
                       p->X, p->in.bwt_dev, p->in.suf_dev, N, p->minlen, nullptr, p->off, out_dev,
                       capacity);
  else
    hipLaunchKernelGGL((mp_walk_kernel<true, uint32_t>), dim3(mp_blocks(N)), dim3(256), 0, s,
                       p->X, p->in.bwt_dev, p->in.suf_dev, N, p->minlen, nullptr, p->off, out_dev,
                       capacity);
  MPCHK(hipGetLastError());
  return 0;
fail:
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

// Host tables -> HBM, count, emit, D2H.  *pairs is malloc'd (3 * *count).
static int mp_host_run(const GtSmaxInput *in, unsigned int minlen, uint64_t **pairs,
                       uint64_t *count, char *errbuf, size_t errlen) {
  uint8_t *lcp = NULL, *bwt = NULL;
  GtSmaxLlv *llv = NULL;
  void *suf = NULL;
  uint64_t *out = NULL, total = 0;
  GtMaxpairsPlan *plan = NULL;
  GtMaxpairsDevInput din;
  uint64_t N;
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
  MPCHK(hipSetDevice(0));
  MPCHK(hipMalloc(&lcp, N + 1));
  MPCHK(hipMalloc(&bwt, N + 1));
  MPCHK(hipMalloc(&suf, (size_t) in->suftab_bytes * (N + 1)));
  MPCHK(hipMemcpy(lcp, in->lcptab, N + 1, hipMemcpyHostToDevice));
  MPCHK(hipMemcpy(bwt, in->bwttab, N + 1, hipMemcpyHostToDevice));
  MPCHK(hipMemcpy(suf, in->suftab, (size_t) in->suftab_bytes * (N + 1), hipMemcpyHostToDevice));
  if (in->numllv > 0) {
    MPCHK(hipMalloc(&llv, sizeof (GtSmaxLlv) * in->numllv));
    MPCHK(hipMemcpy(llv, in->llvtab, sizeof (GtSmaxLlv) * in->numllv, hipMemcpyHostToDevice));
  }
  din.lcp_dev = lcp;
  din.bwt_dev = bwt;
  din.llv_dev = llv;
  din.numllv = in->numllv;
  din.suf_dev = suf;
  din.suf_bytes = in->suftab_bytes;
  din.nonspecials = N;
  din.device = 0;
  if (gt_maxpairs_plan_create(&plan, &din, minlen, errbuf, errlen) != 0) goto fail_quiet;
  if (gt_maxpairs_plan_count(plan, NULL) != 0 || gt_maxpairs_plan_total(plan, &total) != 0) {
    mp_seterr(errbuf, errlen, "maxpairs count pass failed");
    goto fail_quiet;
  }
  if (total > 0) {
    *pairs = (uint64_t *) malloc(sizeof (uint64_t) * 3 * total);
    if (*pairs == NULL) {
      mp_seterr(errbuf, errlen, "out of memory (%lu pairs)", (unsigned long) total);
      goto fail_quiet;
    }
    MPCHK(hipMalloc(&out, sizeof (uint64_t) * 3 * total));
    if (gt_maxpairs_plan_emit(plan, out, total, NULL) != 0) {
      mp_seterr(errbuf, errlen, "maxpairs emission pass failed");
      goto fail_quiet;
    }
    MPCHK(hipMemcpy(*pairs, out, sizeof (uint64_t) * 3 * total, hipMemcpyDeviceToHost));
  }
  *count = total;
  gt_maxpairs_plan_delete(plan);
  {
    void *bufs[] = {lcp, bwt, suf, llv, out};
    for (size_t i = 0; i < sizeof bufs / sizeof bufs[0]; i++)
      if (bufs[i]) (void) hipFree(bufs[i]);
  }
  return 0;
fail:
fail_quiet:
  gt_maxpairs_plan_delete(plan);
  {
    void *bufs[] = {lcp, bwt, suf, llv, out};
    for (size_t i = 0; i < sizeof bufs / sizeof bufs[0]; i++)
      if (bufs[i]) (void) hipFree(bufs[i]);
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
