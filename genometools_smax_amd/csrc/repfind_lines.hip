// repfind_lines.hip -- `gt repfind` output lines formatted on the GPU
// (SURVEY.md §8(f) F4).  Every pair (len, pos1, pos2) becomes the line
// gt_simpleexactselfmatchoutput + gt_querymatch_output print
// (src/tools/gt_repfind.c:49-84, src/match/querymatch.c:130-190):
//
//   "<len> <seqnum1> <relpos1> F <len> <seqnum2> <relpos2>\n"
//
// with pos1 < pos2 after the swap (gt_repfind.c:60-65), seqnum = number of
// separators before the position (gt_encseq_seqnum, src/core/encseq.c:3815-3840),
// relpos = position - start of its sequence, and the line suppressed when
// both positions lie in one sequence and relpos1 > relpos2
// (querymatch.c:157-159; never true after the swap, kept for fidelity).
//
// Two passes per chunk of pairs: line lengths -> exclusive scan -> every
// thread writes its line at its offset (byte stores; text is ~30 B/line).
// The pairs come either from a device pair array (maximal pairs, F2) or are
// generated from supermaximal-repeat records -- all occurrence pairs a < b of
// every interval, in the order the host CLI prints them -- by mapping a
// global pair index to (interval, a, b) with a binary search over the
// intervals' pair offsets, so no pair array is materialised for smax.
// Chunks of at most RL_CHUNK pairs bound the device text buffer; each chunk
// goes to the caller's GtRepfindTextFunc.
#include <hip/hip_runtime.h>
#include <math.h>
#include <rocprim/device/device_scan.hpp>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gt_maxpairs_hip.h"
#include "smax_internal.h"

static void rl_seterr(char *errbuf, size_t errlen, const char *fmt, ...) {
  if (errbuf == NULL || errlen == 0) return;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(errbuf, errlen, fmt, ap);
  va_end(ap);
}

#define RLCHK(call)                                                                  \
  do {                                                                               \
    hipError_t e_ = (call);                                                          \
    if (e_ != hipSuccess) {                                                          \
      rl_seterr(errbuf, errlen, "%s: %s (%s:%d)", #call, hipGetErrorString(e_),      \
                __FILE__, __LINE__);                                                 \
      goto fail;                                                                     \
    }                                                                                \
  } while (0)

#define RL_CHUNK (1ull << 22)   // pairs per chunk (<= 128 B per line)

static unsigned rl_blocks(uint64_t n) { return (unsigned) ((n + 255) / 256); }

__device__ __forceinline__ uint32_t rl_digits(uint64_t v) {
  uint32_t d = 1;
  while (v >= 10) { v /= 10; d++; }
  return d;
}

__device__ __forceinline__ char *rl_put(char *w, uint64_t v, uint32_t d) {
  for (uint32_t k = d; k > 0; k--) { w[k - 1] = (char) ('0' + v % 10); v /= 10; }
  return w + d;
}

struct RlSep {
  const uint64_t *sep;
  uint64_t nsep;
};

// (seqnum, relpos) of position p
__device__ __forceinline__ void rl_seqpos(const RlSep &s, uint64_t p, uint64_t *sn, uint64_t *rp) {
  uint64_t lo = 0, hi = s.nsep;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (s.sep[mid] < p) lo = mid + 1; else hi = mid;
  }
  *sn = lo;
  *rp = p - (lo == 0 ? 0 : s.sep[lo - 1] + 1);
}

// length of the pair's line (0: suppressed); writes it when w != nullptr
__device__ __forceinline__ uint32_t rl_line(const RlSep &s, uint64_t len, uint64_t p1, uint64_t p2,
                                            char *w) {
  if (p1 > p2) { const uint64_t t = p1; p1 = p2; p2 = t; }
  uint64_t s1, r1, s2, r2;
  rl_seqpos(s, p1, &s1, &r1);
  rl_seqpos(s, p2, &s2, &r2);
  if (s1 == s2 && r1 > r2) return 0;
  const uint32_t dl = rl_digits(len), d1 = rl_digits(s1), e1 = rl_digits(r1), d2 = rl_digits(s2),
                 e2 = rl_digits(r2);
  const uint32_t n = 2 * dl + d1 + e1 + d2 + e2 + 8;   // 6 blanks, 'F', '\n'
  if (w != nullptr) {
    w = rl_put(w, len, dl); *w++ = ' ';
    w = rl_put(w, s1, d1); *w++ = ' ';
    w = rl_put(w, r1, e1); *w++ = ' '; *w++ = 'F'; *w++ = ' ';
    w = rl_put(w, len, dl); *w++ = ' ';
    w = rl_put(w, s2, d2); *w++ = ' ';
    w = rl_put(w, r2, e2); *w = '\n';
  }
  return n;
}

// pair source 1: a device array of (len, pos1, pos2) triples
struct RlPairs {
  const uint64_t *p;
  __device__ __forceinline__ void get(uint64_t g, uint64_t *len, uint64_t *a, uint64_t *b) const {
    *len = p[3 * g]; *a = p[3 * g + 1]; *b = p[3 * g + 2];
  }
};

// pair source 2: supermaximal-repeat records; record r covers occurrences
// occ[rec[r].lb .. rec[r].lb + width) and the pairs [poff[r], poff[r+1]) in
// the order (a, b), a < b, a outer
struct RlSmax {
  const GtSmaxRecord *rec;
  const uint64_t *poff;       // nrec + 1 inclusive-from-0 offsets
  uint64_t nrec;
  const void *occ;
  int occ_bytes;
  __device__ __forceinline__ uint64_t pos(uint64_t k) const {
    return occ_bytes == 8 ? reinterpret_cast<const uint64_t *>(occ)[k]
                          : (uint64_t) reinterpret_cast<const uint32_t *>(occ)[k];
  }
  __device__ __forceinline__ void get(uint64_t g, uint64_t *len, uint64_t *pa, uint64_t *pb) const {
    uint64_t lo = 0, hi = nrec;                 // last r with poff[r] <= g
    while (hi - lo > 1) {
      const uint64_t mid = (lo + hi) >> 1;
      if (poff[mid] <= g) lo = mid; else hi = mid;
    }
    const GtSmaxRecord R = rec[lo];
    const uint64_t w = R.width, k = g - poff[lo];
    // a = largest a with start(a) = a(w-1) - a(a-1)/2 <= k
    const double W = (double) (2 * w - 1);
    int64_t a = (int64_t) ((W - sqrt(W * W - 8.0 * (double) k)) * 0.5);
    if (a < 0) a = 0;
    auto start = [w](int64_t x) { return (uint64_t) x * (w - 1) - (uint64_t) x * (uint64_t) (x - 1) / 2; };
    while (a > 0 && start(a) > k) a--;
    while ((uint64_t) (a + 1) < w && start(a + 1) <= k) a++;
    const uint64_t b = (uint64_t) a + 1 + (k - start(a));
    *len = R.lcp;
    *pa = pos(R.lb + (uint64_t) a);
    *pb = pos(R.lb + b);
  }
};

template <typename Src>
__global__ void __launch_bounds__(256) rl_len_kernel(Src src, RlSep s, uint64_t g0, uint64_t n,
                                                     uint64_t *len_out) {
  const uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t l, a, b;
  src.get(g0 + i, &l, &a, &b);
  len_out[i] = rl_line(s, l, a, b, nullptr);
}

template <typename Src>
__global__ void __launch_bounds__(256) rl_write_kernel(Src src, RlSep s, uint64_t g0, uint64_t n,
                                                       const uint64_t *off, char *text) {
  const uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t l, a, b;
  src.get(g0 + i, &l, &a, &b);
  (void) rl_line(s, l, a, b, text + off[i]);
}

// pairs per record: width (width - 1) / 2
__global__ void __launch_bounds__(256) rl_smax_pairs_kernel(const GtSmaxRecord *rec, uint64_t n,
                                                            uint64_t *cnt) {
  const uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t w = rec[i].width;
  cnt[i] = w * (w - 1) / 2;
}

// Formats pairs [0, total) of src chunk by chunk into device text and hands
// every chunk (copied to host) to cb.  Runs on the current device.
template <typename Src>
static int rl_format(const Src &src, uint64_t total, const RlSep &s, GtRepfindTextFunc cb,
                     void *data, char *errbuf, size_t errlen) {
  uint64_t *len = NULL, *off = NULL;
  char *text = NULL, *host = NULL;
  void *tmp = NULL;
  size_t tb = 0;
  uint64_t textcap = 0, hostcap = 0;
  const uint64_t C = total < RL_CHUNK ? total : RL_CHUNK;
  int rc = -1;
  if (total == 0) return 0;
  RLCHK(hipMalloc(&len, sizeof (uint64_t) * (C + 1)));
  RLCHK(hipMalloc(&off, sizeof (uint64_t) * (C + 1)));
  RLCHK(rocprim::exclusive_scan(nullptr, tb, len, off, (uint64_t) 0, (size_t) (C + 1),
                                rocprim::plus<uint64_t>()));
  RLCHK(hipMalloc(&tmp, tb ? tb : 16));
  for (uint64_t g0 = 0; g0 < total; g0 += C) {
    const uint64_t n = total - g0 < C ? total - g0 : C;
    uint64_t bytes = 0;
    hipLaunchKernelGGL(rl_len_kernel<Src>, dim3(rl_blocks(n)), dim3(256), 0, 0, src, s, g0, n, len);
    RLCHK(hipGetLastError());
    RLCHK(hipMemset(len + n, 0, sizeof (uint64_t)));
    size_t b = tb;
    RLCHK(rocprim::exclusive_scan(tmp, b, len, off, (uint64_t) 0, (size_t) (n + 1),
                                  rocprim::plus<uint64_t>()));
    RLCHK(hipMemcpy(&bytes, off + n, sizeof bytes, hipMemcpyDeviceToHost));
    if (bytes == 0) continue;
    if (bytes > textcap) {
      if (text) RLCHK(hipFree(text));
      text = NULL;
      RLCHK(hipMalloc(&text, bytes));
      textcap = bytes;
    }
    if (bytes > hostcap) {
      if (host) RLCHK(hipHostFree(host));
      host = NULL;
      RLCHK(hipHostMalloc((void **) &host, bytes, hipHostMallocDefault));
      hostcap = bytes;
    }
    hipLaunchKernelGGL(rl_write_kernel<Src>, dim3(rl_blocks(n)), dim3(256), 0, 0, src, s, g0, n, off,
                       text);
    RLCHK(hipGetLastError());
    RLCHK(hipMemcpy(host, text, bytes, hipMemcpyDeviceToHost));
    if (cb(data, host, bytes) != 0) {
      rl_seterr(errbuf, errlen, "output callback returned non-zero");
      goto fail;
    }
  }
  rc = 0;
fail:
  if (len) (void) hipFree(len);
  if (off) (void) hipFree(off);
  if (tmp) (void) hipFree(tmp);
  if (text) (void) hipFree(text);
  if (host) (void) hipHostFree(host);
  return rc;
}

extern "C" int gt_repfind_pairs_lines_dev(const uint64_t *pairs_dev, uint64_t count,
                                          const uint64_t *sep_dev, uint64_t nsep, int device,
                                          GtRepfindTextFunc cb, void *data, char *errbuf,
                                          size_t errlen) {
  int cur = -1;
  (void) hipGetDevice(&cur);
  if (hipSetDevice(device) != hipSuccess) {
    rl_seterr(errbuf, errlen, "hipSetDevice(%d) failed", device);
    return -1;
  }
  RlPairs src{pairs_dev};
  RlSep s{sep_dev, nsep};
  const int rc = rl_format(src, count, s, cb, data, errbuf, errlen);
  if (cur >= 0) (void) hipSetDevice(cur);   // the caller's device again
  return rc;
}

extern "C" int gt_repfind_smax_lines(const GtSmaxRecord *rec, uint64_t nrec, const uint64_t *occpos,
                                     uint64_t nocc, const uint64_t *sep, uint64_t nsep,
                                     GtRepfindTextFunc cb, void *data, char *errbuf,
                                     size_t errlen) {
  GtSmaxRecord *drec = NULL;
  uint64_t *docc = NULL, *dsep = NULL, *cnt = NULL, *poff = NULL;
  void *tmp = NULL;
  size_t tb = 0;
  uint64_t total = 0;
  int rc = -1;
  if (errbuf && errlen) errbuf[0] = 0;
  for (uint64_t r = 0; r < nrec; r++)
    if (rec[r].width < 2 || rec[r].lb + rec[r].width > nocc) {
      rl_seterr(errbuf, errlen, "record %lu: occurrences [%lu, +%u) outside the %lu positions",
                (unsigned long) r, (unsigned long) rec[r].lb, rec[r].width, (unsigned long) nocc);
      return -1;
    }
  if (nrec == 0) return 0;
  // formats on the caller's current device (hipSetDevice before the call)
  RLCHK(hipMalloc(&drec, sizeof (GtSmaxRecord) * nrec));
  RLCHK(hipMalloc(&docc, sizeof (uint64_t) * (nocc ? nocc : 1)));
  RLCHK(hipMalloc(&dsep, sizeof (uint64_t) * (nsep ? nsep : 1)));
  RLCHK(hipMalloc(&cnt, sizeof (uint64_t) * (nrec + 1)));
  RLCHK(hipMalloc(&poff, sizeof (uint64_t) * (nrec + 1)));
  RLCHK(hipMemcpy(drec, rec, sizeof (GtSmaxRecord) * nrec, hipMemcpyHostToDevice));
  if (nocc) RLCHK(hipMemcpy(docc, occpos, sizeof (uint64_t) * nocc, hipMemcpyHostToDevice));
  if (nsep) RLCHK(hipMemcpy(dsep, sep, sizeof (uint64_t) * nsep, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(rl_smax_pairs_kernel, dim3(rl_blocks(nrec)), dim3(256), 0, 0, drec, nrec, cnt);
  RLCHK(hipGetLastError());
  RLCHK(hipMemset(cnt + nrec, 0, sizeof (uint64_t)));
  RLCHK(rocprim::exclusive_scan(nullptr, tb, cnt, poff, (uint64_t) 0, (size_t) (nrec + 1),
                                rocprim::plus<uint64_t>()));
  RLCHK(hipMalloc(&tmp, tb ? tb : 16));
  RLCHK(rocprim::exclusive_scan(tmp, tb, cnt, poff, (uint64_t) 0, (size_t) (nrec + 1),
                                rocprim::plus<uint64_t>()));
  RLCHK(hipMemcpy(&total, poff + nrec, sizeof total, hipMemcpyDeviceToHost));
  {
    RlSmax src{drec, poff, nrec, docc, 8};
    RlSep s{dsep, nsep};
    rc = rl_format(src, total, s, cb, data, errbuf, errlen);
  }
fail:
  {
    void *bufs[] = {drec, docc, dsep, cnt, poff, tmp};
    for (size_t i = 0; i < sizeof bufs / sizeof bufs[0]; i++)
      if (bufs[i]) (void) hipFree(bufs[i]);
  }
  return rc;
}
