// esa_build64.hip -- GPU construction of the smax inputs for texts of any
// length (64-bit suffix array; SURVEY.md §8(f) F1, BASELINE config C5: 12 Gbp
// needs > 2^32 suffixes, for which the reference makes the 8-byte suftab
// mandatory, src/match/sfx-suffixgetset.c:48-51), restricted to a range of
// suffix-array rows so that every rank of a multi-GPU run builds only the
// rows it scans.
//
// Output tables are those of `gt suffixerator -dna -suf -lcp -bwt`
// (src/match/sfx-run.c:174-300, src/match/sfx-lcpvalues.c:371-470): rows
// ordered by suffix with specials (WILDCARD, SEPARATOR, end of text) unique
// and ranked by position after every base; .lcp bytes with values >= 255 in
// .llv; .bwt bytes (254 for suffix 0), plus the packed bit-plane BWT the smax
// scan streams.  Byte-identical to esa_build.hip where both apply (tested).
//
// Algorithm (MI355X-first, memory-bounded; no global inverse suffix array,
// so a rank never holds more than its rows' state):
//   1. the text goes to HBM in chunks and is packed to 2 bits + a special
//      bitmap + a separator bitmap (the .bwt distinguishes 254 and 255);
//   2. every suffix gets a bucket: its first 10 symbols in a 5-letter order
//      alphabet (a special ends the prefix as the largest letter); a global
//      histogram + scan gives each bucket its first suffix-array row;
//   3. consecutive buckets covering the requested rows form batches of at
//      most `batch_max` suffixes; per batch: the suffix positions of its
//      buckets are selected in position order (rocPRIM select over all
//      positions), stably radix-sorted by bucket, then refined in rounds:
//      the still-tied suffixes get keys (dense group id, next 21-ish symbols
//      at 3 bits) and one stable radix sort per round splits their groups;
//      keys holding a special are final (ties by position, kept by the
//      stable sorts);
//   4. each row's LCP with its predecessor starts from the depth at which the
//      two last shared a group (at most one 32-symbol compare), the BWT byte
//      comes from the bitmaps, .llv entries are compacted per batch.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "esa_common.h"
#include "gt_smax_esa.h"
#include "gt_smax_hip.h"

namespace {

constexpr int kB = 10;                       // bucket prefix symbols
constexpr uint32_t kNB = 9765625;            // 5^10 buckets
constexpr uint64_t kChunk = 1ull << 30;      // positions per select call

void seterr(char *errbuf, size_t errlen, const char *fmt, ...) {
  if (errbuf == NULL || errlen == 0) return;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(errbuf, errlen, fmt, ap);
  va_end(ap);
}

#define HIPCHK(call)                                                         \
  do {                                                                       \
    hipError_t e_ = (call);                                                  \
    if (e_ != hipSuccess) {                                                  \
      seterr(errbuf, errlen, "%s: %s (%s:%d)", #call, hipGetErrorString(e_), \
             __FILE__, __LINE__);                                            \
      goto fail;                                                             \
    }                                                                        \
  } while (0)

// Launch sizes: a dispatch holds fewer than 2^32 work-items (the packet's
// grid size is 32-bit), so every kernel that may see more elements than
// that (positions of a > 4 Gbp text) is a grid-stride loop over a capped grid.
constexpr uint64_t kMaxBlocks = (1ull << 32) / 256 - 1;
inline unsigned blocks(uint64_t n, unsigned t = 256) {
  uint64_t b = (n + t - 1) / t;
  return (unsigned) (b > kMaxBlocks ? kMaxBlocks : (b ? b : 1));
}

// ------------------------------------------------------------ kernels

// words [w0, w0 + nw) of P/S/SEP from text bytes T[0 ..) = positions
// 64*w0 .. (a chunk starting at a word boundary); positions >= n special
__global__ void k_pack64(const uint8_t *T, uint64_t w0, uint64_t nw, uint64_t n, uint64_t *P,
                         uint64_t *S, uint64_t *SEP) {
  const uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (i >= nw) return;
  const uint64_t w = w0 + i, base = w * 64;
  uint64_t s = 0, sep = 0, p0 = 0, p1 = 0;
  for (int k = 0; k < 64; k++) {
    const uint64_t p = base + k;
    const uint32_t c = p < n ? T[i * 64 + k] : 255u;
    uint64_t sym = 0;
    if (c >= 254) {
      s |= 1ull << k;
      if (c == 255 && p < n) sep |= 1ull << k;
    } else {
      sym = c & 3u;
    }
    if (k < 32) p0 |= sym << (2 * k); else p1 |= sym << (2 * (k - 32));
  }
  S[w] = s;
  SEP[w] = sep;
  P[2 * w] = p0;
  P[2 * w + 1] = p1;
}

__global__ void k_count_specials(const uint64_t *S, uint64_t n, unsigned long long *cnt) {
  const uint64_t w = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  uint32_t c = 0;
  if (w * 64 < n) {
    uint64_t v = S[w];
    const uint64_t left = n - w * 64;
    if (left < 64) v &= (1ull << left) - 1;
    c = (uint32_t) __popcll(v);
  }
  for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(cnt, (unsigned long long) c);
}

__device__ __forceinline__ uint32_t bucket_of(const uint64_t *P, const uint64_t *S, uint64_t p) {
  const uint64_t sy = esa_sym32(P, p);
  const uint32_t sp = esa_spec32(S, p) & ((1u << kB) - 1u);
  const int first = sp ? __builtin_ctz(sp) : kB;
  uint32_t id = 0;
#pragma unroll
  for (int c = 0; c < kB; c++) {
    const uint32_t d = c < first ? (uint32_t) ((sy >> (2 * c)) & 3u) : (c == first ? 4u : 0u);
    id = id * 5u + d;
  }
  return id;
}

// bucket ids whose prefix ends in a special: all their suffixes are ranked
// by position (resolved at once)
__device__ __forceinline__ bool bucket_special(uint32_t id) {
  for (int c = 0; c < kB; c++) {
    if (id % 5u == 4u) return true;
    id /= 5u;
  }
  return false;
}

__global__ void k_bucket_count(const uint64_t *P, const uint64_t *S, uint64_t m,
                               unsigned long long *cnt) {
  const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
  for (uint64_t p = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; p < m; p += stride)
    atomicAdd(&cnt[bucket_of(P, S, p)], 1ull);
}

struct InBuckets {
  const uint64_t *P, *S;
  uint32_t ba, bb;
  __device__ bool operator()(uint64_t p) const {
    const uint32_t b = bucket_of(P, S, p);
    return b >= ba && b < bb;
  }
};

__global__ void k_bucket_keys(const uint64_t *P, const uint64_t *S, const uint64_t *pos, uint64_t cnt,
                              uint32_t ba, uint32_t *key) {
  const uint64_t j = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (j < cnt) key[j] = bucket_of(P, S, pos[j]) - ba;
}

// after the bucket sort: group starts (hv for a max-scan), depth bounds,
// unresolved flags
__global__ void k_init_groups(const uint32_t *key, uint64_t cnt, uint32_t ba, uint32_t *hv,
                              uint32_t *dep, uint8_t *unres) {
  const uint64_t j = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (j >= cnt) return;
  const bool sp = bucket_special(key[j] + ba);
  const bool head = j == 0 || key[j] != key[j - 1] || sp;
  const bool nhead = j + 1 == cnt || key[j + 1] != key[j] || sp;
  hv[j] = head ? (uint32_t) j : 0u;
  dep[j] = 0;
  unres[j] = !(head && nhead);
}

__global__ void k_iota32(uint32_t *a, uint64_t n) {
  const uint64_t k = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (k < n) a[k] = (uint32_t) k;
}

// hu[k] = 1 where U[k] starts a new group (dense group ids by a sum scan)
__global__ void k_group_heads(const uint32_t *U, uint64_t mu, const uint32_t *grp, uint32_t *hu) {
  const uint64_t k = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (k < mu) hu[k] = (k == 0 || grp[U[k]] != grp[U[k - 1]]) ? 1u : 0u;
}

__global__ void k_round_keys64(const uint64_t *P, const uint64_t *S, const uint32_t *U, uint64_t mu,
                               const uint64_t *SA, const uint32_t *gid, uint64_t h, int ns,
                               uint64_t *key, uint64_t *val) {
  const uint64_t k = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (k >= mu) return;
  const uint64_t p = SA[U[k]];
  bool sp;
  const uint64_t code = esa_key3(P, S, p + h, ns, &sp);
  key[k] = ((uint64_t) (gid[k] - 1u) << (3 * ns)) | code;
  val[k] = p;
}

__global__ void k_round_apply64(const uint64_t *key, const uint64_t *val, const uint32_t *U,
                                uint64_t mu, int ns, uint32_t h32, uint64_t *SA, uint32_t *dep,
                                uint32_t *hv, uint8_t *unres) {
  const uint64_t k = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (k >= mu) return;
  const uint64_t cm = (3 * ns == 64) ? ~0ull : ((1ull << (3 * ns)) - 1);
  const uint64_t spm = 0x4924924924924924ull & cm & 0x7fffffffffffffffull;   // bit 2 of each field
  const uint32_t slot = U[k];
  SA[slot] = val[k];
  const uint64_t kk = key[k];
  const bool sp = (kk & spm & cm) != 0;
  const bool same_grp = k > 0 && (key[k - 1] >> (3 * ns)) == (kk >> (3 * ns));
  if (same_grp) dep[slot] = h32;                      // shared the group through depth h
  const bool head = k == 0 || key[k - 1] != kk || sp;
  bool nhead = true;
  if (k + 1 < mu) {
    const uint64_t kn = key[k + 1];
    nhead = kn != kk || (kn & spm & cm) != 0;
  }
  hv[k] = head ? slot : 0u;
  unres[k] = !(head && nhead);
}

__global__ void k_scatter_grp(const uint32_t *U, uint64_t mu, const uint32_t *g, uint32_t *grp) {
  const uint64_t k = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (k < mu) grp[U[k]] = g[k];
}

// rows of the batch: LCP (from the group depth), .lcp byte, .llv flag, BWT
// byte, suffix; only rows in [row_lo, row_hi) are written
__global__ void k_emit64(const uint64_t *P, const uint64_t *S, const uint64_t *SEP,
                         const uint64_t *SA, const uint32_t *dep, uint64_t cnt,
                         const uint64_t *prev, uint64_t r0, uint64_t row_lo, uint64_t row_hi,
                         uint8_t *lcptab, uint8_t *bwttab, uint64_t *suftab, uint8_t *big,
                         unsigned long long *sum, unsigned long long *maxv) {
  const uint64_t j = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  uint64_t v = 0;
  if (j < cnt) {
    const uint64_t r = r0 + j;
    big[j] = 0;
    if (r >= row_lo && r < row_hi) {
      const uint64_t s = SA[j];
      const uint64_t q = j == 0 ? *prev : SA[j - 1];
      v = (r == 0 || q == UINT64_MAX) ? 0 : esa_extend(P, S, q, s, j == 0 ? 0 : dep[j]);
      const uint64_t i = r - row_lo;
      lcptab[i] = v < 255 ? (uint8_t) v : 255;
      big[j] = v >= 255;
      uint8_t b = 254;
      if (s > 0) {
        const uint64_t t = s - 1;
        if ((S[t >> 6] >> (t & 63)) & 1u) b = ((SEP[t >> 6] >> (t & 63)) & 1u) ? 255 : 254;
        else b = (uint8_t) ((P[t >> 5] >> (2 * (t & 31))) & 3u);
      }
      bwttab[i] = b;
      if (suftab) suftab[i] = s;
    }
  }
  unsigned long long vs = v, vm = v;
  for (int d = 32; d >= 1; d >>= 1) {
    vs += __shfl_xor(vs, d, 64);
    const unsigned long long o = __shfl_xor(vm, d, 64);
    vm = o > vm ? o : vm;
  }
  if ((threadIdx.x & 63) == 0) {
    if (vs) atomicAdd(sum, vs);
    if (vm) atomicMax(maxv, vm);
  }
}

// .llv entries of the batch's flagged rows (j list): exact values again
__global__ void k_llv64(const uint64_t *P, const uint64_t *S, const uint64_t *SA, const uint32_t *dep,
                        const uint32_t *js, uint64_t nj, const uint64_t *prev, uint64_t r0,
                        GtSmaxLlv *out) {
  const uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (i >= nj) return;
  const uint64_t j = js[i];
  const uint64_t q = j == 0 ? *prev : SA[j - 1];
  out[i].position = r0 + j;
  out[i].value = esa_extend(P, S, q, SA[j], j == 0 ? 0 : dep[j]);
}

__global__ void k_last(const uint64_t *SA, uint64_t cnt, uint64_t *prev) { *prev = SA[cnt - 1]; }

// packed BWT groups of the local byte table (layout GT_SMAX_PK_GROUPS)
__global__ void k_pack_bwt64(const uint8_t *bwt, uint64_t len, uint64_t ngroups, uint64_t *pk) {
  const uint64_t gi = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (gi >= ngroups) return;
  const int64_t r0 = ((int64_t) gi - 1) * 16;
  uint64_t w = 0;
  for (int q = 0; q < 16; q++) {
    const int64_t r = r0 + q;
    if (r < 0 || (uint64_t) r >= len) continue;
    const uint32_t b = bwt[r];
    if (b >= 254) w |= 1ull << (32 + q);
    else w |= (uint64_t) (b & 1u) << q | (uint64_t) ((b >> 1) & 1u) << (16 + q);
  }
  pk[gi] = w;
}

struct Temp {
  void *p = nullptr;
  size_t bytes = 0;
  hipError_t ensure(size_t need) {
    if (need <= bytes) return hipSuccess;
    if (p) (void) hipFree(p);
    p = nullptr;
    bytes = 0;
    hipError_t e = hipMalloc(&p, need);
    if (e == hipSuccess) bytes = need;
    return e;
  }
  ~Temp() { if (p) (void) hipFree(p); }
};

template <typename T>
hipError_t dmalloc(T **p, uint64_t count) {
  return hipMalloc(reinterpret_cast<void **>(p), sizeof (T) * (count ? count : 1));
}

}  // namespace

extern "C" void gt_smax_esa64_release(GtSmaxEsa64Dev *e) {
  if (e == NULL) return;
  (void) hipSetDevice(e->device);
  if (e->lcptab_dev) gt_smax_dev_free_table(e->device, e->lcptab_dev);
  if (e->bwttab_dev) gt_smax_dev_free_table(e->device, e->bwttab_dev);
  if (e->bwtpk_dev) (void) hipFree(e->bwtpk_dev);
  if (e->llvtab_dev) (void) hipFree(e->llvtab_dev);
  if (e->suftab_dev) (void) hipFree(e->suftab_dev);
  e->lcptab_dev = e->bwttab_dev = NULL;
  e->bwtpk_dev = NULL;
  e->llvtab_dev = NULL;
  e->suftab_dev = NULL;
}

extern "C" int gt_smax_esa64_build(int device, const uint8_t *text, uint64_t n, uint64_t row_lo,
                                   uint64_t row_hi, int keep_suftab, uint64_t batch_max,
                                   GtSmaxEsa64Dev *out, char *errbuf, size_t errlen) {
  const uint64_t m = n + 1;
  const uint64_t nws = (n + 64 + 63) / 64 + 2;          // special/separator words, padded
  uint8_t *T = NULL, *flags = NULL, *big = NULL;
  uint64_t *P = NULL, *S = NULL, *SEP = NULL, *pos = NULL, *SA = NULL, *keyA = NULL, *keyB = NULL,
           *valA = NULL, *valB = NULL, *prev = NULL, *d64 = NULL;
  uint32_t *k32a = NULL, *k32b = NULL, *hv = NULL, *grp = NULL, *dep = NULL, *U = NULL, *U2 = NULL,
           *gid = NULL;
  unsigned long long *cnt_dev = NULL, *stat = NULL;
  GtSmaxLlv *llv_batch = NULL;
  std::vector<unsigned long long> cnt;
  std::vector<GtSmaxLlv> llv_host;
  Temp tmp;
  hipStream_t s = 0;
  uint64_t local = 0, bmax = 0;
  memset(out, 0, sizeof *out);
  out->device = device;
  if (row_hi == 0) row_hi = m;
  if (row_lo >= row_hi || row_hi > m) {
    seterr(errbuf, errlen, "bad row range [%lu, %lu) of %lu suffixes", (unsigned long) row_lo,
           (unsigned long) row_hi, (unsigned long) m);
    return -1;
  }
  local = row_hi - row_lo;
  gt_smax_release_cache();   // the smax runtime's cached buffers: room for the build
  HIPCHK(hipSetDevice(device));

  // ---- 1. packed text, special and separator bitmaps
  HIPCHK(dmalloc(&P, 2 * nws));
  HIPCHK(dmalloc(&S, nws));
  HIPCHK(dmalloc(&SEP, nws));
  HIPCHK(hipMemset(P, 0, sizeof (uint64_t) * 2 * nws));
  HIPCHK(hipMemset(S, 0xff, sizeof (uint64_t) * nws));
  HIPCHK(hipMemset(SEP, 0, sizeof (uint64_t) * nws));
  {
    const uint64_t CH = 256ull << 20;                  // bytes per upload (multiple of 64)
    HIPCHK(dmalloc(&T, CH));
    for (uint64_t off = 0; off < n; off += CH) {
      const uint64_t len = std::min(CH, n - off);
      HIPCHK(hipMemcpy(T, text + off, len, hipMemcpyHostToDevice));
      const uint64_t nw = (len + 63) / 64;
      hipLaunchKernelGGL(k_pack64, dim3(blocks(nw)), dim3(256), 0, s, T, off / 64, nw, n, P, S, SEP);
      HIPCHK(hipGetLastError());
    }
    HIPCHK(hipDeviceSynchronize());
    (void) hipFree(T);
    T = NULL;
  }
  HIPCHK(dmalloc(&stat, 4));
  HIPCHK(hipMemset(stat, 0, sizeof (unsigned long long) * 4));
  hipLaunchKernelGGL(k_count_specials, dim3(blocks(nws)), dim3(256), 0, s, S, n, stat);
  {
    unsigned long long nsp = 0;
    HIPCHK(hipMemcpy(&nsp, stat, sizeof nsp, hipMemcpyDeviceToHost));
    out->totallength = n;
    out->nonspecials = n - nsp;
  }
  HIPCHK(hipMemset(stat, 0, sizeof (unsigned long long) * 4));

  // ---- 2. bucket histogram -> first row of every bucket (host)
  HIPCHK(dmalloc(&cnt_dev, kNB));
  HIPCHK(hipMemset(cnt_dev, 0, sizeof (unsigned long long) * kNB));
  hipLaunchKernelGGL(k_bucket_count, dim3(blocks(m)), dim3(256), 0, s, P, S, m, cnt_dev);
  HIPCHK(hipGetLastError());
  cnt.resize(kNB);
  HIPCHK(hipMemcpy(cnt.data(), cnt_dev, sizeof (unsigned long long) * kNB, hipMemcpyDeviceToHost));
  {
    // every suffix counted once: the batches' buffers are sized from these
    unsigned long long tot = 0;
    for (unsigned long long c : cnt) tot += c;
    if (tot != m) {
      seterr(errbuf, errlen, "bucket histogram counts %llu suffixes, expected %lu", tot,
             (unsigned long) m);
      goto fail;
    }
  }
  (void) hipFree(cnt_dev);
  cnt_dev = NULL;

  // ---- outputs (local rows [row_lo, row_hi))
  if (gt_smax_dev_alloc_table(device, local, &out->lcptab_dev, errbuf, errlen)) goto fail;
  if (gt_smax_dev_alloc_table(device, local, &out->bwttab_dev, errbuf, errlen)) goto fail;
  HIPCHK(dmalloc(&out->bwtpk_dev, GT_SMAX_PK_GROUPS(local)));
  if (keep_suftab) HIPCHK(dmalloc(&out->suftab_dev, local));
  out->row_lo = row_lo;
  out->row_hi = row_hi;

  {
    // batch size: what the free HBM allows (about 80 B per suffix of a batch)
    size_t fr = 0, tot = 0;
    HIPCHK(hipMemGetInfo(&fr, &tot));
    bmax = fr > (8ull << 30) ? (fr - (8ull << 30)) / 96 : (1ull << 20);
    bmax = std::min<uint64_t>(bmax, 0x7fffffffull);
    if (batch_max) bmax = std::min(bmax, batch_max);
    // first needed row: row_lo - 1 (the predecessor of LCP[row_lo])
    const uint64_t need_lo = row_lo > 0 ? row_lo - 1 : 0;
    uint64_t start = 0, maxb = 0;
    uint32_t b = 0;
    while (b < kNB && start + cnt[b] <= need_lo) start += cnt[b++];   // first bucket with a needed row
    // batches over the buckets up to the one holding row_hi - 1
    std::vector<uint32_t> bs;
    std::vector<uint64_t> br;
    uint64_t acc = 0;
    bs.push_back(b);
    br.push_back(start);
    for (uint32_t c = b; c < kNB && start < row_hi; c++) {
      if (cnt[c] > bmax) {
        seterr(errbuf, errlen, "bucket of %llu suffixes exceeds the batch limit %lu", cnt[c],
               (unsigned long) bmax);
        goto fail;
      }
      if (acc + cnt[c] > bmax) {
        bs.push_back(c);
        br.push_back(start);
        acc = 0;
      }
      acc += cnt[c];
      start += cnt[c];
      maxb = std::max(maxb, acc);
      if (start >= row_hi || c + 1 == kNB) { bs.push_back(c + 1); br.push_back(start); break; }
    }
    out->batches = (int) bs.size() - 1;
    // per-batch buffers, sized for the largest batch
    const uint64_t B = maxb;
    HIPCHK(dmalloc(&pos, B));
    HIPCHK(dmalloc(&SA, B));
    HIPCHK(dmalloc(&k32a, B));
    HIPCHK(dmalloc(&k32b, B));
    HIPCHK(dmalloc(&hv, B));
    HIPCHK(dmalloc(&grp, B));
    HIPCHK(dmalloc(&dep, B));
    HIPCHK(dmalloc(&U, B));
    HIPCHK(dmalloc(&U2, B));
    HIPCHK(dmalloc(&gid, B));
    HIPCHK(dmalloc(&keyA, B));
    HIPCHK(dmalloc(&keyB, B));
    HIPCHK(dmalloc(&valA, B));
    HIPCHK(dmalloc(&valB, B));
    HIPCHK(dmalloc(&flags, B));
    HIPCHK(dmalloc(&big, B));
    HIPCHK(dmalloc(&prev, 1));
    HIPCHK(dmalloc(&d64, 2));
    {
      const uint64_t none = UINT64_MAX;
      HIPCHK(hipMemcpy(prev, &none, sizeof none, hipMemcpyHostToDevice));
    }
    int rounds_max = 0;
    for (size_t bi = 0; bi + 1 < bs.size(); bi++) {
      const uint32_t ba = bs[bi], bb = bs[bi + 1];
      const uint64_t r0 = br[bi], want = br[bi + 1] - br[bi];
      if (want == 0) continue;
      // 3a. positions of the batch's buckets, position order
      uint64_t got = 0;
      for (uint64_t c0 = 0; c0 < m; c0 += kChunk) {
        const uint64_t len = std::min(kChunk, m - c0);
        InBuckets pred{P, S, ba, bb};
        size_t need = 0;
        rocprim::counting_iterator<uint64_t> it(c0);
        HIPCHK(rocprim::select(nullptr, need, it, pos + got, d64, len, pred, s));
        HIPCHK(tmp.ensure(need));
        HIPCHK(rocprim::select(tmp.p, need, it, pos + got, d64, len, pred, s));
        uint64_t c = 0;
        HIPCHK(hipMemcpy(&c, d64, sizeof c, hipMemcpyDeviceToHost));
        got += c;
        if (got > want) break;
      }
      if (got != want) {
        seterr(errbuf, errlen, "bucket batch collected %lu suffixes, expected %lu",
               (unsigned long) got, (unsigned long) want);
        goto fail;
      }
      // 3b. stable radix sort by bucket
      hipLaunchKernelGGL(k_bucket_keys, dim3(blocks(got)), dim3(256), 0, s, P, S, pos, got, ba, k32a);
      HIPCHK(hipGetLastError());
      {
        const unsigned bits = 32 - __builtin_clz(std::max<uint32_t>(bb - ba, 2) - 1);
        rocprim::double_buffer<uint32_t> kb(k32a, k32b);
        rocprim::double_buffer<uint64_t> vb(pos, SA);
        size_t need = 0;
        HIPCHK(rocprim::radix_sort_pairs(nullptr, need, kb, vb, got, 0, bits, s));
        HIPCHK(tmp.ensure(need));
        HIPCHK(rocprim::radix_sort_pairs(tmp.p, need, kb, vb, got, 0, bits, s));
        if (vb.current() != SA) {
          HIPCHK(hipMemcpyAsync(SA, vb.current(), sizeof (uint64_t) * got, hipMemcpyDeviceToDevice, s));
        }
        if (kb.current() != k32a) {
          HIPCHK(hipMemcpyAsync(k32a, kb.current(), sizeof (uint32_t) * got, hipMemcpyDeviceToDevice, s));
        }
      }
      hipLaunchKernelGGL(k_init_groups, dim3(blocks(got)), dim3(256), 0, s, k32a, got, ba, hv, dep, flags);
      HIPCHK(hipGetLastError());
      uint64_t mu = 0;
      {
        size_t need = 0;
        HIPCHK(rocprim::inclusive_scan(nullptr, need, hv, grp, got, rocprim::maximum<uint32_t>(), s));
        HIPCHK(tmp.ensure(need));
        HIPCHK(rocprim::inclusive_scan(tmp.p, need, hv, grp, got, rocprim::maximum<uint32_t>(), s));
        hipLaunchKernelGGL(k_iota32, dim3(blocks(got)), dim3(256), 0, s, k32b, got);
        need = 0;
        HIPCHK(rocprim::select(nullptr, need, k32b, flags, U, d64, got, s));
        HIPCHK(tmp.ensure(need));
        HIPCHK(rocprim::select(tmp.p, need, k32b, flags, U, d64, got, s));
        HIPCHK(hipMemcpy(&mu, d64, sizeof mu, hipMemcpyDeviceToHost));
      }
      // 3c. refinement rounds
      uint64_t h = kB;
      int rounds = 0;
      while (mu > 0) {
        rounds++;
        if (h > m + 64) {
          seterr(errbuf, errlen, "suffix sorting did not converge");
          goto fail;
        }
        hipLaunchKernelGGL(k_group_heads, dim3(blocks(mu)), dim3(256), 0, s, U, mu, grp, hv);
        uint32_t ngroups = 0;
        {
          size_t need = 0;
          HIPCHK(rocprim::inclusive_scan(nullptr, need, hv, gid, mu, rocprim::plus<uint32_t>(), s));
          HIPCHK(tmp.ensure(need));
          HIPCHK(rocprim::inclusive_scan(tmp.p, need, hv, gid, mu, rocprim::plus<uint32_t>(), s));
          HIPCHK(hipMemcpy(&ngroups, gid + mu - 1, sizeof ngroups, hipMemcpyDeviceToHost));
        }
        const unsigned gbits = ngroups > 1 ? 32 - __builtin_clz(ngroups - 1) : 0;
        const int ns = (int) std::min<unsigned>(21, (64 - gbits) / 3);
        hipLaunchKernelGGL(k_round_keys64, dim3(blocks(mu)), dim3(256), 0, s, P, S, U, mu, SA, gid, h,
                           ns, keyA, valA);
        HIPCHK(hipGetLastError());
        {
          rocprim::double_buffer<uint64_t> kb(keyA, keyB);
          rocprim::double_buffer<uint64_t> vb(valA, valB);
          size_t need = 0;
          const unsigned endbit = gbits + 3 * (unsigned) ns;
          HIPCHK(rocprim::radix_sort_pairs(nullptr, need, kb, vb, mu, 0, endbit, s));
          HIPCHK(tmp.ensure(need));
          HIPCHK(rocprim::radix_sort_pairs(tmp.p, need, kb, vb, mu, 0, endbit, s));
          const uint32_t h32 = (uint32_t) std::min<uint64_t>(h, 0xffffffffull);
          hipLaunchKernelGGL(k_round_apply64, dim3(blocks(mu)), dim3(256), 0, s, kb.current(),
                             vb.current(), U, mu, ns, h32, SA, dep, hv, flags);
          HIPCHK(hipGetLastError());
        }
        {
          // group starts of the new groups (slots ascend with k: a max-scan)
          size_t need = 0;
          HIPCHK(rocprim::inclusive_scan(nullptr, need, hv, gid, mu, rocprim::maximum<uint32_t>(), s));
          HIPCHK(tmp.ensure(need));
          HIPCHK(rocprim::inclusive_scan(tmp.p, need, hv, gid, mu, rocprim::maximum<uint32_t>(), s));
          hipLaunchKernelGGL(k_scatter_grp, dim3(blocks(mu)), dim3(256), 0, s, U, mu, gid, grp);
          need = 0;
          HIPCHK(rocprim::select(nullptr, need, U, flags, U2, d64, mu, s));
          HIPCHK(tmp.ensure(need));
          HIPCHK(rocprim::select(tmp.p, need, U, flags, U2, d64, mu, s));
          HIPCHK(hipMemcpy(&mu, d64, sizeof mu, hipMemcpyDeviceToHost));
          std::swap(U, U2);
        }
        h += (uint64_t) ns;
      }
      rounds_max = std::max(rounds_max, rounds);
      if (getenv("GT_SMAX_VERBOSE"))
        fprintf(stderr, "gt_smax_esa64: batch %zu/%zu: %lu suffixes, %d rounds (depth %lu)\n",
                bi + 1, bs.size() - 1, (unsigned long) got, rounds, (unsigned long) h);
      // 4. rows
      hipLaunchKernelGGL(k_emit64, dim3(blocks(got)), dim3(256), 0, s, P, S, SEP, SA, dep, got, prev, r0,
                         row_lo, row_hi, out->lcptab_dev, out->bwttab_dev, out->suftab_dev, big,
                         stat, stat + 1);
      HIPCHK(hipGetLastError());
      {
        hipLaunchKernelGGL(k_iota32, dim3(blocks(got)), dim3(256), 0, s, k32b, got);
        size_t need = 0;
        uint64_t nj = 0;
        HIPCHK(rocprim::select(nullptr, need, k32b, big, k32a, d64, got, s));
        HIPCHK(tmp.ensure(need));
        HIPCHK(rocprim::select(tmp.p, need, k32b, big, k32a, d64, got, s));
        HIPCHK(hipMemcpy(&nj, d64, sizeof nj, hipMemcpyDeviceToHost));
        if (nj > 0) {
          HIPCHK(dmalloc(&llv_batch, nj));
          hipLaunchKernelGGL(k_llv64, dim3(blocks(nj)), dim3(256), 0, s, P, S, SA, dep, k32a, nj, prev,
                             r0, llv_batch);
          HIPCHK(hipGetLastError());
          const size_t o = llv_host.size();
          llv_host.resize(o + nj);
          HIPCHK(hipMemcpy(llv_host.data() + o, llv_batch, sizeof (GtSmaxLlv) * nj,
                           hipMemcpyDeviceToHost));
          (void) hipFree(llv_batch);
          llv_batch = NULL;
        }
      }
      hipLaunchKernelGGL(k_last, dim3(1), dim3(1), 0, s, SA, got, prev);
      HIPCHK(hipGetLastError());
    }
    out->sort_rounds = rounds_max;
  }
  {
    unsigned long long st[2] = {0, 0};
    HIPCHK(hipMemcpy(st, stat, sizeof st, hipMemcpyDeviceToHost));
    out->averagelcp = (double) st[0] / (double) local;
    out->maxbranchdepth = st[1];
  }
  hipLaunchKernelGGL(k_pack_bwt64, dim3(blocks(GT_SMAX_PK_GROUPS(local))), dim3(256), 0, s,
                     out->bwttab_dev, local, (uint64_t) GT_SMAX_PK_GROUPS(local), out->bwtpk_dev);
  HIPCHK(hipGetLastError());
  out->numllv = llv_host.size();
  HIPCHK(dmalloc(&out->llvtab_dev, out->numllv + 1));
  if (out->numllv)
    HIPCHK(hipMemcpy(out->llvtab_dev, llv_host.data(), sizeof (GtSmaxLlv) * out->numllv,
                     hipMemcpyHostToDevice));
  HIPCHK(hipDeviceSynchronize());
  {
    void *f[] = {P, S, SEP, pos, SA, k32a, k32b, hv, grp, dep, U, U2, gid, keyA, keyB, valA, valB,
                 flags, big, prev, d64, stat};
    for (void *x : f)
      if (x) (void) hipFree(x);
  }
  return 0;
fail:
  {
    void *f[] = {T, P, S, SEP, pos, SA, k32a, k32b, hv, grp, dep, U, U2, gid, keyA, keyB, valA, valB,
                 flags, big, prev, d64, stat, cnt_dev, llv_batch};
    for (void *x : f)
      if (x) (void) hipFree(x);
  }
  gt_smax_esa64_release(out);
  return -1;
}

extern "C" int gt_smax_esa64_download(const GtSmaxEsa64Dev *e, uint8_t *lcptab, uint8_t *bwttab,
                                      GtSmaxLlv *llvtab, uint64_t *suftab, uint64_t *bwtpk,
                                      char *errbuf, size_t errlen) {
  const uint64_t L = e->row_hi - e->row_lo;
  HIPCHK(hipSetDevice(e->device));
  if (lcptab) HIPCHK(hipMemcpy(lcptab, e->lcptab_dev, L, hipMemcpyDeviceToHost));
  if (bwttab) HIPCHK(hipMemcpy(bwttab, e->bwttab_dev, L, hipMemcpyDeviceToHost));
  if (llvtab && e->numllv)
    HIPCHK(hipMemcpy(llvtab, e->llvtab_dev, sizeof (GtSmaxLlv) * e->numllv, hipMemcpyDeviceToHost));
  if (bwtpk)
    HIPCHK(hipMemcpy(bwtpk, e->bwtpk_dev, sizeof (uint64_t) * GT_SMAX_PK_GROUPS(L),
                     hipMemcpyDeviceToHost));
  if (suftab) {
    if (e->suftab_dev == NULL) {
      seterr(errbuf, errlen, "suftab was not kept on the device");
      return -1;
    }
    HIPCHK(hipMemcpy(suftab, e->suftab_dev, sizeof (uint64_t) * L, hipMemcpyDeviceToHost));
  }
  return 0;
fail:
  return -1;
}
