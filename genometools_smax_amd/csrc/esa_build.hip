// esa_build.hip -- GPU construction of a GenomeTools enhanced suffix array
// (the `gt suffixerator -suf -lcp -bwt` producer of the smax inputs;
// SURVEY.md §8(f) row F1), for texts with n+1 < 2^32 suffixes.
//
// Output layout is byte-identical to suffixerator (checked against the
// oracle, which reproduces the reference's golden repfind output):
//   suftab  suffix order with special symbols (WILDCARD 254, SEPARATOR 255,
//           end of text) unique and ranked by position above every base
//   lcptab  u8, values >= 255 stored as 255 + {position,value} in llvtab
//           (src/match/sfx-lcpvalues.c:371-470)
//   bwttab  254 for suftab[k]==0, else text[suftab[k]-1]
//           (src/match/sfx-run.c:174-212)
//
// Algorithm (MI355X-first, not the reference's bucket sort):
//   1. 2-bit packed text + special bitmap in HBM;
//   2. 63-bit keys = first 21 symbols at 3 bits (a special becomes 4 and
//      ends the key), one rocPRIM radix sort of (key, position) pairs --
//      stable, so suffixes ending in the same special run stay position
//      ordered;
//   3. prefix doubling (Manber-Myers with group-start ranks) on the still
//      unresolved groups only: keys (rank[i], rank[i+h]) radix-sorted,
//      scattered back into the group's SA slots;
//   4. Phi array + chunked Kasai (PLCP[i] >= PLCP[i-1]-1 within a chunk),
//      comparing 32 symbols per step on the packed text;
//   5. gathers for LCP (by SA) and BWT -- bytes and the packed bit planes
//      the smax scan streams -- and stream compaction for .llv.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gt_smax_hip.h"
#include "gt_smax_esa.h"

namespace {

constexpr int kKeyChars = 21;
constexpr uint64_t kSpecialMask = 0x4924924924924924ull;  // bit 2 of each 3-bit field (21 fields)
constexpr uint32_t kNone = 0xffffffffu;

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

inline unsigned blocks_for(uint64_t n, unsigned t = 256) {
  uint64_t b = (n + t - 1) / t;
  return (unsigned) (b > 0x7fffffffull ? 0x7fffffffull : (b ? b : 1));
}

// ------------------------------------------------------------ kernels

// P: 32 symbols per word (2 bits, symbol k at bits 2k..2k+1), specials 0;
// S: bit p set iff position p is special or p >= n.
__global__ void k_pack(const uint8_t *T, uint64_t n, uint64_t nwords_s,
                       uint64_t *P, uint64_t *S) {
  uint64_t w = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (w >= nwords_s) return;
  uint64_t base = w * 64, s = 0, p0 = 0, p1 = 0;
  for (int k = 0; k < 64; k++) {
    uint64_t p = base + k;
    uint32_t c = p < n ? T[p] : 255u;
    uint64_t sym = 0;
    if (c >= 254) s |= 1ull << k;
    else sym = c & 3;
    if (k < 32) p0 |= sym << (2 * k); else p1 |= sym << (2 * (k - 32));
  }
  S[w] = s;
  P[2 * w] = p0;
  P[2 * w + 1] = p1;
}

__device__ __forceinline__ uint64_t sym32(const uint64_t *P, uint64_t a) {
  uint64_t w = a >> 5;
  unsigned sh = (unsigned) (a & 31) * 2;
  uint64_t v = P[w] >> sh;
  if (sh) v |= P[w + 1] << (64 - sh);
  return v;
}
__device__ __forceinline__ uint32_t spec32(const uint64_t *S, uint64_t a) {
  uint64_t w = a >> 6;
  unsigned sh = (unsigned) (a & 63);
  uint64_t v = S[w] >> sh;
  if (sh) v |= S[w + 1] << (64 - sh);
  return (uint32_t) v;
}

__global__ void k_init_keys(const uint64_t *P, const uint64_t *S, uint64_t m,
                            uint64_t *key, uint32_t *val) {
  uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (i >= m) return;
  uint64_t sy = sym32(P, i);
  uint32_t sp = spec32(S, i) & ((1u << kKeyChars) - 1);
  int first = sp ? __builtin_ctz(sp) : kKeyChars;
  uint64_t k = 0;
  for (int c = 0; c < kKeyChars; c++) {
    uint64_t code = c < first ? ((sy >> (2 * c)) & 3) : (c == first ? 4 : 0);
    k = (k << 3) | code;
  }
  key[i] = k;
  val[i] = (uint32_t) i;
}

// hv[k] = k if k starts a group of the sorted keys, else 0 (for a max-scan)
__global__ void k_heads(const uint64_t *key, uint64_t m, bool split_specials,
                        uint32_t *hv) {
  uint64_t k = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (k >= m) return;
  bool head = k == 0 || key[k] != key[k - 1] ||
              (split_specials && (key[k] & kSpecialMask));
  hv[k] = head ? (uint32_t) k : 0;
}

// initial pass: ISA from group starts, unresolved flags
__global__ void k_init_apply(const uint64_t *key, const uint32_t *SA,
                             const uint32_t *gs, uint64_t m, uint32_t *ISA,
                             uint8_t *unres) {
  uint64_t k = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (k >= m) return;
  ISA[SA[k]] = gs[k];
  bool head = k == 0 || key[k] != key[k - 1] || (key[k] & kSpecialMask);
  bool nexthead = k + 1 == m || key[k + 1] != key[k] || (key[k + 1] & kSpecialMask);
  unres[k] = !(head && nexthead);
}

__global__ void k_iota(uint32_t *a, uint64_t m) {
  uint64_t k = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (k < m) a[k] = (uint32_t) k;
}

__global__ void k_round_keys(const uint32_t *U, uint64_t mu, const uint32_t *SA,
                             const uint32_t *ISA, uint64_t h, uint64_t *key,
                             uint32_t *val) {
  uint64_t j = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (j >= mu) return;
  uint32_t i = SA[U[j]];
  key[j] = ((uint64_t) ISA[i] << 32) | ISA[(uint64_t) i + h];
  val[j] = i;
}

__global__ void k_round_apply(const uint64_t *key, const uint32_t *val,
                              const uint32_t *gs, const uint32_t *U, uint64_t mu,
                              uint32_t *SA, uint32_t *ISA, uint8_t *unres) {
  uint64_t j = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (j >= mu) return;
  uint32_t k = U[j];
  SA[k] = val[j];
  ISA[val[j]] = U[gs[j]];
  bool head = j == 0 || key[j] != key[j - 1];
  bool nexthead = j + 1 == mu || key[j + 1] != key[j];
  unres[j] = !(head && nexthead);
}

__global__ void k_phi(const uint32_t *SA, uint64_t m, uint32_t *phi) {
  uint64_t k = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (k >= m) return;
  phi[SA[k]] = k == 0 ? kNone : SA[k - 1];
}

__device__ uint64_t extend(const uint64_t *P, const uint64_t *S, uint64_t a,
                           uint64_t b, uint64_t h) {
  for (;;) {
    uint64_t x = sym32(P, a + h) ^ sym32(P, b + h);
    uint32_t sp = spec32(S, a + h) | spec32(S, b + h);
    uint32_t d1 = x ? (uint32_t) (__builtin_ctzll(x) >> 1) : 32u;
    uint32_t d2 = sp ? (uint32_t) __builtin_ctz(sp) : 32u;
    uint32_t d = d1 < d2 ? d1 : d2;
    h += d;
    if (d < 32) return h;
  }
}

__global__ void k_plcp(const uint64_t *P, const uint64_t *S, const uint32_t *phi,
                       uint64_t m, uint64_t chunk, uint32_t *plcp) {
  uint64_t c = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  uint64_t lo = c * chunk;
  if (lo >= m) return;
  uint64_t hi = lo + chunk < m ? lo + chunk : m;
  uint64_t h = 0;
  for (uint64_t i = lo; i < hi; i++) {
    uint32_t j = phi[i];
    if (j == kNone) { plcp[i] = 0; h = 0; continue; }
    h = extend(P, S, i, j, h);
    plcp[i] = (uint32_t) h;
    if (h > 0) h--;
  }
}

// LCP bytes, .llv flags, BWT bytes and the packed BWT (bit planes, layout of
// GT_SMAX_PK_GROUPS in include/gt_smax_hip.h: group k/16 + 1 holds row k)
// from three wave ballots -- 16 consecutive lanes are one group's rows
__global__ void k_finish(const uint32_t *SA, const uint32_t *plcp, const uint8_t *T,
                         uint64_t m, uint8_t *lcptab, uint8_t *bwttab, uint64_t *bwtpk,
                         uint8_t *bigflag, unsigned long long *sum,
                         unsigned int *maxv) {
  uint64_t k = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  uint64_t v = 0;
  uint32_t b = 0;
  if (k < m) {
    uint32_t s = SA[k];
    v = k == 0 ? 0 : plcp[s];
    lcptab[k] = v < 255 ? (uint8_t) v : 255;
    bigflag[k] = v >= 255;
    b = s == 0 ? 254 : T[s - 1];
    bwttab[k] = (uint8_t) b;
  }
  {
    const bool sp = k < m && b >= 254;
    const uint64_t m0 = __ballot(!sp && (b & 1u)), m1 = __ballot(!sp && (b & 2u)), ms = __ballot(sp);
    const uint32_t lane = threadIdx.x & 63;
    if ((lane & 15) == 0)
      bwtpk[k / 16 + 1] = ((m0 >> lane) & 0xffffull) | (((m1 >> lane) & 0xffffull) << 16) |
                          (((ms >> lane) & 0xffffull) << 32);
  }
  // block reductions for averagelcp / maxbranchdepth (.prj)
  __shared__ unsigned long long ssum[256];
  __shared__ unsigned int smax[256];
  ssum[threadIdx.x] = v;
  smax[threadIdx.x] = (unsigned int) v;
  __syncthreads();
  for (int d = 128; d > 0; d >>= 1) {
    if ((int) threadIdx.x < d) {
      ssum[threadIdx.x] += ssum[threadIdx.x + d];
      unsigned int o = smax[threadIdx.x + d];
      if (o > smax[threadIdx.x]) smax[threadIdx.x] = o;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    atomicAdd(sum, ssum[0]);
    atomicMax(maxv, smax[0]);
  }
}

__global__ void k_llv(const uint32_t *pos, uint64_t cnt, const uint32_t *SA,
                      const uint32_t *plcp, GtSmaxLlv *llv) {
  uint64_t j = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (j >= cnt) return;
  uint32_t k = pos[j];
  llv[j].position = k;
  llv[j].value = plcp[SA[k]];
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

}  // namespace

extern "C" void gt_smax_esa_release(GtSmaxEsaDev *e) {
  if (e == NULL) return;
  (void) hipSetDevice(e->device);
  if (e->lcptab_dev) gt_smax_dev_free_table(e->device, e->lcptab_dev);
  if (e->bwttab_dev) gt_smax_dev_free_table(e->device, e->bwttab_dev);
  if (e->llvtab_dev) (void) hipFree(e->llvtab_dev);
  if (e->suftab_dev) (void) hipFree(e->suftab_dev);
  if (e->bwtpk_dev) (void) hipFree(e->bwtpk_dev);
  e->bwtpk_dev = NULL;
  e->lcptab_dev = e->bwttab_dev = NULL;
  e->llvtab_dev = NULL;
  e->suftab_dev = NULL;
}

extern "C" int gt_smax_esa_build(int device, const uint8_t *text, uint64_t n,
                                 int keep_suftab, GtSmaxEsaDev *out,
                                 char *errbuf, size_t errlen) {
  const uint64_t m = n + 1;
  const uint64_t nws = (n + 64 + 63) / 64 + 2;     // special words, padded
  uint8_t *T = NULL, *unres = NULL, *bigflag = NULL;
  uint64_t *P = NULL, *S = NULL, *keyA = NULL, *keyB = NULL;
  uint32_t *SA = NULL, *ISA = NULL, *valA = NULL, *valB = NULL, *U = NULL,
           *U2 = NULL, *gs = NULL, *hv = NULL, *cntd = NULL, *llvpos = NULL;
  unsigned long long *sumd = NULL;
  unsigned int *maxd = NULL;
  uint64_t mu = 0, h = kKeyChars, numllv = 0, nspecial = 0;
  hipStream_t s = 0;
  Temp tmp;
  int rounds = 0;
  memset(out, 0, sizeof *out);
  out->device = device;
  gt_smax_release_cache();   // the smax runtime's cached buffers: room for the build
  if (m >= 0xffffffffull) {
    seterr(errbuf, errlen, "text of %lu symbols exceeds the 32-bit suffix array "
           "path (n+1 < 2^32)", (unsigned long) n);
    return -1;
  }
  for (uint64_t i = 0; i < n; i++) nspecial += text[i] >= 254;
  HIPCHK(hipSetDevice(device));
  HIPCHK(hipMalloc(&T, n + 64));
  HIPCHK(hipMemcpy(T, text, n, hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&P, sizeof (uint64_t) * 2 * nws));
  HIPCHK(hipMalloc(&S, sizeof (uint64_t) * nws));
  hipLaunchKernelGGL(k_pack, dim3(blocks_for(nws)), dim3(256), 0, s, T, n, nws, P, S);
  HIPCHK(hipGetLastError());

  // ---- initial 21-symbol sort
  HIPCHK(hipMalloc(&keyA, sizeof (uint64_t) * m));
  HIPCHK(hipMalloc(&keyB, sizeof (uint64_t) * m));
  HIPCHK(hipMalloc(&valA, sizeof (uint32_t) * m));
  HIPCHK(hipMalloc(&valB, sizeof (uint32_t) * m));
  hipLaunchKernelGGL(k_init_keys, dim3(blocks_for(m)), dim3(256), 0, s, P, S, m, keyA, valA);
  HIPCHK(hipGetLastError());
  {
    rocprim::double_buffer<uint64_t> kb(keyA, keyB);
    rocprim::double_buffer<uint32_t> vb(valA, valB);
    size_t need = 0;
    HIPCHK(rocprim::radix_sort_pairs(nullptr, need, kb, vb, m, 0, 3 * kKeyChars, s));
    HIPCHK(tmp.ensure(need));
    HIPCHK(rocprim::radix_sort_pairs(tmp.p, need, kb, vb, m, 0, 3 * kKeyChars, s));
    if (kb.current() != keyA) { uint64_t *t = keyA; keyA = keyB; keyB = t; }
    if (vb.current() != valA) { uint32_t *t = valA; valA = valB; valB = t; }
  }
  // sorted keys in keyA, positions in valA -> SA
  SA = valA;
  valA = NULL;
  HIPCHK(hipMalloc(&ISA, sizeof (uint32_t) * (m + 64)));
  HIPCHK(hipMalloc(&gs, sizeof (uint32_t) * m));
  HIPCHK(hipMalloc(&hv, sizeof (uint32_t) * m));
  HIPCHK(hipMalloc(&unres, m));
  HIPCHK(hipMalloc(&U, sizeof (uint32_t) * m));
  HIPCHK(hipMalloc(&U2, sizeof (uint32_t) * m));
  HIPCHK(hipMalloc(&cntd, sizeof (uint32_t) * 2));
  hipLaunchKernelGGL(k_heads, dim3(blocks_for(m)), dim3(256), 0, s, keyA, m, true, hv);
  {
    size_t need = 0;
    HIPCHK(rocprim::inclusive_scan(nullptr, need, hv, gs, m, rocprim::maximum<uint32_t>(), s));
    HIPCHK(tmp.ensure(need));
    HIPCHK(rocprim::inclusive_scan(tmp.p, need, hv, gs, m, rocprim::maximum<uint32_t>(), s));
  }
  hipLaunchKernelGGL(k_init_apply, dim3(blocks_for(m)), dim3(256), 0, s, keyA, SA, gs, m,
                     ISA, unres);
  HIPCHK(hipGetLastError());
  {
    // U = SA slots of unresolved groups, ascending
    hipLaunchKernelGGL(k_iota, dim3(blocks_for(m)), dim3(256), 0, s, hv, m);
    size_t need = 0;
    HIPCHK(rocprim::select(nullptr, need, hv, unres, U, cntd, m, s));
    HIPCHK(tmp.ensure(need));
    HIPCHK(rocprim::select(tmp.p, need, hv, unres, U, cntd, m, s));
    uint32_t c32 = 0;
    HIPCHK(hipMemcpy(&c32, cntd, sizeof c32, hipMemcpyDeviceToHost));
    mu = c32;
  }

  // ---- prefix doubling on unresolved groups
  while (mu > 0) {
    rounds++;
    if (h >= m) {
      seterr(errbuf, errlen, "suffix sorting did not converge");
      goto fail;
    }
    hipLaunchKernelGGL(k_round_keys, dim3(blocks_for(mu)), dim3(256), 0, s, U, mu, SA, ISA, h,
                       keyA, valB);
    HIPCHK(hipGetLastError());
    {
      rocprim::double_buffer<uint64_t> kb(keyA, keyB);
      rocprim::double_buffer<uint32_t> vb(valB, hv);
      size_t need = 0;
      HIPCHK(rocprim::radix_sort_pairs(nullptr, need, kb, vb, mu, 0, 64, s));
      HIPCHK(tmp.ensure(need));
      HIPCHK(rocprim::radix_sort_pairs(tmp.p, need, kb, vb, mu, 0, 64, s));
      uint64_t *ks = kb.current();
      uint32_t *vs = vb.current();
      uint32_t *hv2 = (vs == hv) ? valB : hv;   // free u32 buffer for head values
      hipLaunchKernelGGL(k_heads, dim3(blocks_for(mu)), dim3(256), 0, s, ks, mu, false, hv2);
      need = 0;
      HIPCHK(rocprim::inclusive_scan(nullptr, need, hv2, gs, mu, rocprim::maximum<uint32_t>(), s));
      HIPCHK(tmp.ensure(need));
      HIPCHK(rocprim::inclusive_scan(tmp.p, need, hv2, gs, mu, rocprim::maximum<uint32_t>(), s));
      hipLaunchKernelGGL(k_round_apply, dim3(blocks_for(mu)), dim3(256), 0, s, ks, vs, gs, U, mu,
                         SA, ISA, unres);
      HIPCHK(hipGetLastError());
      need = 0;
      HIPCHK(rocprim::select(nullptr, need, U, unres, U2, cntd, mu, s));
      HIPCHK(tmp.ensure(need));
      HIPCHK(rocprim::select(tmp.p, need, U, unres, U2, cntd, mu, s));
      uint32_t c32 = 0;
      HIPCHK(hipMemcpy(&c32, cntd, sizeof c32, hipMemcpyDeviceToHost));
      mu = c32;
      uint32_t *t = U; U = U2; U2 = t;
    }
    h *= 2;
  }
  (void) hipFree(U); U = NULL;
  (void) hipFree(U2); U2 = NULL;
  (void) hipFree(gs); gs = NULL;
  (void) hipFree(unres); unres = NULL;
  (void) hipFree(keyB); keyB = NULL;

  // ---- LCP via Phi + chunked Kasai (phi in ISA's storage, plcp in keyA's)
  {
    uint32_t *phi = ISA;
    uint32_t *plcp = (uint32_t *) keyA;
    const uint64_t chunk = 512;
    hipLaunchKernelGGL(k_phi, dim3(blocks_for(m)), dim3(256), 0, s, SA, m, phi);
    hipLaunchKernelGGL(k_plcp, dim3(blocks_for((m + chunk - 1) / chunk)), dim3(256), 0, s,
                       P, S, phi, m, chunk, plcp);
    HIPCHK(hipGetLastError());
    if (gt_smax_dev_alloc_table(device, m, &out->lcptab_dev, errbuf, errlen)) goto fail;
    if (gt_smax_dev_alloc_table(device, m, &out->bwttab_dev, errbuf, errlen)) goto fail;
    HIPCHK(hipMalloc(&out->bwtpk_dev, sizeof (uint64_t) * GT_SMAX_PK_GROUPS(m)));
    HIPCHK(hipMemsetAsync(out->bwtpk_dev, 0, sizeof (uint64_t) * GT_SMAX_PK_GROUPS(m), s));
    HIPCHK(hipMalloc(&bigflag, m));
    HIPCHK(hipMalloc(&sumd, sizeof *sumd));
    HIPCHK(hipMalloc(&maxd, sizeof *maxd));
    HIPCHK(hipMemset(sumd, 0, sizeof *sumd));
    HIPCHK(hipMemset(maxd, 0, sizeof *maxd));
    hipLaunchKernelGGL(k_finish, dim3(blocks_for(m)), dim3(256), 0, s, SA, plcp, T, m,
                       out->lcptab_dev, out->bwttab_dev, out->bwtpk_dev, bigflag, sumd, maxd);
    HIPCHK(hipGetLastError());
    llvpos = hv;   // reuse
    hipLaunchKernelGGL(k_iota, dim3(blocks_for(m)), dim3(256), 0, s, valB, m);
    size_t need = 0;
    HIPCHK(rocprim::select(nullptr, need, valB, bigflag, llvpos, cntd, m, s));
    HIPCHK(tmp.ensure(need));
    HIPCHK(rocprim::select(tmp.p, need, valB, bigflag, llvpos, cntd, m, s));
    uint32_t c32 = 0;
    HIPCHK(hipMemcpy(&c32, cntd, sizeof c32, hipMemcpyDeviceToHost));
    numllv = c32;
    HIPCHK(hipMalloc(&out->llvtab_dev, sizeof (GtSmaxLlv) * (numllv + 1)));
    if (numllv > 0)
      hipLaunchKernelGGL(k_llv, dim3(blocks_for(numllv)), dim3(256), 0, s, llvpos, numllv, SA,
                         plcp, out->llvtab_dev);
    HIPCHK(hipGetLastError());
    unsigned long long sum = 0;
    unsigned int mx = 0;
    HIPCHK(hipMemcpy(&sum, sumd, sizeof sum, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&mx, maxd, sizeof mx, hipMemcpyDeviceToHost));
    out->averagelcp = (double) sum / (double) m;
    out->maxbranchdepth = mx;
  }
  out->totallength = n;
  out->nonspecials = n - nspecial;
  out->numllv = numllv;
  out->sort_rounds = rounds;
  if (keep_suftab) {
    out->suftab_dev = SA;
    SA = NULL;
  }
  HIPCHK(hipDeviceSynchronize());
  (void) hipFree(T); (void) hipFree(P); (void) hipFree(S); (void) hipFree(keyA);
  (void) hipFree(valB); (void) hipFree(ISA); (void) hipFree(hv); (void) hipFree(cntd);
  (void) hipFree(bigflag); (void) hipFree(sumd); (void) hipFree(maxd);
  if (SA) (void) hipFree(SA);
  return 0;
fail:
  if (T) (void) hipFree(T);
  if (P) (void) hipFree(P);
  if (S) (void) hipFree(S);
  if (keyA) (void) hipFree(keyA);
  if (keyB) (void) hipFree(keyB);
  if (valA) (void) hipFree(valA);
  if (valB) (void) hipFree(valB);
  if (SA) (void) hipFree(SA);
  if (ISA) (void) hipFree(ISA);
  if (U) (void) hipFree(U);
  if (U2) (void) hipFree(U2);
  if (gs) (void) hipFree(gs);
  if (hv) (void) hipFree(hv);
  if (unres) (void) hipFree(unres);
  if (cntd) (void) hipFree(cntd);
  if (bigflag) (void) hipFree(bigflag);
  if (sumd) (void) hipFree(sumd);
  if (maxd) (void) hipFree(maxd);
  gt_smax_esa_release(out);
  return -1;
}

extern "C" int gt_smax_esa_download(const GtSmaxEsaDev *e, uint8_t *lcptab,
                                    uint8_t *bwttab, GtSmaxLlv *llvtab,
                                    uint64_t *suftab, char *errbuf,
                                    size_t errlen) {
  const uint64_t m = e->totallength + 1;
  uint32_t *s32 = NULL;
  HIPCHK(hipSetDevice(e->device));
  if (lcptab) HIPCHK(hipMemcpy(lcptab, e->lcptab_dev, m, hipMemcpyDeviceToHost));
  if (bwttab) HIPCHK(hipMemcpy(bwttab, e->bwttab_dev, m, hipMemcpyDeviceToHost));
  if (llvtab && e->numllv)
    HIPCHK(hipMemcpy(llvtab, e->llvtab_dev, sizeof (GtSmaxLlv) * e->numllv,
                     hipMemcpyDeviceToHost));
  if (suftab) {
    if (e->suftab_dev == NULL) {
      seterr(errbuf, errlen, "suftab was not kept on the device");
      return -1;
    }
    s32 = (uint32_t *) malloc(sizeof (uint32_t) * m);
    if (s32 == NULL) { seterr(errbuf, errlen, "out of memory"); return -1; }
    HIPCHK(hipMemcpy(s32, e->suftab_dev, sizeof (uint32_t) * m, hipMemcpyDeviceToHost));
    for (uint64_t k = 0; k < m; k++) suftab[k] = s32[k];
    free(s32);
  }
  return 0;
fail:
  free(s32);
  return -1;
}

extern "C" int gt_smax_esa_download_packed(const GtSmaxEsaDev *e, uint64_t *pk, char *errbuf,
                                           size_t errlen) {
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipMemcpy(pk, e->bwtpk_dev, sizeof (uint64_t) * GT_SMAX_PK_GROUPS(e->totallength + 1),
                   hipMemcpyDeviceToHost));
  return 0;
fail:
  return -1;
}
