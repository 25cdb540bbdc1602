// esa_common.h -- device helpers shared by the GPU ESA builders
// (esa_build.hip: 32-bit suffix array, esa_build64.hip: 64-bit, bucketed,
// range-restricted).  Text layout in HBM:
//   P   2-bit symbols, 32 per u64 word (symbol k of the word at bits 2k..2k+1),
//       specials stored as 0;
//   S   special bitmap, bit p set iff position p holds WILDCARD/SEPARATOR or
//       p >= n (the end of the text is a special, ranked last by position).
#ifndef GT_SMAX_ESA_COMMON_H
#define GT_SMAX_ESA_COMMON_H

#include <hip/hip_runtime.h>
#include <stdint.h>

// 32 symbols starting at position a
__device__ __forceinline__ uint64_t esa_sym32(const uint64_t *P, uint64_t a) {
  const uint64_t w = a >> 5;
  const unsigned sh = (unsigned) (a & 31) * 2;
  uint64_t v = P[w] >> sh;
  if (sh) v |= P[w + 1] << (64 - sh);
  return v;
}

// special bits of positions a .. a+31
__device__ __forceinline__ uint32_t esa_spec32(const uint64_t *S, uint64_t a) {
  const uint64_t w = a >> 6;
  const unsigned sh = (unsigned) (a & 63);
  uint64_t v = S[w] >> sh;
  if (sh) v |= S[w + 1] << (64 - sh);
  return (uint32_t) v;
}

// longest common prefix of the suffixes at a and b, known to be >= h
// (specials never match: the comparison ends at the first special of either)
__device__ __forceinline__ uint64_t esa_extend(const uint64_t *P, const uint64_t *S, uint64_t a,
                                               uint64_t b, uint64_t h) {
  for (;;) {
    const uint64_t x = esa_sym32(P, a + h) ^ esa_sym32(P, b + h);
    const uint32_t sp = esa_spec32(S, a + h) | esa_spec32(S, b + h);
    const uint32_t d1 = x ? (uint32_t) (__builtin_ctzll(x) >> 1) : 32u;
    const uint32_t d2 = sp ? (uint32_t) __builtin_ctz(sp) : 32u;
    const uint32_t d = d1 < d2 ? d1 : d2;
    h += d;
    if (d < 32) return h;
  }
}

// Order key of the ns (<= 21) symbols at position p, 3 bits each, first
// symbol most significant: bases 0..3, the first special 4 and zeros after
// it (a special ends the comparison; ties between keys holding a special are
// broken by position, which the stable sorts preserve).  *special is set
// when the key holds one.
__device__ __forceinline__ uint64_t esa_key3(const uint64_t *P, const uint64_t *S, uint64_t p,
                                             int ns, bool *special) {
  const uint64_t sy = esa_sym32(P, p);
  const uint32_t sp = esa_spec32(S, p) & ((1u << ns) - 1u);
  const int first = sp ? __builtin_ctz(sp) : ns;
  uint64_t k = 0;
  for (int c = 0; c < ns; c++) {
    const uint64_t code = c < first ? ((sy >> (2 * c)) & 3u) : (c == first ? 4u : 0u);
    k = (k << 3) | code;
  }
  *special = first < ns;
  return k;
}

#endif
