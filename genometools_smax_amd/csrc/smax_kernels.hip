// smax_kernels.hip -- CDNA4 (gfx950) kernels for the supermaximal-repeat
// hot path, plus the C-ABI declared in include/gt_smax_hip.h.
//
// Replaces the serial stack walk of gt_esa_bottomup
// (src/match/esa-bottomup.c:116-273, specialised at
// src/match/esa-bottomup-maxpairs.inc:136-264) by a data-parallel plateau
// segmentation of the LCP array.  An smax interval [lb..rb] of lcp-value l
//  is a maximal run LCP[lb+1..rb] == l with
// LCP[lb] < l and LCP[rb+1] < l (a leaf-only lcp-interval: the interval the
// reference pops without a branching edge), l >= minlen, whose BWT symbols
// BWT[lb..rb] below 254 are pairwise distinct (ISLEFTDIVERSE semantics of
// src/match/esa-maxpairs.c:24-31: WILDCARD/SEPARATOR/UNDEFBWTCHAR are unique).
//
// One pass = three launches on one stream, no host synchronisation
// (DESIGN.md §4); gt_smax_plan_run_part splits them into part 0 (scan: K1,
// K1b; the boundary record is final after it) and part 1 (compaction: K3):
//   K1  smax_scan_kernel     the streaming kernel; its block 0 also clears
//                            the pending-plateau slot of this run
//   K1b smax_defer_wg_kernel<4|8> one workgroup of 4 or 8 waves per
//                            deferred tile (8 when the launch fits one
//                            generation of them): the plan-time
//                            static list (shard edges, windows with more
//                            .llv values than K1 stages), then K1's runtime
//                            deferrals (exact-queue overflow, tiles with more
//                            records than a slot holds); one extra workgroup
//                            computes the boundary head, and its last
//                            workgroups add up the records per 256 tiles
//                            (K3's offsets; a separate block-sum launch was
//                            measured and retired, and a decoupled look-back
//                            inside K3 measured 1.3 -> 1.9 ms at C3: the
//                            prefix chain over 5663 workgroups serialises)
//   K3  smax_compact_kernel  ordered copy of the tiles' records -> ascending
//                            lb; resets the deferral count and pool cursor
//                            for the next run (their last reader, K1b, is done)
// (smax_head_kernel -- "K0" -- runs only for an empty shard.)
//
// K1: every wave is an independent worker on 2048-row tiles (tile = wave id
// + k * waves in grid; 8-16 generations of resident one-wave workgroups, 6
// per SIMD for the 2-plane windows), no workgroup barrier.  Per tile:
//   window   LCP bytes (+16-row halos), packed BWT bit planes (DNA) or BWT
//            bytes, and the window's .llv values (u16) go global -> LDS by
//            LDS-DMA into one of the wave's two windows; the next tile's
//            DMA is issued as soon as this one has landed;
//   filter   per 16-row segment "any byte >= min(minlen,128)", refined to
//            segments where a row can start a record when more than one
//            64-lane step would be needed;
//   classify active segments are compacted and classified with SWAR byte
//            relations: 2- and 3-row intervals are decided in place (local
//            maximum + left diversity from the bit planes); plateaus of
//            >= 3 rows and 255 bytes (.llv values by rank) go to an exact
//            queue of 56 starts, evaluated one per lane;
//   output   owning lanes put packed 8-byte records in row order into an
//            LDS staging slot; lane r then holds record r, and the tile's
//            slot store (one coalesced instruction) and count are issued at
//            the start of the next tile, right after its window wait.
// No MFMA: integer/byte work bounded by HBM bandwidth.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <type_traits>
#include <chrono>
#include <vector>

#include "gt_smax_hip.h"
#include "smax_internal.h"

// per-chunk 255-byte ranks: K1 windows stage at most SMAX_LLV_CAP (< 256)
// .llv entries (more: the tile is static, K1b), so a byte holds every rank
typedef uint8_t SmaxRank;
// the next-but-one tile's llv_win words into their LDS ring slot (lanes 0-1),
// part of every window DMA
#define SMAX_ASM_INFO                        \
  "s_mov_b64 exec, %13\n\t"                 \
  "s_mov_b32 m0, %7\n\t"                    \
  "s_nop 0\n\t"                             \
  "global_load_lds_dword %3, %12 offset:0\n\t"
#define SMAX_THREADS 256                              // 4 waves per K3 workgroup (and the 4-wave K1b)
// K1 workgroup: ONE wave.  K1's waves share nothing (no barrier, each its own
// LDS windows), so a one-wave workgroup frees its LDS and wave slot as soon
// as that wave is done -- with four waves per workgroup, a wave that ran out
// of tiles early held its slot idle until the slowest of the four finished
#define SMAX_K1_THREADS 64
#define SMAX_SEGS 2                                   // 16-row segments per lane
#define SMAX_WAVE_BYTES (SMAX_SEGS * 64 * 16)         // 2048 rows per wave tile
#define SMAX_TILE SMAX_WAVE_BYTES                     // a tile is one wave's work
#define SMAX_LH 16                                    // left halo (bytes)
#define SMAX_RH 16                                    // right halo (bytes)
#define SMAX_LDSB (SMAX_LH + SMAX_TILE + SMAX_RH)     // LDS window bytes
#define SMAX_NCHUNK (SMAX_LDSB / 16)                  // 16-byte window chunks
// tile slot formats: K1 writes packed 8-byte records (row + 1 in the tile:
// 11 bits, width: 21 bits, lcp: 32 bits; wider records send the tile to
// K1b), K1b writes GtSmaxRecord (16 bytes) and flags its tile count
#define SMAX_PK_WMAX ((1u << 21) - 1)
#define SMAX_CPB 256                                  // tiles per K3 workgroup / block sum
#define SMAX_SBB 64                                   // blocks per superblock sum (K3's two-level prefix)
// K1b workgroups for K1's runtime deferrals: 64 + one per this many tiles
// (about one tile in 10^4 defers; more loop; 4096 against 1024: 1/8 shards
// of C3 -0.1 to -1.8 %, profiles/s5/k1b_slack_ab_*)
#define SMAX_K1B_SLACK 4096u
// one run's block-sum buffer (block sums added up in K1b's launch): the
// blocks' sums, then the superblocks' sums
__host__ __device__ __forceinline__ uint64_t smax_bs_stride(uint64_t nblocks) {
  return nblocks + (nblocks + SMAX_SBB - 1) / SMAX_SBB;
}
#define SMAX_SLOT_WIDE 0x80000000u
#define SMAX_LLV_CAP 240                              // .llv values staged in K1's LDS (u16):
                                                      // one 16-byte DMA per lane; windows
                                                      // with more go to the static K1b list
                                                      // (the LDS budget of 5 workgroups/CU)
// llv_win[t].y: entries in the window (12 bits), of them in the left halo
// (5 bits, <= 16), bit 31: K1 leaves the tile to the static K1b list
#define SMAX_WIN_N(y) ((y) & 0xfffu)
#define SMAX_WIN_HALO(y) (((y) >> 12) & 0x1fu)
// (6 bits): the 16-byte lanes of u16 .llv values K1's window DMA moves (from
// the 8-aligned index at or below the first entry, at most SMAX_LLV_CAP / 8),
// computed at plan time -- K1 turns it into an EXEC mask with two scalar ops
#define SMAX_WIN_LANES(y) (((y) >> 17) & 0x3fu)
#define SMAX_WIN_STATIC 0x80000000u
#define SMAX_SSLOT 64                                 // packed records per K1 tile slot
#define SMAX_FFPV_DENSITY 0.006                       // .llv entries per row: dense K1 above
                                                      // (0.25 B per row; a tile with more
                                                      // goes to K1b, whose 16-byte records
                                                      // are allocated from the plan's pool)

static_assert(GT_SMAX_PAD_BACK >= SMAX_TILE + SMAX_RH,
              "back padding must cover a whole tile plus halo");
static_assert(GT_SMAX_PAD_FRONT >= SMAX_LH, "front padding covers the halo");
static_assert(SMAX_LDSB % 16 == 0, "window is whole 16-byte chunks");

// K1 grid generations with their own tile counts (guided schedule)
#define SMAX_SCHED_MAX 12
#ifndef SMAX_K1_GUIDED
#define SMAX_K1_GUIDED 1
#endif
#ifndef SMAX_GUIDE_NUM                                // a generation takes NUM/DEN of the tiles left
#define SMAX_GUIDE_NUM 2
#define SMAX_GUIDE_DEN 3
#endif
struct SmaxScanArgs {
  const uint8_t *lcp;        // local tables: index i <-> global base+i
  const uint8_t *bwt;
  const uint64_t *bwtpk;     // packed BWT, 16 rows per u64 (index local_row/16 + 1), or null
  const uint32_t *bwt2;      // its two code planes alone, 16 rows per u32 (same index), or
                             // null: K1's window stream when no window holds a special
  const GtSmaxLlv *llv;      // shard's llv entries (global positions)
  const uint16_t *llv16;     // their values as u16 (plan time; windows with larger ones defer)
  uint64_t numllv;
  const uint2 *llv_win;      // per tile: {first llv index >= g0 - LH, entries in the window}
  uint64_t base, begin, end, N;
  uint64_t local_len;        // readable: [-PAD_FRONT, local_len + PAD_BACK)
  uint32_t *err;             // sticky error bits (bounds), read by the host
  uint64_t tile_first;       // first local tile holding an owned row
  uint32_t minlen;
  uint32_t num_tiles;
  uint64_t *slots;           // [tile][SMAX_SSLOT] K1's packed records, row order
  GtSmaxRecord *pool;        // K1b's records, per tile a run allocated at tile_off
  uint64_t pool_cap;         // records the pool holds
  unsigned long long *pool_cursor;   // reset by K0
  uint64_t *tile_off;        // per K1b tile: its first pool record (~0: pool full)
  uint32_t *tile_count;      // [tile][wave] record counts
  uint32_t *block_sum;       // records per SMAX_CPB tiles (K3's workgroups), summed in K1b's launch
  GtSmaxBoundary *bnd;
  uint32_t *defer_list;      // tiles left to K1b (num_tiles capacity)
  uint2 *defer_info;         // beside each entry: the tile's llv_win word pair (K1b's
                             // .llv loads need not wait for a load of llv_win[tile])
  uint32_t *defer_count;     // reset by K0
  uint32_t k1b_head;         // K1b: one workgroup computes the boundary head
  uint32_t wide_slot0;       // K1b: wide slot of list entry 0 (static list 0, runtime n_static)
  uint32_t defer_base;       // K0 resets *defer_count to this (combined list: n_static)
  uint32_t k1_reset;         // combined placement without K0: K1 clears the pending slot
  uint32_t wide_cap;         // wide slots (SMAX_TILE / 2 records each) at the pool's start
  uint32_t dbg;              // diagnostic ablation bits (GT_SMAX_DEBUG), 0 in use
  uint32_t bs_wgs;           // block-sum workgroups at the end of the K1b grid;
                             // K1 then marks its deferred and static tiles' counts
  unsigned long long *stamps; // diagnostic (GT_SMAX_STAMPS, diag build only): per-section
                              // s_memtime cycles of K1 summed over waves, [7] = tiles
  // K1's tile schedule (plan time, plan_size_grid), or null: per workgroup
  // {first tile, stride, end of its generation's tile range}
  const uint4 *sched_wg;
};

// Diagnostic ablation bits (GT_SMAX_DEBUG) exist only in the diagnostic build
// (-DGT_SMAX_DIAG: lib/diag/libgtsmax_hip.so beside the production library,
// loaded through GT_SMAX_LIB); the production library reads no such switch and
// every diagnostic branch is a compile-time constant there.  Its test hooks
// are plan-time choices (GT_SMAX_ALL_STATIC, GT_SMAX_BYTE_WINDOWS, ...).
#ifdef GT_SMAX_DIAG
#define SMAX_DBG(a) ((a).dbg)
#else
#define SMAX_DBG(a) (0u)
#endif

// K1 section stamps (diagnostic build): cycles since the previous stamp
// into acc[k]; the production build compiles them away
struct SmaxStamps {
  unsigned long long acc[8];
  unsigned long long prev;
};
#define SMAX_STAMP(ST, K)                                                    \
  do {                                                                       \
    if ((ST) != nullptr) {                                                   \
      const unsigned long long tn_ = __builtin_amdgcn_s_memtime();           \
      (ST)->acc[K] += tn_ - (ST)->prev;                                      \
      (ST)->prev = tn_;                                                      \
    }                                                                        \
  } while (0)

// ------------------------------------------------------------ helpers

#define SMAX_ERR_LLV 1u        // a 255 byte without its .llv entry
#define SMAX_ERR_RANGE 2u      // a table read outside the shard's rows
#define SMAX_ERR_EXEC 4u       // diagnostic build: window DMA issued from a divergent wave

// Rare-path global loads of the scan kernels, each with its own wait inside
// one asm statement: hipcc sees no outstanding load, so it never places a
// vmcnt(0) on the common path (which would also drain K1's in-flight DMA of
// the next window); the wait is paid only when the load executes.
__device__ __forceinline__ uint32_t gld_u8(const void *p) {
  uint32_t v;
  asm volatile("global_load_ubyte %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=&v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ uint32_t gld_u32(const void *p) {
  uint32_t v;
  asm volatile("global_load_dword %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=&v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ uint64_t gld_u64(const void *p) {
  uint64_t v;
  asm volatile("global_load_dwordx2 %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=&v"(v) : "v"(p) : "memory");
  return v;
}
// low dword of an .llv record's value (values < 2^32 are checked at plan time)
__device__ __forceinline__ uint32_t llv_value(const GtSmaxLlv *e) {
  return gld_u32(reinterpret_cast<const uint8_t *>(e) + 8);
}

// exact LCP value from the global .llv (binary search in [lo, hi))
__device__ static uint32_t llv_search_global(const GtSmaxLlv *llv, uint64_t lo,
                                             uint64_t hi, uint64_t g, uint32_t *err) {
  const uint64_t stop = hi;
  while (lo < hi) {
    uint64_t mid = (lo + hi) >> 1;
    uint64_t p = gld_u64(&llv[mid].position);
    if (p < g) lo = mid + 1; else hi = mid;
  }
  if (lo >= stop || gld_u64(&llv[lo].position) != g) {   // never for a consistent index
    atomicOr(err, SMAX_ERR_LLV);
    return 255;
  }
  return llv_value(&llv[lo]);
}

// high bit of each byte of w that is >= m (1 <= m <= 128); exact
__device__ __forceinline__ uint32_t bytes_ge(uint32_t w, uint32_t m) {
  uint32_t add = (128u - m) * 0x01010101u;
  return (w | ((w & 0x7f7f7f7fu) + add)) & 0x80808080u;
}
// high bit of each byte of w that equals 0xff; exact
__device__ __forceinline__ uint32_t bytes_ff(uint32_t w) {
  uint32_t x = ~w;
  return ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x | 0x7f7f7f7fu) & 0x80808080u;
}

// SWAR byte compares: high bit of each byte where the relation holds.
__device__ __forceinline__ uint32_t bytes_eq(uint32_t x, uint32_t y) {
  const uint32_t z = x ^ y;
  return ~(((z & 0x7f7f7f7fu) + 0x7f7f7f7fu) | z | 0x7f7f7f7fu) & 0x80808080u;
}

// 64-bit SWAR: high bit of each byte of x equal to the same byte of y
__device__ __forceinline__ uint64_t bytes_eq64(uint64_t x, uint64_t y) {
  return ((uint64_t) bytes_eq((uint32_t) (x >> 32), (uint32_t) (y >> 32)) << 32) |
         bytes_eq((uint32_t) x, (uint32_t) y);
}

// LDS pointers held in Win are 32-bit local addresses (address space 3):
// generic 64-bit pointers kept for their null tests cost an SGPR pair each
// across K1's tile loop, and K1's loop was spilling SGPRs to VGPR lanes
#define LDSP __attribute__((address_space(3)))
template <typename T>
__device__ __forceinline__ const LDSP T *to_lds(const T *p) { return (const LDSP T *) p; }
__device__ __forceinline__ const LDSP uint8_t *to_lds_any(const uint8_t *p) { return to_lds(p); }
__device__ __forceinline__ const LDSP uint8_t *to_lds_any(const LDSP uint8_t *p) { return p; }
// 16 window bytes at an LDS address (16-byte aligned): one ds_read_b128
__device__ __forceinline__ uint4 lds_ld16(const LDSP uint8_t *p) {
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const v4u v = *reinterpret_cast<const LDSP v4u *>(p);
  return make_uint4(v.x, v.y, v.z, v.w);
}

// 8 consecutive window bytes starting at LDS offset o (o + 11 inside the
// window): three aligned dword reads, issued together
template <typename P>
__device__ __forceinline__ uint64_t lds_bytes8(P base, uint32_t o) {
  const auto *w = reinterpret_cast<const LDSP uint32_t *>(to_lds_any(base) + (o & ~3u));
  const uint32_t d0 = w[0], d1 = w[1], d2 = w[2];
  const uint32_t sh = o & 3u;
  return ((uint64_t) __builtin_amdgcn_alignbyte(d2, d1, sh) << 32) |
         __builtin_amdgcn_alignbyte(d1, d0, sh);
}

// The launch's SmaxScanArgs in the kernarg segment: every kernel that builds
// a Win takes them as its first parameter.  The global-fallback paths (rows
// outside the LDS window, .llv values not staged) load the shard's table
// pointers and bounds from there where they are used, through an opaque copy
// of the segment pointer, so that none of them is held in SGPRs across K1's
// tile loop (K1 spilled SGPRs to VGPR lanes, a VALU readlane per reload).
typedef const __attribute__((address_space(4))) SmaxScanArgs *KArgs;
__device__ __forceinline__ KArgs kargs() {
  uint64_t p = (uint64_t) __builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return (KArgs) p;
}

struct Win {
  uint64_t N, end;            // global row bounds (plateau scans)
  const LDSP uint8_t *L;      // LDS window: index o = g - g0 + LH
  const LDSP uint8_t *B;      // BWT bytes of the window (byte kernel), or
  const LDSP uint64_t *P;     // packed BWT of the window, 16 rows per word
  bool p2;                    // P holds u32 words (code planes only, no specials)
  const LDSP SmaxRank *rank;  // per 16-byte chunk: 255 bytes before it
  const LDSP uint32_t *val;   // LDS .llv values in rank order (nval of them), or
  const LDSP uint16_t *val16; // the same as u16 (K1 windows: values < 65536)
  int nval;                   // -1: values not staged (read global by rank)
  uint32_t halo_ff;           // 255 bytes in the window's left halo (K1)
  bool staged_all;            // K1: every value of the window is staged (nval of
                              // them; the static flag guarantees it) -- a constant
                              // in K1, so the global fallback folds away
  uint64_t g0;                // global row of the tile start
  uint64_t llv_base;          // first llv entry of the window
};

__device__ __forceinline__ void win_init(Win &t, const SmaxScanArgs &a) {
  t.N = a.N; t.end = a.end;
  t.L = nullptr; t.B = nullptr; t.P = nullptr; t.p2 = false; t.rank = nullptr; t.val = nullptr;
  t.val16 = nullptr; t.nval = -1; t.halo_ff = 0; t.staged_all = false;
  t.g0 = 0; t.llv_base = 0;
}

__device__ __forceinline__ int64_t win_off(const Win &t, uint64_t g) {
  return (int64_t) (g - t.g0) + SMAX_LH;
}

// packed BWT group gi of the window as a u64 word (the 2-plane form reads
// as the u64 form with no special bits)
__device__ __forceinline__ uint64_t pk_word(const Win &t, uint32_t gi) {
  return t.p2 ? (uint64_t) reinterpret_cast<const LDSP uint32_t *>(t.P)[gi] : t.P[gi];
}

// exact LCP of a row whose byte is 255
__device__ static uint32_t lcp_big(const Win &t, uint64_t g) {
  const int64_t o = win_off(t, g);
  if (t.rank != nullptr && o >= 0 && o < SMAX_LDSB) {
    const int chunk = (int) (o >> 4), within = (int) (o & 15);
    const uint4 v = lds_ld16(&t.L[chunk * 16]);
    const uint64_t lo = (uint64_t) bytes_ff(v.x) | ((uint64_t) bytes_ff(v.y) << 32);
    const uint64_t hi = (uint64_t) bytes_ff(v.z) | ((uint64_t) bytes_ff(v.w) << 32);
    int cnt;
    if (within < 8) cnt = __popcll(lo & ((1ull << (8 * within)) - 1));
    else cnt = __popcll(lo) + __popcll(hi & ((1ull << (8 * (within - 8))) - 1));
    const uint32_t r = t.rank[chunk] + (uint32_t) cnt;
    if (t.staged_all) return t.val16[min((int) r, t.nval - 1)];
    if ((int) r < t.nval) return t.val16 != nullptr ? t.val16[r] : t.val[r];
    const KArgs k = kargs();
    if (t.llv_base + r >= k->numllv) { atomicOr(k->err, SMAX_ERR_LLV); return 255; }
    return llv_value(&k->llv[t.llv_base + r]);
  }
  const KArgs k = kargs();
  return llv_search_global(k->llv, 0, k->numllv, g, k->err);
}

// byte of LCP[g] (LCP[0] = LCP[N] = 0 are returned as 0)
__device__ __forceinline__ uint32_t lcp_byte(const Win &t, uint64_t g) {
  if (g == 0 || g >= t.N) return 0;
  const int64_t o = win_off(t, g);
  if (t.L != nullptr && o >= 0 && o < SMAX_LDSB) return t.L[o];
  const KArgs k = kargs();
  if (g < k->base || g - k->base >= k->local_len) { atomicOr(k->err, SMAX_ERR_RANGE); return 0; }
  return gld_u8(&k->lcp[g - k->base]);
}

__device__ __forceinline__ uint32_t lcp_exact(const Win &t, uint64_t g) {
  const uint32_t b = lcp_byte(t, g);
  return b < 255 ? b : lcp_big(t, g);
}

// Packed BWT (DNA): per 16 rows one u64 in bit planes -- bit q the low bit
// and bit 16+q the high bit of row q's symbol code (0..3), bit 32+q set when
// row q holds a special symbol (254/255, unique for left diversity; decoded
// as 254).  Planes make the row-vs-neighbour compares of the diversity tests
// plain 16-bit shifts and xors (no 2-bit field compression).
__device__ __forceinline__ uint32_t pk_sym(uint64_t w, uint32_t q) {
  return ((w >> (32 + q)) & 1u) ? 254u
                                : (uint32_t) (((w >> q) & 1u) | (((w >> (16 + q)) & 1u) << 1));
}

__device__ __forceinline__ uint32_t bwt_at(const Win &t, uint64_t g) {
  const int64_t o = win_off(t, g);
  if (t.B != nullptr && o >= 0 && o < SMAX_LDSB) return t.B[o];
  if (t.P != nullptr && o >= 0 && o < SMAX_LDSB) return pk_sym(pk_word(t, (uint32_t) (o >> 4)), (uint32_t) (o & 15));
  const KArgs k = kargs();
  const uint64_t base = k->base;
  if (g < base || g - base >= k->local_len) { atomicOr(k->err, SMAX_ERR_RANGE); return 254; }
  if (k->bwtpk != nullptr)
    return pk_sym(gld_u64(&k->bwtpk[(g - base) / 16 + 1]), (uint32_t) ((g - base) & 15));
  return gld_u8(&k->bwt[g - base]);
}

// the 16 rows of a packed group as BWT bytes (specials as 254)
__device__ __forceinline__ uint4 pk_expand(uint64_t w) {
  uint32_t o[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    uint32_t x = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) x |= pk_sym(w, (uint32_t) (4 * k + q)) << (8 * q);
    o[k] = x;
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
}

// Plateau scan from start c with exact value l: returns j (last row of the
// run); *rel = sign of LCP[j+1] - l (-1 / +1); *pending when the run reaches
// the shard end (LCP[end] == l with end < N).
__device__ static uint64_t plateau_end(const Win &t, uint64_t c, uint32_t l,
                                       int *rel, bool *pending) {
  const uint32_t lb = l < 255 ? l : 255;
  uint64_t j = c;
  *pending = false;
  // long plateaus inside the LDS window: 8 rows per step (exact: lb < 255,
  // rows j+1 .. j+8 all below end and N)
  if (lb < 255 && t.L != nullptr) {
    const uint64_t splat = lb * 0x0101010101010101ull;
    for (;;) {
      const int64_t o = win_off(t, j + 1);
      if (o < 0 || o + 11 >= SMAX_LDSB || j + 8 >= t.end || j + 8 >= t.N) break;
      const uint64_t ne = ~bytes_eq64(lds_bytes8(t.L, (uint32_t) o), splat) &
                          0x8080808080808080ull;
      if (ne != 0) {
        const uint32_t k = (uint32_t) __builtin_ctzll(ne) >> 3;
        const uint32_t nb = t.L[o + k];
        *rel = nb < lb ? -1 : 1;
        return j + k;
      }
      j += 8;
    }
  }
  for (;;) {
    const uint64_t g = j + 1;
    const uint32_t nb = lcp_byte(t, g);
    if (nb != lb) { *rel = nb < lb ? -1 : 1; return j; }
    if (lb == 255) {
      const uint32_t nx = lcp_big(t, g);
      if (nx != l) { *rel = nx < l ? -1 : 1; return j; }
    }
    if (g >= t.end) { *pending = true; *rel = 0; return j; }
    j = g;
  }
}

struct Seen {
  uint64_t w0, w1, w2, w3;
};
__device__ __forceinline__ bool seen_add(Seen &s, uint32_t c) {
  if (c >= 254) return false;
  const uint64_t bit = 1ull << (c & 63);
  const uint32_t wi = c >> 6;
  const uint64_t cur = wi == 0 ? s.w0 : wi == 1 ? s.w1 : wi == 2 ? s.w2 : s.w3;
  s.w0 |= wi == 0 ? bit : 0;
  s.w1 |= wi == 1 ? bit : 0;
  s.w2 |= wi == 2 ? bit : 0;
  s.w3 |= wi == 3 ? bit : 0;
  return (cur & bit) != 0;
}

// ------------------------------------------------------------ K0: head run

// One lane: the boundary record's head (run of LCP == LCP[begin]), reset of
// the pending slot and of the overflow cursor.  Runs before K1.
// The shard's boundary head (run of LCP == LCP[begin] at the shard start),
// one lane, global reads.
__device__ static void compute_head(const SmaxScanArgs &a) {
  Win t;
  win_init(t, a);
  GtSmaxBoundary *b = a.bnd;
  b->shard_begin = a.begin;
  b->shard_end = a.end;
  const uint32_t v = lcp_exact(t, a.begin);
  b->head_v = v;
  Seen s = {0, 0, 0, 0};
  uint64_t dup = 0;
  uint64_t f = UINT64_MAX, nxt = 0;
  if (v >= a.minlen && a.begin < a.end) {
    uint64_t g = a.begin;
    for (;;) {
      if (seen_add(s, bwt_at(t, g))) { dup = 1; break; }
      const uint64_t h = g + 1;
      const uint32_t nx = lcp_exact(t, h);
      if (nx != v) { f = h; nxt = nx; break; }
      if (h >= a.end) break;   // run covers the whole shard: passthrough
      g = h;
    }
  } else {
    f = a.begin;   // irrelevant head: no pending plateau can continue here
    nxt = v;
  }
  b->head_f = f;
  b->head_next = nxt;
  b->head_div.seen[0] = s.w0; b->head_div.seen[1] = s.w1;
  b->head_div.seen[2] = s.w2; b->head_div.seen[3] = s.w3;
  b->head_div.dup = dup;
}

// The plan-time half of K1's deferral rule, shared by K1 and the static list
// kernel: shard-edge tiles (row 0, begin, end, N: halos outside the shard)
// and windows whose .llv entries K1 cannot stage (more than fit from the
// 8-aligned index at or below the first, or a value >= 2^16) -- decided by
// smax_llv_index_kernel into bit 31 of the tile's llv_win word.
__host__ __device__ __forceinline__ bool static_deferred(const SmaxScanArgs &a, uint32_t wnf) {
  return (wnf & SMAX_WIN_STATIC) != 0 || (SMAX_DBG(a) & 64u);
}

// the llv_win words of the combined list's static entries (plan time)
__global__ void __launch_bounds__(256) smax_defer_info_kernel(const uint32_t *list, uint32_t n,
                                                              const uint2 *llv_win, uint2 *info) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) info[k] = llv_win[list[k]];
}

__global__ void __launch_bounds__(256) smax_static_defer_kernel(SmaxScanArgs a, uint32_t *list,
                                                                 uint32_t *count) {
  const uint64_t t = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (t >= a.num_tiles) return;
  const uint64_t g0 = a.base + (a.tile_first + t) * (uint64_t) SMAX_TILE;
  (void) g0;
  if (static_deferred(a, a.llv_win[t].y)) list[atomicAdd(count, 1u)] = (uint32_t) t;
}

// K0, an empty shard's whole pass (begin == end: no tile to scan): the
// per-run resets (pending-plateau slot, pool cursor, deferral count) and the
// boundary head.  Non-empty shards never launch it: K1 clears the pending
// slot, the previous run's K3 resets the rest and K1b computes the head.
__global__ void __launch_bounds__(64) smax_head_kernel(SmaxScanArgs a) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  a.bnd->pend_valid = 0;
  *a.pool_cursor = (unsigned long long) a.wide_cap * (SMAX_TILE / 2);   // past the wide slots
  *a.defer_count = a.defer_base;
  compute_head(a);
}

// ------------------------------------------------------------ K1: scan

// LDS-DMA (global_load_lds): global -> LDS with no VGPR destination, lane
// i writing lds_base + i * size.  Issued from inline asm so that hipcc
// neither counts it nor drains it at __syncthreads(): the next tile's window
// stays in flight across the current tile's barriers, and the kernel waits
// for it itself (s_waitcnt vmcnt(0) before the barrier that publishes it).
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
  return (uint32_t) (uintptr_t) (const __attribute__((address_space(3))) void *) p;
}
__device__ __forceinline__ void glds16(const void *g, uint32_t lds_base) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(g), "s"(lds_base) : "memory");
}
__device__ __forceinline__ void glds4(const void *g, uint32_t lds_base) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
               "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(g), "s"(lds_base) : "memory");
}
__device__ __forceinline__ void glds_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// One tile's LDS window: LCP and BWT bytes of rows [g0 - LH, g0 + TILE + RH)
// and the window's .llv values (rank order, first SMAX_LLV_CAP of them).
struct SmaxWindow {            // byte BWT (any alphabet)
  uint8_t L[SMAX_LDSB];
  uint8_t B[SMAX_LDSB];
  uint16_t val16[SMAX_LLV_CAP];
};
struct SmaxWindowPk {          // packed BWT (DNA): 0.5 B per row
  uint8_t L[SMAX_LDSB];
  uint64_t P[SMAX_LDSB / 16 + 2];   // + 2: the tail DMA moves 2 lanes x 16 B
  uint16_t val16[SMAX_LLV_CAP];
};
// window_scratch: the 64 staged records in the BWT region
static_assert(sizeof(((SmaxWindowPk *) 0)->P) >= 64 * 8, "packed window scratch");
// 2-plane window (the 6-wave K1: 6,816 B of LDS per one-wave workgroup, 24
// per CU, at most 80 VGPRs): groups l0/16 .. l0/16+131 as u32 (the 33-lane
// DMA); once the BWT is dead, the tile's 64 staged records
struct SmaxWindowB2 {
  uint8_t L[SMAX_LDSB];
  uint64_t P[(SMAX_LDSB / 16 + 2) / 2];   // 132 u32 = 528 B
  uint16_t val16[SMAX_LLV_CAP];
};
static_assert(sizeof(((SmaxWindowB2 *) 0)->P) >= 64 * 8, "2-plane window scratch");
static_assert(sizeof(SmaxWindowB2) == 3088, "6-wave LDS budget");
static_assert(SMAX_LDSB >= 64 * 8 + 2 * 64 * 4, "byte window scratch");

// Issue the DMA of tile `l0` (local index) into the calling wave's window
// w: 16 B per lane per instruction (1 KiB per wave instruction), the two
// 16-row halos, and the window's .llv values {lo, n} (low dword of each
// record's value, at most SMAX_LLV_CAP).
static_assert(SMAX_LH == 16 && SMAX_RH == 16 && SMAX_TILE == 2048,
              "packed window: one halo group each side, 128 tile groups");
__device__ __forceinline__ void issue_lcp_llv(const SmaxScanArgs &a, uint64_t l0, uint8_t *L,
                                              uint16_t *val, uint32_t lo, uint32_t n) {
  const int lane = threadIdx.x & 63;
  const uint32_t wl = __builtin_amdgcn_readfirstlane(lds_addr(L));
  const uint32_t wv = __builtin_amdgcn_readfirstlane(lds_addr(val));
  const uint8_t *ls = a.lcp + l0 + lane * 16;
#pragma unroll
  for (int r = 0; r < SMAX_SEGS; r++) glds16(ls + r * 1024, wl + SMAX_LH + r * 1024);
  if (lane == 0) {
    glds16(a.lcp + l0 - SMAX_LH, wl);
    glds16(a.lcp + l0 + SMAX_TILE, wl + SMAX_LH + SMAX_TILE);
  }
  // u16 copies of the values (plan-time array; K1 defers windows holding a
  // value >= 65536): eight per lane from the 8-aligned index at or below lo
  if (n != 0 && lane < SMAX_LLV_CAP / 8 && (uint32_t) (8 * lane) < n + (lo & 7u))
    glds16(a.llv16 + (lo & ~7u) + 8 * lane, wv);
}
__device__ __forceinline__ void issue_window(const SmaxScanArgs &a, uint64_t l0, SmaxWindow *w,
                                             uint32_t lo, uint32_t n) {
  const int lane = threadIdx.x & 63;
  const uint32_t wb = __builtin_amdgcn_readfirstlane(lds_addr(w->B));
  const uint8_t *bs = a.bwt + l0 + lane * 16;
  issue_lcp_llv(a, l0, w->L, w->val16, lo, n);
#pragma unroll
  for (int r = 0; r < SMAX_SEGS; r++) glds16(bs + r * 1024, wb + SMAX_LH + r * 1024);
  if (lane == 0) {
    glds16(a.bwt + l0 - SMAX_LH, wb);
    glds16(a.bwt + l0 + SMAX_TILE, wb + SMAX_LH + SMAX_TILE);
  }
}
// Packed window of local tile start l0 in ONE asm statement (M0 and EXEC
// set once per piece, SGPR base + per-lane VGPR offset; the instruction
// offset moves the global and the LDS address alike): LCP rows
// [l0-LH, l0+TILE+RH) as 1 KiB + 1 KiB + 32 B (2 lanes), packed BWT groups
// l0/16 .. l0/16+131 as 1 KiB + 32 B (2 lanes), the window's .llv values as
// u16 pairs (vlanes lanes x 4 B), and, if ibase != 0, the llv_win entry at
// ibase (2 lanes x 4 B) into LDS address iaddr.
// wl: LDS address of the target window (uniform, precomputed per buffer --
// generic-to-LDS pointer casts carry null checks that cost scalar work per
// tile); ibase: the llv_win entry to stage at iaddr.
// NT: the window stream (LCP bytes, packed BWT: read once per pass) as
// non-temporal LDS-DMA loads.  Measured (profiles/r02zz_nt_policy.txt): on
// shards whose stream exceeds the 256 MB MALL but whose per-tile state stays
// small (the 4- and 8-way C3 splits) the step is 2-6 % shorter; on the whole
// C3 table 6 % longer, on a table the MALL holds (C2) 4 % longer -- so the
// plan picks it by shard size (GtSmaxPlan::nt).
// a wave-uniform pointer as scalars (the asm's SGPR operands: uniform values
// the compiler keeps in VGPRs -- the prologue's tile index -- would not fit
// them; a no-op for values already in SGPRs)
template <typename T>
__device__ __forceinline__ const T *uni_ptr(const T *p) {
  const uint64_t v = (uint64_t) p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t) v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t) (v >> 32));
  return reinterpret_cast<const T *>(((uint64_t) hi << 32) | lo);
}

// PRECONDITION: wave-uniform call with every lane active.  The DMA asm
// below sets EXEC itself (33 lanes as exec_hi = 1 over an all-ones exec_lo,
// then 2, then the value lanes) and leaves it at -1 without saving the
// caller's mask; called from a divergent region it would silently switch
// the inactive lanes back on.  Both call sites (issue_next in the K1 tile
// loop: before the loop and at the top of each iteration) are wave-uniform;
// the diagnostic build checks it and raises SMAX_ERR_EXEC.
template <bool NT, bool BW2 = false, typename WinT = SmaxWindowPk>
__device__ __forceinline__ void issue_window_pk(const SmaxScanArgs &a, uint64_t l0, uint32_t wl,
                                                uint32_t lo, uint32_t nyw, const void *ibase,
                                                uint32_t iaddr, uint32_t v16, uint32_t v4) {
#ifdef GT_SMAX_DIAG
  if (__builtin_amdgcn_read_exec() != ~0ull) atomicOr(a.err, SMAX_ERR_EXEC);
#endif
  const uint32_t wp = wl + (uint32_t) offsetof(WinT, P);
  const uint32_t wv = wl + (uint32_t) offsetof(WinT, val16);
  const uint8_t *vb = uni_ptr(reinterpret_cast<const uint8_t *>(a.llv16 + (lo & ~7u)));
  // 16-byte lanes of values (plan time, llv_win word nyw)
  // (s_bfm: the mask of the low SMAX_WIN_LANES(nyw) lanes in one instruction,
  // its width operand's bits 5:0 being the lane-count field)
  uint64_t vmask;
  static_assert(SMAX_WIN_LANES(~0u) == 0x3fu, "lane count: bits 17..22 of the llv_win word");
  asm("s_bfm_b64 %0, %1, 0" : "=s"(vmask) : "s"(nyw >> 17));
  const uint8_t *ib = uni_ptr(reinterpret_cast<const uint8_t *>(ibase));
  uint32_t keep;
  uint64_t ex;
  if constexpr (BW2) {
    // 2-plane window: LCP rows [l0-LH, l0+TILE+RH) (2 x 1 KiB + 2 lanes),
    // code-plane groups l0/16 .. l0/16+131 (33 lanes x 16 B), the .llv
    // values, the llv_win word of the tile after next
    const uint8_t *lb = uni_ptr(a.lcp + l0 - SMAX_LH);
    const uint8_t *pb = uni_ptr(reinterpret_cast<const uint8_t *>(a.bwt2 + l0 / 16));
    const uint64_t p2mask = (1ull << 33) - 1;
    if constexpr (NT) {
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %4\n\t"
        "global_load_lds_dwordx4 %2, %8 offset:0 nt\n\t"
        "global_load_lds_dwordx4 %2, %8 offset:1024 nt\n\t"
        "s_mov_b32 m0, %5\n\t"
        "s_mov_b32 exec_hi, 1\n\t"   // 33 lanes (exec_lo is all ones)
        "global_load_lds_dwordx4 %2, %9 offset:0 nt\n\t"
        "s_mov_b64 exec, 3\n\t"
        "s_mov_b32 m0, %4\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %2, %8 offset:2048 nt\n\t"
        "s_mov_b64 exec, %11\n\t"
        "s_mov_b32 m0, %6\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %2, %10 offset:0\n\t"
        SMAX_ASM_INFO
        "s_mov_b64 exec, -1\n\t"   // (issued with every lane active)
        "s_mov_b32 m0, %0"
        : "=&s"(keep), "=&s"(ex)
        : "v"(v16), "v"(v4), "s"(wl), "s"(wp), "s"(wv), "s"(iaddr), "s"(lb), "s"(pb), "s"(vb),
          "s"(vmask), "s"(ib), "i"(3), "i"(0)
        : "memory");
    } else if (SMAX_DBG(a) & (1u << 25)) {
    // diagnostic ablation (diagnostic kernel only; records are wrong): the
    // tile's LCP rows [l0, l0+TILE) aligned, without the two halo pieces
    // and their extra 128-B lines -- the FETCH_SIZE and time they cost
    const uint8_t *la = uni_ptr(a.lcp + l0);
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %4\n\t"
        "s_mov_b64 %1, exec\n\t"
        "global_load_lds_dwordx4 %2, %8 offset:0\n\t"
        "global_load_lds_dwordx4 %2, %8 offset:1024\n\t"
        "s_mov_b32 m0, %5\n\t"
        "s_mov_b64 exec, %14\n\t"
        "global_load_lds_dwordx4 %2, %9 offset:0\n\t"
        "s_mov_b64 exec, %11\n\t"
        "s_mov_b32 m0, %6\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %2, %10 offset:0\n\t"
        SMAX_ASM_INFO
        "s_mov_b64 exec, %1\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep), "=&s"(ex)
        : "v"(v16), "v"(v4), "s"(wl + SMAX_LH), "s"(wp), "s"(wv), "s"(iaddr), "s"(la), "s"(pb), "s"(vb),
          "s"(vmask), "s"(ib), "i"(3), "s"(p2mask)
        : "memory");
    } else {
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %4\n\t"
        "global_load_lds_dwordx4 %2, %8 offset:0\n\t"
        "global_load_lds_dwordx4 %2, %8 offset:1024\n\t"
        "s_mov_b32 m0, %5\n\t"
        "s_mov_b32 exec_hi, 1\n\t"   // 33 lanes (exec_lo is all ones)
        "global_load_lds_dwordx4 %2, %9 offset:0\n\t"
        "s_mov_b64 exec, 3\n\t"
        "s_mov_b32 m0, %4\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %2, %8 offset:2048\n\t"
        "s_mov_b64 exec, %11\n\t"
        "s_mov_b32 m0, %6\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %2, %10 offset:0\n\t"
        SMAX_ASM_INFO
        "s_mov_b64 exec, -1\n\t"   // (issued with every lane active)
        "s_mov_b32 m0, %0"
        : "=&s"(keep), "=&s"(ex)
        : "v"(v16), "v"(v4), "s"(wl), "s"(wp), "s"(wv), "s"(iaddr), "s"(lb), "s"(pb), "s"(vb),
          "s"(vmask), "s"(ib), "i"(3), "i"(0)
        : "memory");
    }
    return;
  }
  const uint8_t *lb = uni_ptr(a.lcp + l0 - SMAX_LH);
  const uint8_t *pb = uni_ptr(reinterpret_cast<const uint8_t *>(a.bwtpk + l0 / 16));
  if constexpr (NT) {
  asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %4\n\t"
        "s_mov_b64 %1, exec\n\t"
        "global_load_lds_dwordx4 %2, %8 offset:0 nt\n\t"
        "global_load_lds_dwordx4 %2, %8 offset:1024 nt\n\t"
        "s_mov_b32 m0, %5\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %2, %9 offset:0 nt\n\t"
        "s_mov_b64 exec, 3\n\t"
        "global_load_lds_dwordx4 %2, %9 offset:1024 nt\n\t"
        "s_mov_b32 m0, %4\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %2, %8 offset:2048 nt\n\t"
        "s_mov_b64 exec, %11\n\t"
        "s_mov_b32 m0, %6\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %2, %10 offset:0\n\t"
        SMAX_ASM_INFO
        "s_mov_b64 exec, %1\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep), "=&s"(ex)
        : "v"(v16), "v"(v4), "s"(wl), "s"(wp), "s"(wv), "s"(iaddr), "s"(lb), "s"(pb), "s"(vb),
          "s"(vmask), "s"(ib), "i"(3)
        : "memory");
  } else {
  asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %4\n\t"
        "s_mov_b64 %1, exec\n\t"
        "global_load_lds_dwordx4 %2, %8 offset:0\n\t"
        "global_load_lds_dwordx4 %2, %8 offset:1024\n\t"
        "s_mov_b32 m0, %5\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %2, %9 offset:0\n\t"
        "s_mov_b64 exec, 3\n\t"
        "global_load_lds_dwordx4 %2, %9 offset:1024\n\t"
        "s_mov_b32 m0, %4\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %2, %8 offset:2048\n\t"
        "s_mov_b64 exec, %11\n\t"
        "s_mov_b32 m0, %6\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %2, %10 offset:0\n\t"
        SMAX_ASM_INFO
        "s_mov_b64 exec, %1\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep), "=&s"(ex)
        : "v"(v16), "v"(v4), "s"(wl), "s"(wp), "s"(wv), "s"(iaddr), "s"(lb), "s"(pb), "s"(vb),
          "s"(vmask), "s"(ib), "i"(3)
        : "memory");
  }
}

__device__ __forceinline__ uint32_t seg_ge(const uint4 v, uint32_t mf) {
  return bytes_ge(v.x, mf) | bytes_ge(v.y, mf) | bytes_ge(v.z, mf) | bytes_ge(v.w, mf);
}
__device__ __forceinline__ uint32_t seg_ffcount(const uint4 v) {
  // flags at bits 7,15,23,31 of each word: merge the four words, one popcount
  return __popc((bytes_ff(v.x) >> 7) | (bytes_ff(v.y) >> 6) | (bytes_ff(v.z) >> 5) |
                (bytes_ff(v.w) >> 4));
}


__device__ __forceinline__ uint32_t bytes_lt(uint32_t x, uint32_t y) {   // x < y
  const uint32_t H = 0x80808080u;
  const uint32_t d = (x | H) - (y & ~H);      // per byte 128 + xl - yl, no borrow
  return (~x & y & H) | (~(x ^ y) & H & ~d);
}
// 4 byte-flags (bits 7,15,23,31) -> 4 consecutive bits
__device__ __forceinline__ uint32_t pack4(uint32_t m) {
  return (((m >> 7) * 0x00204081u) >> 21) & 0xfu;
}

// four byte-flag words (bits 7,15,23,31; word k = rows 4k..4k+3) -> 16-bit
// row mask: dot products of the flag bytes with weights 2^q (VALU dot4)
__device__ __forceinline__ uint32_t pack16(const uint32_t f[4]) {
  const uint32_t lo = __builtin_amdgcn_udot4(f[1], 0x80402010u, __builtin_amdgcn_udot4(f[0], 0x08040201u, 0u, false), false);
  const uint32_t hi = __builtin_amdgcn_udot4(f[3], 0x80402010u, __builtin_amdgcn_udot4(f[2], 0x08040201u, 0u, false), false);
  return (lo >> 7) | (hi << 1);
}

__device__ __forceinline__ uint64_t lanemask_lt() {
  return (1ull << (threadIdx.x & 63)) - 1;
}

__device__ __forceinline__ uint32_t llv_by_rank(const Win &t, uint32_t r) {
  if (t.staged_all) return t.val16[min((int) r, t.nval - 1)];
  if ((int) r < t.nval) return t.val16 != nullptr ? t.val16[r] : t.val[r];
  const KArgs k = kargs();
  if (t.llv_base + r >= k->numllv) { atomicOr(k->err, SMAX_ERR_LLV); return 255; }
  return llv_value(&k->llv[t.llv_base + r]);
}

// rank of window offset o among the window's 255 bytes (t.rank staged)
__device__ __forceinline__ uint32_t rank_at(const Win &t, uint32_t o) {
  const uint32_t chunk = o >> 4, within = o & 15;
  const uint4 v = lds_ld16(&t.L[chunk * 16]);
  const uint64_t lo = (uint64_t) bytes_ff(v.x) | ((uint64_t) bytes_ff(v.y) << 32);
  const uint64_t hi = (uint64_t) bytes_ff(v.z) | ((uint64_t) bytes_ff(v.w) << 32);
  const uint32_t cnt = within < 8 ? __popcll(lo & ((1ull << (8 * within)) - 1))
                                  : __popcll(lo) + __popcll(hi & ((1ull << (8 * (within - 8))) - 1));
  return t.rank[chunk] + cnt;
}

// diversity of BWT rows [lo, hi] (pairwise distinct symbols < 254)
__device__ __forceinline__ bool diverse_rows(const Win &t, uint64_t lo, uint64_t hi) {
  Seen s = {0, 0, 0, 0};
  for (uint64_t g = lo; g <= hi; g++)
    if (seen_add(s, bwt_at(t, g))) return false;
  return true;
}

// left diversity of the first w (2..8) symbols of X: symbols < 254 pairwise
// distinct
__device__ __forceinline__ bool diverse8(uint64_t X, uint32_t w) {
  for (uint32_t m = 1; m < w; m++) {
    const uint32_t x = (uint32_t) (X >> (8 * m)) & 0xffu;
    if (x >= 254) continue;
    const uint64_t hit = bytes_eq64(X, x * 0x0101010101010101ull) &
                         (0x8080808080808080ull >> (8 * (8 - m)));
    if (hit != 0) return false;
  }
  return true;
}

// left diversity of the first w (2..8) rows of a packed-BWT window given as
// 8-bit fields (bit k: row k): code low plane, code high plane, special mask;
// non-special rows are pairwise distinct iff each of the 4 codes occurs at
// most once (no 8-symbol byte expansion)
__device__ __forceinline__ bool diverse_planes(uint32_t lo, uint32_t hi, uint32_t sp, uint32_t w) {
  const uint32_t ns = ~sp & ((1u << w) - 1u);
  const uint32_t c0 = ns & ~lo & ~hi, c1 = ns & lo & ~hi, c2 = ns & ~lo & hi, c3 = ns & lo & hi;
  return ((c0 & (c0 - 1u)) | (c1 & (c1 - 1u)) | (c2 & (c2 - 1u)) | (c3 & (c3 - 1u))) == 0u;
}

// Exact evaluation of one plateau start (row offset `ro` inside the tile, its
// .llv rank `rk` when its LCP byte is 255): *cur = LCP value, *j = last row of
// the plateau; returns whether [c-1 .. j] is a supermaximal-repeat interval.
// Interior tiles take the fast path (start value, plateau of <= 7 rows and
// diversity over <= 8 BWT symbols from two 8-byte LDS windows, one LDS round
// trip; a plateau in an interior tile never reaches `end` within them);
// everything else the exact generic path, which also records the pending
// plateau at the shard end.  A 255-byte start whose predecessor is also 255
// is only a start if its exact value is larger (checked here).
__device__ static bool eval_start(const Win &t, const SmaxScanArgs &a, uint64_t g0,
                                  const uint8_t *sL, uint32_t ro, uint32_t rk, bool interior,
                                  uint32_t *curo, uint64_t *jo) {
  const uint64_t cc = g0 + ro;
  bool acc = false, slow = !interior;
  uint32_t cur = 0;
  uint64_t j = cc;
  if (interior) {
    const uint32_t co = SMAX_LH + ro;
    const uint64_t LX = lds_bytes8(sL, co);
    // BWT symbols of rows c-1 .. c+6: bit planes (packed window) or bytes
    uint64_t BX = 0;
    uint32_t plo = 0, phi = 0, psp = 0;
    if (t.B == nullptr) {   // packed window (K1 sets B = nullptr: folds at compile time)
      const uint32_t o = co - 1, gi = o >> 4, q = o & 15u;
      const uint64_t w0 = pk_word(t, gi), w1 = pk_word(t, gi + 1);
      const uint32_t a0 = (uint32_t) w0, a1 = (uint32_t) w1;
      plo = (((a0 & 0xffffu) | (a1 << 16)) >> q) & 0xffu;
      phi = (((a0 >> 16) | (a1 & 0xffff0000u)) >> q) & 0xffu;
      psp = ((uint32_t) (((w0 >> 32) & 0xffffu) | (((w1 >> 32) & 0xffffu) << 16)) >> q) & 0xffu;
    } else {
      BX = lds_bytes8(t.B, co - 1);
    }
    auto div = [&](uint32_t w) {
      return t.B == nullptr ? diverse_planes(plo, phi, psp, w) : diverse8(BX, w);
    };
    const uint32_t cb = (uint32_t) LX & 0xffu;
    if (cb == 255) {
      // .llv start: exact values by rank; a run of equal values >= 255
      // is a run of 255 bytes, so its ranks are consecutive
      if (t.rank == nullptr) {
        slow = true;
      } else {
        const uint32_t v = llv_by_rank(t, rk);
        const bool start = sL[co - 1] != 255 || llv_by_rank(t, rk - 1) < v;
        if (start && v >= a.minlen) {
          cur = v;
          uint32_t k = 0;
          int rel = 0;
          for (; k < 7; k++) {
            const uint32_t nb = (uint32_t) (LX >> (8 * (k + 1))) & 0xffu;
            if (nb != 255) { rel = -1; break; }
            const uint32_t nv = llv_by_rank(t, rk + k + 1);
            if (nv != v) { rel = nv < v ? -1 : 1; break; }
          }
          if (rel == 0) {
            slow = true;
          } else {
            j = cc + k;
            if (rel < 0) acc = div(k + 2);
          }
        }
      }
    } else if (cb >= a.minlen) {
      cur = cb;
      const uint64_t nx = LX >> 8;
      const uint64_t ne = ~bytes_eq64(nx, cb * 0x0101010101010101ull) &
                          0x0080808080808080ull;
      if (ne == 0) {
        slow = true;
      } else {
        const uint32_t k = (uint32_t) __builtin_ctzll(ne) >> 3;
        const uint32_t nb = (uint32_t) (nx >> (8 * k)) & 0xffu;
        j = cc + k;
        if (nb < cb) acc = div(k + 2);
      }
    }
  }
  if (slow && !(SMAX_DBG(a) & 32u)) {
    acc = false;
    cur = lcp_exact(t, cc);
    const bool start = !interior || lcp_exact(t, cc - 1) < cur;
    if (start && cur >= a.minlen) {
      int rel;
      bool pend;
      j = plateau_end(t, cc, cur, &rel, &pend);
      if (pend) {
        Seen sn = {0, 0, 0, 0};
        bool dup = false;
        for (uint64_t g = cc - 1; g < a.end && !dup; g++) dup = seen_add(sn, bwt_at(t, g));
        if (!dup) {
          GtSmaxBoundary *b = a.bnd;
          b->pend_c = cc;
          b->pend_lcp = cur;
          b->pend_div.seen[0] = sn.w0; b->pend_div.seen[1] = sn.w1;
          b->pend_div.seen[2] = sn.w2; b->pend_div.seen[3] = sn.w3;
          b->pend_div.dup = 0;
          b->pend_valid = 1;
        }
      } else if (rel < 0) {
        acc = diverse_rows(t, cc - 1, j);
      }
    }
  }
  *curo = cur;
  *jo = j;
  return acc;
}

// ---- interior tiles: SWAR classification of every plateau start
//
// Most supermaximal-repeat intervals are two rows wide (a plateau of one
// row: LCP[c-1] < LCP[c] > LCP[c+1]); their whole predicate is byte-local, so
// each lane decides them for its 16 rows with SWAR compares on the LCP bytes
// c-1, c, c+1 and the BWT bytes c-1, c ("D" rows).  Only starts that need
// exact values or a longer scan -- a 255 LCP byte (.llv value), or a plateau
// of >= 2 rows (LCP[c+1] == LCP[c]) -- are queued ("L" rows) and evaluated
// exactly, 64 at a time (eval_start).  Records are then written in row
// order by their owning lanes.
#define SMAX_DLIST 56                                 // queued exact starts per tile


// high bit of each byte >= 254 (WILDCARD / SEPARATOR / UNDEFBWTCHAR)
__device__ __forceinline__ uint32_t bytes_sp(uint32_t w) { return bytes_ff(w | 0x01010101u); }


// Left diversity of the 16 rows c of segment `so` for the two interval
// shapes decided here: *div2 = {BWT[c-1], BWT[c]} pairwise distinct (specials
// unique), *div3 = {BWT[c-1], BWT[c], BWT[c+1]} pairwise distinct.
__device__ __forceinline__ void segment_div(const Win &t, uint32_t so, uint32_t *div2,
                                            uint32_t *div3) {
  if (t.B == nullptr) {   // packed window
    const uint64_t w = pk_word(t, so >> 4), pw = pk_word(t, (so >> 4) - 1), nw = pk_word(t, (so >> 4) + 1);
    // both code planes at once (low plane bits 0..15, high plane 16..31)
    const uint32_t c = (uint32_t) w, pc = (uint32_t) pw, nc = (uint32_t) nw;
    const uint32_t sp = (uint32_t) (w >> 32) & 0xffffu;
    const uint32_t spm1 = ((sp << 1) | ((uint32_t) (pw >> 47) & 1u)) & 0xffffu;   // row q-1
    const uint32_t spp1 = (sp >> 1) | (((uint32_t) (nw >> 32) & 1u) << 15);       // row q+1
    const uint32_t cp = ((c << 1) & 0xfffefffeu) | ((pc >> 15) & 0x00010001u);   // row q-1
    const uint32_t cn = ((c >> 1) & 0x7fff7fffu) | ((nc << 15) & 0x80008000u);   // row q+1
    const uint32_t x1 = c ^ cp, x1n = c ^ cn, x2 = cp ^ cn;
    const uint32_t ne1 = (x1 | (x1 >> 16)) & 0xffffu;        // q-1 vs q
    const uint32_t ne1n = (x1n | (x1n >> 16)) & 0xffffu;     // q vs q+1
    const uint32_t ne2 = (x2 | (x2 >> 16)) & 0xffffu;        // q-1 vs q+1
    const uint32_t d2 = ne1 | sp | spm1;
    *div2 = d2;
    *div3 = d2 & (ne1n | sp | spp1) & (ne2 | spm1 | spp1);
    return;
  }
  const uint4 bv = lds_ld16(&t.B[so]);
  const uint32_t bp = t.B[so - 1], bn = t.B[so + 16];
  uint32_t r2 = 0, r3 = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t bc = k == 0 ? bv.x : k == 1 ? bv.y : k == 2 ? bv.z : bv.w;
    const uint32_t bpv = k == 0 ? ((bv.x << 8) | bp)
                       : __builtin_amdgcn_alignbyte(bc, k == 1 ? bv.x : k == 2 ? bv.y : bv.z, 3);
    const uint32_t bnx = k == 3 ? ((bv.w >> 8) | (bn << 24))
                       : __builtin_amdgcn_alignbyte(k == 0 ? bv.y : k == 1 ? bv.z : bv.w, bc, 1);
    const uint32_t sc = bytes_sp(bc), sp = bytes_sp(bpv), sn = bytes_sp(bnx);
    const uint32_t d2 = ~bytes_eq(bpv, bc) | sc | sp;
    const uint32_t d3 = d2 & (~bytes_eq(bnx, bc) | sc | sn) & (~bytes_eq(bnx, bpv) | sp | sn);
    r2 |= pack4(d2 & 0x80808080u) << (4 * k);
    r3 |= pack4(d3 & 0x80808080u) << (4 * k);
  }
  *div2 = r2;
  *div3 = r3;
}

// Classification of the 16 rows c of segment `so`:
//   *Dm  records [c-1 .. c] and [c-1 .. c+1] (D3 marks the latter): start,
//        then LCP[c+1] < LCP[c], or LCP[c+1] == LCP[c] > LCP[c+2]; with the
//        matching left diversity
//   *Lm  starts needing exact evaluation: plateaus of >= 3 rows (LCP[c] ==
//        LCP[c+1] == LCP[c+2])
//   *Fm  255 bytes (ranks)
// where start = LCP[c] >= minlen (exact for minlen <= 128) and LCP[c] >
// LCP[c-1].  Only two relations are computed, each row against its
// predecessor (UP: LCP[r-1] < LCP[r], EQ: LCP[r-1] == LCP[r]) for rows
// 0..17; successor relations are the same bits shifted.  Byte compares are
// exact except between two 255 bytes: those pairs (rare) are re-decided
// from the exact .llv values by rank (crank = 255 bytes before the segment).
struct SegRel {
  uint32_t UP, EQ, GE, FF, F18, pb;
};

// Part 1: the relations of rows 0..17 of segment `so` to their predecessors
// (byte compares), the >= min(minlen,128) filter and the 255 bytes.
__device__ __forceinline__ void classify_rel(const Win &t, uint32_t so, uint32_t mf, SegRel &r) {
  const LDSP uint8_t *L = t.L;
  const uint4 v = lds_ld16(&L[so]);
  const uint32_t pb = L[so - 1], nb = L[so + 16], nb2 = L[so + 17];
  const uint32_t w0 = v.x, w1 = v.y, w2 = v.z, w3 = v.w;
  uint32_t up[4], eq[4], ge[4], ff[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t cur = k == 0 ? w0 : k == 1 ? w1 : k == 2 ? w2 : w3;
    const uint32_t prv = k == 0 ? ((w0 << 8) | pb)
                       : __builtin_amdgcn_alignbyte(cur, k == 1 ? w0 : k == 2 ? w1 : w2, 3);
    up[k] = bytes_lt(prv, cur);
    eq[k] = bytes_eq(prv, cur);
    ge[k] = bytes_ge(cur, mf);
    ff[k] = bytes_ff(cur);
  }
  r.UP = pack16(up);
  r.EQ = pack16(eq);
  r.GE = pack16(ge);
  r.FF = pack16(ff);
  // rows 16, 17 against their predecessors
  const uint32_t b15 = w3 >> 24;
  r.UP |= (b15 < nb ? 1u << 16 : 0u) | (nb < nb2 ? 1u << 17 : 0u);
  r.EQ |= (b15 == nb ? 1u << 16 : 0u) | (nb == nb2 ? 1u << 17 : 0u);
  r.F18 = r.FF | (nb == 255u ? 1u << 16 : 0u) | (nb2 == 255u ? 1u << 17 : 0u);
  r.pb = pb;
}

// Per tile, once a classification step meets a 255-after-255 row: the
// relations of every staged .llv value to its predecessor in rank order, as
// bit masks (bit r of GT: value(r) > value(r-1), of EQ: equal; r < 256) in
// the wave's LDS scratch -- four 64-rank ballot rounds.  Each segment then
// reads its 18 relations with two LDS dwords and a funnel shift per mask.
// ffp_resolve funnels words crank >> 5 and the one after it of each set of 8
// (for crank >= 224 the word after is the next set's first, or the word past
// the masks); the bits it uses are those of ranks < nval <= SMAX_LLV_CAP, so
// they all come from the set's own 8 words while SMAX_LLV_CAP <= 256 -- the
// word after only supplies bits of ranks >= 256, which no row reads
static_assert(SMAX_LLV_CAP <= 256, "rank relation masks: 8 words per set cover every rank");
__device__ __forceinline__ void ffp_masks(const Win &t, LDSP uint32_t *relm) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int r = 64 * j + lane;
    bool gt = false, eq = false;
    if (r >= 1 && r < t.nval) {
      const uint32_t v = t.val16[r], vp = t.val16[r - 1];
      gt = v > vp;
      eq = v == vp;
    }
    const uint64_t g = __ballot(gt), e = __ballot(eq);
    if (lane == 0) {
      relm[2 * j] = (uint32_t) g;
      relm[2 * j + 1] = (uint32_t) (g >> 32);
      relm[8 + 2 * j] = (uint32_t) e;
      relm[8 + 2 * j + 1] = (uint32_t) (e >> 32);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// UP/EQ of the rows q in FFP (255 bytes after 255 bytes) from the rank
// relation masks (ffp_masks): bit k of gtm/eqm = rank crank+k vs crank+k-1,
// and rank index k maps back to row q: k = 255 bytes of the segment before
// q -- a plain shift when the segment's 255 bytes are one run (dense .llv
// regions), otherwise one register-only step per row.  Replaces a loop of
// two dependent LDS reads per row (a quarter of K1 on the 12 Gbp plant
// genome, whose long repeat families are dense in .llv values).
__device__ __forceinline__ void ffp_resolve(const LDSP uint32_t *relm, uint32_t F18, uint32_t FFP,
                                            uint32_t crank, uint32_t *UP, uint32_t *EQ) {
  const uint32_t wi = crank >> 5, sh = crank & 31u;
  const uint32_t gtm = __builtin_amdgcn_alignbit(relm[wi + 1], relm[wi], sh);
  const uint32_t eqm = __builtin_amdgcn_alignbit(relm[8 + wi + 1], relm[8 + wi], sh);
  uint32_t up = 0, eqr = 0;
  const uint32_t low = F18 & (0u - F18);
  if ((F18 & (F18 + low)) == 0) {                               // one run from row q0
    const uint32_t q0 = (uint32_t) __builtin_ctz(F18);
    up = gtm << q0;
    eqr = eqm << q0;
  } else {
    uint32_t m = FFP;
    while (m) {
      const uint32_t q = (uint32_t) __builtin_ctz(m);
      m &= m - 1;
      const uint32_t k = (uint32_t) __popc(F18 & ((1u << q) - 1));
      up |= ((gtm >> k) & 1u) << q;
      eqr |= ((eqm >> k) & 1u) << q;
    }
  }
  *UP = (*UP & ~FFP) | (up & FFP);
  *EQ = (*EQ & ~FFP) | (eqr & FFP);
}

// Part 2, given the rank of the segment's first row among the window's 255
// bytes (crank):
//   *Dm  records [c-1 .. c] and [c-1 .. c+1] (D3 marks the latter): start,
//        then LCP[c+1] < LCP[c], or LCP[c+1] == LCP[c] > LCP[c+2]; with the
//        matching left diversity
//   *Lm  starts needing exact evaluation: plateaus of >= 3 rows (LCP[c] ==
//        LCP[c+1] == LCP[c+2])
// where start = LCP[c] >= minlen (exact for minlen <= 128) and LCP[c] >
// LCP[c-1].  Only two relations are computed, each row against its
// predecessor (UP, EQ) for rows 0..17; successor relations are the same bits
// shifted.  Byte compares are exact except between two 255 bytes: those
// pairs (rare) are re-decided from the exact .llv values by rank.
template <bool FFPV>
__device__ __forceinline__ void classify_fin(const Win &t, uint32_t so, SegRel r, uint32_t crank,
                                             bool all_exact, uint32_t *Dm, uint32_t *D3m,
                                             uint32_t *Lm, const LDSP uint32_t *relm = nullptr) {
  uint32_t UP = r.UP, EQ = r.EQ;
  uint32_t FFP = r.F18 & ((r.F18 << 1) | (r.pb == 255u ? 1u : 0u));    // 255 after 255
  bool unresolved = false;
  // (the rank tests first: wave-uniform, so a tile without .llv values skips
  // the per-row loop's exec bookkeeping)
  if (t.rank == nullptr) {
    unresolved = r.F18 != 0;                // no ranks (inconsistent index): exact queue
  } else if (FFPV && t.staged_all) {
    if (FFP != 0) ffp_resolve(relm, r.F18, FFP, crank, &UP, &EQ);
  } else {
    while (FFP) {
      const int q = __builtin_ctz(FFP);
      FFP &= FFP - 1;
      const uint32_t rk = crank + (uint32_t) __popc(r.F18 & ((1u << q) - 1));
      const uint32_t vr = llv_by_rank(t, rk), vp = llv_by_rank(t, rk - 1);
      UP = (UP & ~(1u << q)) | ((vp < vr ? 1u : 0u) << q);
      EQ = (EQ & ~(1u << q)) | ((vp == vr ? 1u : 0u) << q);
    }
  }
  const uint32_t A = r.GE & (UP | (unresolved ? r.FF & ((r.FF << 1) | (r.pb == 255u ? 1u : 0u)) : 0u))
                     & 0xffffu;
  const uint32_t eqn = EQ >> 1, dn = ~((UP | EQ) >> 1);            // vs row c+1
  const uint32_t eqn1 = EQ >> 2, dn1 = ~((UP | EQ) >> 2);          // c+1 vs c+2
  const uint32_t D = A & dn & 0xffffu;
  const uint32_t D3 = A & eqn & dn1 & 0xffffu;
  // (the early exit pays for its exec bookkeeping on the plant genome, whose
  // active segments often hold no start: profiles/s5/output_loop_ab_*.txt)
  if (A == 0) {
    *Dm = 0;
    *D3m = 0;
    *Lm = 0;
    return;
  }
  // left diversity of rows (c-1, c) and (c-1, c, c+1): every interval
  // [c-1 .. j] needs the first, every plateau of >= 3 rows the second, so
  // the exact queue only receives starts that can still be accepted (on
  // repeat-rich DNA most plateau starts share their left symbols)
  uint32_t div2, div3;
  segment_div(t, so, &div2, &div3);
  if (all_exact || unresolved) {
    *Lm = A & div2;
    *Dm = 0;
    *D3m = 0;
  } else {
    *Lm = A & eqn & eqn1 & div3;
    *Dm = (D & div2) | (D3 & div3);
    *D3m = D3 & div3;
  }
}

// exclusive prefix over the wave's lanes and total of a per-lane count:
// DPP inclusive scan (row_shr 1/2/4/8 inside each 16-lane row, then
// row_bcast 15/31 across rows) -- VALU only, no ballots or scalar popcounts
__device__ __forceinline__ uint32_t wave_excl(uint32_t c, uint32_t *tot) {
  int x = (int) c;
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);   // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);   // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);   // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);   // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);   // row_bcast:15
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);   // row_bcast:31
  // (opaque to the optimiser: otherwise x - c is rewritten as the sum of the
  // five shifted partials, which keeps them live and splits every step into
  // a DPP move and an add -- ~15 more VALU per scan)
  asm("" : "+v"(x));
  *tot = (uint32_t) __builtin_amdgcn_readlane(x, 63);
  return (uint32_t) x - c;
}

// Returns the tile's record count, or UINT32_MAX when more than SMAX_DLIST
// starts need exact evaluation (the caller then runs wave_detect).
// Only the tile's 16-row segments holding a byte >= min(minlen,128) are
// classified: they are compacted (row order) so that each classification
// step keeps all 64 lanes busy (about a third of the segments are active on
// repeat-rich DNA, so one step usually covers the whole tile).
template <int DL, bool FFPV>
__device__ static uint32_t wave_detect_direct(const Win &t, const SmaxScanArgs &a, uint64_t g0,
                                              const uint8_t *sL, uint32_t *ent,
                                              uint64_t *stg, uint32_t segpre,
                                              SmaxStamps *st = nullptr) {
  const int lane = threadIdx.x & 63;
  const uint32_t mf = a.minlen < 128 ? a.minlen : 128;
  const bool all_exact = a.minlen > 128;
  // the staged records live in the window's BWT region, dead once the
  // starts are evaluated (nothing after reads BWT symbols); the next DMA
  // into this window is issued after the records have moved to registers
  // (smax_scan_body)
  // results packed into the queue entries (lane i reads entry i, then
  // writes result i): LCP value (16 bits) | width << 16; a larger value or
  // width sends the tile to K1b.  Which starts were accepted is one wave
  // ballot over the queue (queue index = lane), so the output finds its
  // position without a third scan or per-segment LDS masks.
  uint32_t *res = ent;
  // the dense variant's rank relation masks (ffp_masks): 16 words after the queue
  uint32_t *accw = ent + DL;
  // compact the active segments (id = round * 64 + lane, row order): the
  // k-th active segment goes to step k / 64, lane k % 64.  Two forward
  // permutes (ds_permute_b32: no LDS memory, one round trip) instead of an
  // LDS list written and read back: lane d0 receives the d0-th active
  // first-half segment; the second-half ones go to lanes (n0 + j) mod 64
  // (step 0 for n0 + j < 64, step 1 otherwise -- one lane never holds both,
  // n1 <= 64).  Inactive segments fill the other lanes, so each permute is a
  // bijection.
  const uint64_t m0 = __ballot(segpre & 1u), m1 = __ballot((segpre >> 1) & 1u);
  const uint32_t n0 = (uint32_t) __popcll(m0), n1 = (uint32_t) __popcll(m1), nseg = n0 + n1;
  const bool a0 = (segpre & 1u) != 0, a1 = (segpre & 2u) != 0;
  // active lanes below this one (mbcnt: two VALU, no branch); the inactive
  // ones below are the rest of the lanes below
  const uint32_t c0 = __builtin_amdgcn_mbcnt_hi((uint32_t) (m0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t) m0, 0u));
  const uint32_t c1 = __builtin_amdgcn_mbcnt_hi((uint32_t) (m1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t) m1, 0u));
  const uint32_t d0 = a0 ? c0 : n0 + (uint32_t) lane - c0;
  const uint32_t d1 = (a1 ? n0 + c1 : n0 + n1 + (uint32_t) lane - c1) & 63u;
  const uint32_t segA = (uint32_t) __builtin_amdgcn_ds_permute((int) (d0 * 4u), lane);
  const uint32_t segB = (uint32_t) __builtin_amdgcn_ds_permute((int) (d1 * 4u), 64 + lane);
  // per step: D = decided records (2 or 3 rows), W3 = the 3-row ones; set
  // for every step k < nsteps and read only there (no zero-fill: each
  // initialiser was a per-tile VALU move, and VALU issue bounds K1)
  uint32_t Dm0, Lm0, Dm1, Lm1, Lpre0, Lpre1, Dpre0, Dpre1, ro0, ro1;
  uint32_t W30, W31, F0, F1, R0, R1;
  uint32_t nL = 0, nD = 0;
  const uint32_t nsteps = (nseg + 63) >> 6;      // 1 or 2
  // 255-byte ranks: the left halo's count, then a prefix over the compacted
  // segments in row order (an inactive segment holds no byte >= 128)
  uint32_t fbase = 0;
  LDSP SmaxRank *rank = const_cast<LDSP SmaxRank *>(t.rank);
  // dense variant: the rank relation masks in the accepted-mask scratch
  // (free until the exact evaluation), built at the first step that needs
  // them (ffp_masks)
  LDSP uint32_t *relm = (LDSP uint32_t *) accw;
  bool relm_ready = false;
  if (rank != nullptr) fbase = t.halo_ff;   // plan time (llv_win): the halo's 255 bytes
#pragma unroll
  for (int k = 0; k < 2; k++) {
    if ((uint32_t) k >= nsteps) break;
    const uint32_t i = k * 64 + lane;
    uint32_t D = 0, D3 = 0, Lq = 0;
    // every lane classifies a segment (no exec-mask bookkeeping): lanes
    // past the active ones hold an inactive segment or, in the second step,
    // one the first step already took -- their masks are cleared, so they
    // add no start, record or rank, and their rank entry goes to the left
    // halo chunk (set after the steps)
    const bool act = i < nseg;
    const uint32_t sid = (k == 0 && (uint32_t) lane < n0) ? segA : segB;
    const uint32_t ro = (sid >> 6) * 1024 + (sid & 63) * 16;   // segment's first row in the tile
    SegRel rel;
    classify_rel(t, SMAX_LH + ro, mf, rel);
    rel.GE = act ? rel.GE : 0u;
    rel.FF = act ? rel.FF : 0u;
    rel.F18 = act ? rel.F18 : 0u;
    uint32_t crank = 0;
    if (rank != nullptr) {
      uint32_t ftot;
      crank = fbase + wave_excl((uint32_t) __popc(rel.FF), &ftot);
      rank[act ? (SMAX_LH + ro) >> 4 : 0u] = (SmaxRank) crank;
      fbase += ftot;
    }
    if constexpr (FFPV) {
      const uint32_t ffp = rel.F18 & ((rel.F18 << 1) | (rel.pb == 255u ? 1u : 0u));
      if (!relm_ready && rank != nullptr && __ballot(ffp != 0) != 0) {
        ffp_masks(t, relm);
        relm_ready = true;
      }
    }
    // every row is owned: tiles holding rows before `begin` are static K1b
    classify_fin<FFPV>(t, SMAX_LH + ro, rel, crank, all_exact, &D, &D3, &Lq, relm);
    const uint32_t F = rel.FF;
    // one scan for the queue positions (low half) and the decided records
    // before this lane (high half): <= 1024 each, no carry between them
    uint32_t tot2;
    const uint32_t excl2 = wave_excl((uint32_t) __popc(Lq) | ((uint32_t) __popc(D) << 16), &tot2);
    const uint32_t excl = excl2 & 0xffffu, tot = tot2 & 0xffffu;
    if (nL + tot <= DL) {
      // queue entry: row in the tile (11 bits) | its .llv rank << 18
      uint32_t pos = nL + excl, bits = Lq;
      while (bits) {
        const int q = __builtin_ctz(bits);
        bits &= bits - 1;
        const uint32_t rk = ((F >> q) & 1u) ? crank + (uint32_t) __popc(F & ((1u << q) - 1)) : 0u;
        ent[pos++] = (ro + (uint32_t) q) | (rk << 18);
      }
    }
    if (k == 0) { Dm0 = D; W30 = D3; F0 = F; R0 = crank; Lm0 = Lq; Lpre0 = nL + excl; Dpre0 = nD + (excl2 >> 16); ro0 = ro; }
    else { Dm1 = D; W31 = D3; F1 = F; R1 = crank; Lm1 = Lq; Lpre1 = nL + excl; Dpre1 = nD + (excl2 >> 16); ro1 = ro; }
    nL += tot;
    nD += tot2 >> 16;
  }
  if (rank != nullptr && lane == 0) {   // halo chunks (ranks of rows the slow paths may read)
    rank[0] = 0;
    rank[1 + SMAX_TILE / 16] = (SmaxRank) fbase;
  }
  SMAX_STAMP(st, 3);
  if (nL > DL) return UINT32_MAX;
  if (SMAX_DBG(a) & 8u) return (Dm0 ^ Dm1 ^ Lm0 ^ Lm1) == 0x12345u ? 1u : 0u;   // ablation: classify only
  // exact evaluation of the queued starts (one per lane); accm: bit i set
  // when queue entry i was accepted
  uint64_t accm = 0;
  if (nL != 0 && !(SMAX_DBG(a) & 4u)) {
    static_assert(DL <= 64, "one exact start per lane");
    const uint32_t i = lane;
    uint32_t cur = 0, width = 0;
    bool acc = false;
    if (i < nL) {
      const uint32_t e = ent[i];
      const uint32_t ro = e & 0x7ffu;
      uint64_t j;
      acc = eval_start(t, a, g0, sL, ro, e >> 18, true, &cur, &j);
      width = (uint32_t) (j - (g0 + ro) + 2);
      res[i] = cur | (width << 16);
    }
    // an accepted record wider than the packed formats hold (the slot's
    // 21-bit width, the result's 16-bit halves): the tile goes to K1b
    // (16-byte records); rejected starts' results are never read
    const bool wide = acc && (width > SMAX_PK_WMAX || (cur | width) >= 65536u);
    if (__ballot(wide) != 0) return UINT32_MAX;
    accm = __ballot(acc);
    // every lane's BWT reads and result writes are done before the staged
    // records (in the window's BWT region) and the result reads below
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  SMAX_STAMP(st, 4);
  // records in row order, written by the owning lanes: a lane's first
  // record follows the decided records of the segments before it (the
  // classification's scan) and the accepted queue entries before its own
  // (the ballot); a tile with more records than its slot holds goes to K1b
  // (the writes past the slot land on its last entry; K1b redoes the tile)
  const uint32_t wcount = nD + (uint32_t) __popcll(accm);
#pragma unroll
  for (int k = 0; k < 2; k++) {
    if ((uint32_t) k >= nsteps) break;
    const uint32_t D = k == 0 ? Dm0 : Dm1, Lq = k == 0 ? Lm0 : Lm1, W3 = k == 0 ? W30 : W31;
    const uint32_t Fk = k == 0 ? F0 : F1, Rk = k == 0 ? R0 : R1;
    const uint32_t Lpre = k == 0 ? Lpre0 : Lpre1, ro = k == 0 ? ro0 : ro1;
    const uint32_t Dpre = k == 0 ? Dpre0 : Dpre1;
    // accepted queue entries before this lane's first (Lpre < 64 when any
    // entry is accepted: the queue holds at most SMAX_DLIST)
    uint32_t pos = Dpre + (uint32_t) __popcll(accm & ((1ull << (Lpre & 63u)) - 1ull)) +
                   (Lpre >= 64u ? (uint32_t) __popcll(accm) : 0u);
    uint32_t bits = D | Lq, qi = Lpre;
    while (bits) {
      const int q = __builtin_ctz(bits);
      bits &= bits - 1;
      uint32_t lcp, width;
      if ((D >> q) & 1u) {
        const uint32_t b = sL[SMAX_LH + ro + q];
        lcp = b < 255 ? b : llv_by_rank(t, Rk + (uint32_t) __popc(Fk & ((1u << q) - 1)));
        width = 2 + ((W3 >> q) & 1u);
      } else {
        const bool ok = qi < 64u && ((accm >> qi) & 1ull);
        const uint32_t i = qi++;
        if (!ok) continue;
        const uint32_t rw = res[i];
        lcp = rw & 0xffffu;
        width = rw >> 16;
      }
      if (!(SMAX_DBG(a) & (4096u | (1u << 21))))
        stg[min(pos, (uint32_t) SMAX_SSLOT - 1u)] = (uint64_t) (ro + q) | ((uint64_t) width << 11) | ((uint64_t) lcp << 32);
      pos++;
    }
  }
  SMAX_STAMP(st, 5);
  return wcount;   // > SMAX_SSLOT: the caller defers the tile
}

// next tile's window + the llv_win entry of the tile after it (ring slot iaddr)
template <bool NT, bool BW2 = false>
__device__ __forceinline__ void issue_next(const SmaxScanArgs &a, uint64_t l0, SmaxWindowPk *w,
                                           uint32_t wl, uint32_t lo, uint32_t n, const uint2 *info,
                                           uint32_t iaddr, uint32_t v16, uint32_t v4) {
  issue_window_pk<NT, BW2>(a, l0, wl, lo, n, info, iaddr, v16, v4);
}
template <bool NT, bool BW2 = false>
__device__ __forceinline__ void issue_next(const SmaxScanArgs &a, uint64_t l0, SmaxWindowB2 *w,
                                           uint32_t wl, uint32_t lo, uint32_t n, const uint2 *info,
                                           uint32_t iaddr, uint32_t v16, uint32_t v4) {
  static_assert(BW2, "SmaxWindowB2 holds the 2-plane form only");
  issue_window_pk<NT, BW2, SmaxWindowB2>(a, l0, wl, lo, n, info, iaddr, v16, v4);
}
template <bool NT, bool BW2 = false>
__device__ __forceinline__ void issue_next(const SmaxScanArgs &a, uint64_t l0, SmaxWindow *w,
                                           uint32_t wl, uint32_t lo, uint32_t n, const uint2 *info,
                                           uint32_t iaddr, uint32_t v16, uint32_t v4) {
  issue_window(a, l0, w, lo, SMAX_WIN_N(n));
  if ((threadIdx.x & 63) < 2) glds4(reinterpret_cast<const uint32_t *>(info) + (threadIdx.x & 63), iaddr);
}

__device__ __forceinline__ void set_bwt_window(Win &t, SmaxWindow *W) { t.B = to_lds<uint8_t>(W->B); t.P = nullptr; }
__device__ __forceinline__ void set_bwt_window(Win &t, SmaxWindowPk *W) { t.P = to_lds<uint64_t>(W->P); t.B = nullptr; }
__device__ __forceinline__ void set_bwt_window(Win &t, SmaxWindowB2 *W) { t.P = to_lds<uint64_t>(W->P); t.B = nullptr; }

// A window's BWT region once the tile's exact starts are evaluated: the
// staged records (SMAX_SSLOT u64); nothing of the tile reads BWT symbols
// after that point, and the wave's next DMA into this window follows the
// move of the records to registers.
__device__ __forceinline__ uint64_t *window_scratch(SmaxWindow *W) {
  return reinterpret_cast<uint64_t *>(W->B);
}
__device__ __forceinline__ uint64_t *window_scratch(SmaxWindowPk *W) { return W->P; }
__device__ __forceinline__ uint64_t *window_scratch(SmaxWindowB2 *W) { return W->P; }

// Filter of a landed window (one wave): per-lane segment "any byte >=
// min(minlen,128)" bits; the .llv values are staged with the window, their
// ranks are computed during the classification (wave_detect_direct).
// rows of segment `so` (16 LCP bytes v) with LCP >= mf whose BWT differs
// from the predecessor's (packed bit-plane window), or any 255 byte
__device__ __forceinline__ bool seg_can_start(const Win &t, const uint4 v, uint32_t so,
                                              uint32_t mf) {
  const uint32_t g[4] = {bytes_ge(v.x, mf), bytes_ge(v.y, mf), bytes_ge(v.z, mf),
                         bytes_ge(v.w, mf)};
  // any 0xff byte: a zero byte of ~w (exact as an any-test)
  const uint32_t ff = ((0xfefefefeu - v.x) & v.x) | ((0xfefefefeu - v.y) & v.y) |
                      ((0xfefefefeu - v.z) & v.z) | ((0xfefefefeu - v.w) & v.w);
  const uint64_t w = pk_word(t, so >> 4), pw = pk_word(t, (so >> 4) - 1);
  const uint32_t c = (uint32_t) w, pc = (uint32_t) pw;
  const uint32_t sp = (uint32_t) (w >> 32) & 0xffffu;
  const uint32_t spm1 = ((sp << 1) | ((uint32_t) (pw >> 47) & 1u)) & 0xffffu;
  const uint32_t cp = ((c << 1) & 0xfffefffeu) | ((pc >> 15) & 0x00010001u);
  const uint32_t x1 = c ^ cp;
  const uint32_t d2 = ((x1 | (x1 >> 16)) & 0xffffu) | sp | spm1;
  return (ff & 0x80808080u) != 0 || (pack16(g) & d2) != 0;
}

__device__ __forceinline__ uint32_t prepare_window(Win &t, const SmaxScanArgs &a, SmaxRank *rank,
                                                   uint32_t wlo, uint32_t wn) {
  const int lane = threadIdx.x & 63;
  const uint32_t mf = a.minlen < 128 ? a.minlen : 128;
  const uint32_t so = SMAX_LH + lane * 16;
  const uint4 v0 = lds_ld16(&t.L[so]);
  const uint4 v1 = lds_ld16(&t.L[so + 1024]);
  uint32_t segpre_bits = (seg_ge(v0, mf) ? 1u : 0u) | (seg_ge(v1, mf) ? 2u : 0u);
  if (t.B == nullptr && !(SMAX_DBG(a) & 1u) &&
      __popcll(__ballot(segpre_bits & 1u)) + __popcll(__ballot(segpre_bits & 2u)) > 64) {
    // more active segments than one classification step holds (packed
    // windows): keep only segments where some row c can start a record --
    // LCP[c] >= min(minlen,128) with BWT[c-1] != BWT[c] (or a special
    // symbol) -- or that hold a 255 byte (the rank prefix of the
    // classification counts the 255 bytes of active segments only)
    if ((segpre_bits & 1u) && !seg_can_start(t, v0, so, mf)) segpre_bits &= ~1u;
    if ((segpre_bits & 2u) && !seg_can_start(t, v1, so + 1024, mf)) segpre_bits &= ~2u;
  }
  t.llv_base = wlo;
  // no .llv entry in the window: no 255 byte (in a consistent index; a
  // stray 255 still resolves exactly through the global .llv search)
  t.rank = wn == 0 ? nullptr : to_lds<SmaxRank>(rank);
  t.nval = -1;
  if (wn != 0) {
    const uint32_t cap = SMAX_LLV_CAP - (wlo & 7u);   // staged from the 8-aligned index below wlo
    t.val16 += wlo & 7u;
    t.nval = (int) (wn < cap ? wn : cap);
  }
  return segpre_bits;
}

// A finished tile's records (lane r holds record r) to its slot with one
// coalesced store, its count, and its share of the 256-tile block sum.
__device__ __forceinline__ void smax_flush_tile(const SmaxScanArgs &a, uint64_t tile, uint64_t rec,
                                                uint32_t cnt) {
  const int lane = threadIdx.x & 63;
  if (SMAX_DBG(a) & 4096u) return;
  if ((uint32_t) lane < cnt && !(SMAX_DBG(a) & (1u << 21))) a.slots[tile * (uint64_t) SMAX_SSLOT + lane] = rec;
  if (lane == 0) {
    if (!(SMAX_DBG(a) & (1u << 22))) a.tile_count[tile] = cnt;
  }
}

// K1 body.  Interior tiles whose starts the direct path covers are finished
// here; shard-edge tiles and tiles with more exact starts than the direct
// path queues are deferred to K1b (their generic path is kept out of K1,
// whose register budget it would otherwise set).
template <typename WinT, bool DIAG, bool FFPV = false, bool NT = false, bool BW2 = false>
__device__ __forceinline__ void smax_scan_body(const SmaxScanArgs &a_in) {
  // the production kernel sees dbg == 0 as a constant: every diagnostic
  // branch (GT_SMAX_DEBUG) folds away, a scalar test and branch each
  SmaxScanArgs a = a_in;
  if (!DIAG) a.dbg = 0;
  // every wave is an independent worker with its own double-buffered window:
  // no workgroup barrier anywhere in K1
  __shared__ __attribute__((aligned(16))) WinT sWin[SMAX_K1_THREADS / 64][2];
  __shared__ __attribute__((aligned(16))) uint32_t sInfo[SMAX_K1_THREADS / 64][2][2];
  __shared__ SmaxRank sRank[SMAX_K1_THREADS / 64][SMAX_NCHUNK];
  // per wave: wave_detect_direct's queue of exact starts (then their
  // packed results) and accepted masks (the tile's staged records go to
  // the current window's BWT region once it is dead: window_scratch)
  __shared__ uint32_t sQueue[SMAX_K1_THREADS / 64][SMAX_DLIST + 16];

  const int lane = threadIdx.x & 63;
  // one-wave workgroups: wave 0, so every LDS address below is a constant
  // (no SGPRs held for them across the loop)
  const int wave = SMAX_K1_THREADS == 64 ? 0 : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // tile indices are 32-bit (num_tiles < 2^32): one scalar op each.  This
  // workgroup's generation of the schedule: its tiles are those of the
  // generation's range, strided by the generation's workgroup count
  // (one plan-time entry per workgroup: {first tile, stride, end}; without
  // the table every workgroup strides the whole range)
  uint32_t t0 = blockIdx.x * (SMAX_K1_THREADS / 64), stride = gridDim.x * (SMAX_K1_THREADS / 64),
           tend = a.num_tiles;
  uint4 wi = make_uint4(0u, 0u, 0u, 0u);   // llv_win words of the first two tiles
  if (a.sched_wg != nullptr) {
    const uint4 w = a.sched_wg[2 * blockIdx.x];
    wi = a.sched_wg[2 * blockIdx.x + 1];
    t0 = __builtin_amdgcn_readfirstlane(w.x);
    stride = __builtin_amdgcn_readfirstlane(w.y);
    tend = __builtin_amdgcn_readfirstlane(w.z);
  }
  const uint32_t last = tend - 1;

  uint32_t tile = t0 + (uint32_t) wave;
  // no K0 (combined placement): K1 never fills the pending slot and K1b runs
  // after it, so clearing the slot here is K0's only remaining reset (the
  // deferral count and pool cursor are reset by the previous run's K3)
  if (a.k1_reset && blockIdx.x == 0 && threadIdx.x == 0) a.bnd->pend_valid = 0;
  if (tile >= tend) return;
  Win t;
  win_init(t, a);
  t.staged_all = true;   // non-static tiles: all window values staged
  SmaxRank *rank = sRank[wave];

  // prologue: .llv windows of the first two tiles, then the first window
  const uint32_t wbase = __builtin_amdgcn_readfirstlane(lds_addr(&sWin[wave][0]));
  const uint32_t info0 = __builtin_amdgcn_readfirstlane(lds_addr(&sInfo[wave][0][0]));
  const uint32_t info1 = __builtin_amdgcn_readfirstlane(lds_addr(&sInfo[wave][1][0]));
  const uint32_t v16 = (uint32_t) lane * 16u, v4 = (uint32_t) lane * 4u;
  const uint32_t first_next = tile + stride <= last ? tile + stride : last;
  uint32_t lo0, n0;
  if (a.sched_wg != nullptr) {
    // the words came with the schedule entry: into their ring slots (LDS
    // stores, ordered before the loop's reads), and the first window at once
    lo0 = __builtin_amdgcn_readfirstlane(wi.x);
    n0 = __builtin_amdgcn_readfirstlane(wi.y);
    if (lane < 4) {
      const uint32_t v = lane == 0 ? wi.x : lane == 1 ? wi.y : lane == 2 ? wi.z : wi.w;
      (&sInfo[wave][0][0])[lane] = v;
    }
  } else {
    if (lane < 2) {
      glds4(reinterpret_cast<const uint32_t *>(a.llv_win + tile) + lane, info0);
      glds4(reinterpret_cast<const uint32_t *>(a.llv_win + first_next) + lane, info1);
    }
    glds_wait();
    lo0 = __builtin_amdgcn_readfirstlane(sInfo[wave][0][0]);
    n0 = __builtin_amdgcn_readfirstlane(sInfo[wave][0][1]);
  }
  // (the llv_win word of the tile after is loaded again into its slot:
  // the same value)
  // (wave-uniform, all lanes active: issue_window_pk's precondition)
  issue_next<NT, BW2>(a, (a.tile_first + tile) * (uint64_t) SMAX_TILE, &sWin[wave][0], wbase, lo0,
                      n0, a.llv_win + first_next, info1, v16, v4);
  // the previous tile's records (lane r holds record r) and count: stored
  // one iteration late, right after the window wait, so that those stores
  // (and the block-sum atomic) have a whole tile of work to complete before
  // the next s_waitcnt vmcnt(0) -- issued at the end of their own tile they
  // made that wait take their latency (measured 0.22 ms of K1 at C3)
  uint64_t prec = 0;
  uint32_t ptile = ~0u, pcnt = 0;
  SmaxStamps stv;
  SmaxStamps *st = nullptr;
  if constexpr (DIAG) {
    if (a.stamps != nullptr) {
      st = &stv;
      for (int k = 0; k < 8; k++) stv.acc[k] = 0;
      stv.prev = __builtin_amdgcn_s_memtime();
    }
  }
  // the loop body twice per trip, once per window buffer: the buffer
  // parity is a compile-time constant in each (no per-tile selects of the
  // window, ring slot and LDS addresses; the scalar pipe, which the four
  // SIMDs of a CU share, issues about 220 instructions per tile)
  bool first = true;
  auto step = [&](auto curc) -> bool {
    constexpr uint32_t cur = decltype(curc)::value;
    const uint64_t l0 = (a.tile_first + tile) * (uint64_t) SMAX_TILE;   // local index
    const uint64_t g0 = a.base + l0;                                      // global row
    const uint32_t next = tile + stride;
    WinT *W = &sWin[wave][cur];
    t.g0 = g0;
    t.L = to_lds<uint8_t>(W->L);
    set_bwt_window(t, W);
    t.p2 = BW2;
    t.val = nullptr;
    t.val16 = to_lds<uint16_t>(W->val16);

    // ---- this tile's window has landed (the wave's own DMA: no barrier)
    glds_wait();
    if constexpr (DIAG) SMAX_STAMP(st, 0);
    if (ptile != ~0u) {
      smax_flush_tile(a, ptile, prec, pcnt);
      ptile = ~0u;
    }
    // .llv windows of this tile and the next {lo, packed count word}: one
    // 16-byte LDS read
    // (wave-uniform: to scalars first, then scalar selects)
    const uint4 info = *reinterpret_cast<const uint4 *>(&sInfo[wave][0][0]);
    const uint32_t ix = __builtin_amdgcn_readfirstlane(info.x);
    const uint32_t iy = __builtin_amdgcn_readfirstlane(info.y);
    const uint32_t iz = __builtin_amdgcn_readfirstlane(info.z);
    const uint32_t iw = __builtin_amdgcn_readfirstlane(info.w);
    const uint32_t wlo = cur ? iz : ix;
    const uint32_t wnf = cur ? iw : iy;
    const uint32_t wn = SMAX_WIN_N(wnf);
    const uint32_t nlo = cur ? ix : iz;
    const uint32_t nn = cur ? iy : iw;   // the next tile's llv_win word (count, DMA lanes)

    // ---- DMA of the next tile's window (and the .llv window of the tile
    // after it, into the ring slot just read): in flight during all of this
    // tile's work
    if (next < tend && !((SMAX_DBG(a) & (1u << 23)) && !first)) {   // diagnostic: compute only
      const uint32_t n2 = next + stride <= last ? next + stride : last;
      // the condition is wave-uniform (next, tend, first are per wave), all
      // lanes active: issue_window_pk's precondition
      issue_next<NT, BW2>(a, (a.tile_first + next) * (uint64_t) SMAX_TILE, &sWin[wave][cur ^ 1u],
                 wbase + (cur ^ 1u) * (uint32_t) sizeof(WinT), nlo, nn,
                 a.llv_win + n2, cur ? info1 : info0, v16, v4);
    }
    if constexpr (DIAG) SMAX_STAMP(st, 1);
    t.halo_ff = SMAX_WIN_HALO(wnf);
    uint32_t segpre_bits = prepare_window(t, a, rank, wlo, wn);
    if constexpr (DIAG) SMAX_STAMP(st, 2);
    if (SMAX_DBG(a) & (3u << 17)) {   // diagnostic: 64 extra dependent VALU / SALU per tile (cost model)
      if (SMAX_DBG(a) & (1u << 17)) {
        uint32_t x = segpre_bits;
#pragma unroll
        for (int q = 0; q < 64; q++) asm volatile("v_add_u32 %0, %0, 1" : "+v"(x));
        segpre_bits = x - 64;
      } else {
        uint32_t y = a.minlen;
#pragma unroll
        for (int q = 0; q < 64; q++) asm volatile("s_add_u32 %0, %0, 1" : "+s"(y));
        if (y == 12345) segpre_bits = 0;
      }
    }
    const bool wave_pre = __ballot(segpre_bits != 0) != 0 && !(SMAX_DBG(a) & 2u);

    // ---- detection, diversity, records (row order)
    uint32_t wcount = 0;
    // shard-edge tiles and windows with more .llv values than K1 stages
    // belong to the static K1b list (plan time, smax_static_defer_kernel;
    // run concurrently on the plan's side stream): K1 leaves them alone and
    // never waits on a global .llv read
    const bool stat = static_deferred(a, wnf);
    bool defer = !stat && wave_pre && (SMAX_DBG(a) & 128u);
    if (!stat && !defer && wave_pre) {
      wcount = wave_detect_direct<SMAX_DLIST, FFPV>(t, a, g0, W->L, sQueue[wave],
                                                    window_scratch(W), segpre_bits,
                                                    DIAG ? st : nullptr);
      // exact-queue overflow (UINT32_MAX) or more records than the tile's
      // slot holds: runtime K1b list
      defer = wcount > SMAX_SSLOT;
    }
    // (uniform tests first, then lane 0: a `lane == 0 && flag` condition
    // costs exec-mask bookkeeping on every tile, taken or not)
    if (defer) {
      if (lane == 0) {
        const uint32_t k = atomicAdd(a.defer_count, 1u);
        a.defer_list[k] = (uint32_t) tile;
        a.defer_info[k] = make_uint2(wlo, wnf);
      }
    }
    // K1b's tiles: their count words carry the wide bit (K1b writes
    // count | wide), so the block sums in K1b's launch skip them and K1b adds
    // their records itself
    if ((stat || defer) && a.bs_wgs) {
      if (lane == 0) a.tile_count[tile] = SMAX_SLOT_WIDE;
    }
    if (!stat && !defer) {
      // the tile's records move from the LDS staging to one lane each; they
      // are stored at the start of the next iteration (see above)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      prec = window_scratch(W)[lane];
      ptile = tile;
      pcnt = wcount;
    }
    if constexpr (DIAG) {
      SMAX_STAMP(st, 6);
      if (st != nullptr) st->acc[7]++;
    }

    tile = next;
    first = false;
    return tile < tend;
  };
  for (;;) {
    if (!step(std::integral_constant<uint32_t, 0>())) break;
    if (!step(std::integral_constant<uint32_t, 1>())) break;
  }
  if (ptile != ~0u) smax_flush_tile(a, ptile, prec, pcnt);
  glds_wait();
  if constexpr (DIAG) {
    if (st != nullptr && lane == 0)
      for (int k = 0; k < 8; k++) atomicAdd(&a.stamps[k], st->acc[k]);
  }
}

// K1b: the tiles K1 defers -- shard edges (row 0, begin, end, N), windows
// with more .llv values than K1 stages, exact-queue overflow -- plus the
// shard's boundary head.  One wave per tile, everything exact: the window's
// LCP values are expanded to u32 in LDS (bytes, then the window's .llv
// values scattered over their 255 bytes), so no rank arithmetic and no
// lane-serial scan over a run of 255 bytes.  Per 64-row step every lane
// decides one row (start: LCP[c] > LCP[c-1], LCP[c] >= minlen, c owned;
// plateau end: LCP[c+1] != LCP[c]) into wave ballots; the starts are then
// compacted (row order, 512 rows at a time) and evaluated 64 at a time:
// plateau end from the ballot words, local maximum, left diversity over the
// window's BWT bytes, the pending plateau at the shard end.  Plateaus that
// run past the window take the generic global path (eval_start).
#define SMAX_XSTEPS ((SMAX_TILE + 64 + 63) / 64)      // ballot steps incl. right halo

struct SmaxWindowX {
  uint8_t L[SMAX_LDSB];
  uint8_t B[SMAX_LDSB];
  uint32_t X[SMAX_LDSB];        // exact LCP of window row o (0 outside [1, N))
  uint64_t ne[SMAX_XSTEPS];     // bit b: LCP[row b + 1] != LCP[row b] (tile rows b)
  uint64_t st[SMAX_TILE / 64];  // bit b: row b is an owned plateau start
};

// Loads tile l0's window (rows g0-LH .. g0+TILE+RH-1) into W and expands the
// exact LCP values.  Sets the error bit when the window's 255 bytes and its
// .llv entries disagree.
__device__ static void load_exact_window(const SmaxScanArgs &a, uint64_t l0, SmaxWindowX *W) {
  const int lane = threadIdx.x & 63;
  const uint64_t g0 = a.base + l0;
  const uint2 info = a.llv_win[l0 / SMAX_TILE - a.tile_first];
  const uint32_t lo = info.x, n = SMAX_WIN_N(info.y);
  const uint64_t wb = g0 - SMAX_LH;
  // every load of the window first (3 chunks of LCP and BWT per lane, the
  // first 4 .llv entries per lane), then the LDS writes
  uint4 lv[3], bv[3];
#pragma unroll
  for (int r = 0; r < 3; r++) {
    const int i = lane + 64 * r;
    if (r < 2 || i < SMAX_NCHUNK) {
      const int64_t r0 = (int64_t) l0 - SMAX_LH + 16 * i;
      lv[r] = *reinterpret_cast<const uint4 *>(a.lcp + r0);
      // packed shards: group l0/16 + i holds the chunk's 16 rows
      bv[r] = a.bwtpk != nullptr ? pk_expand(a.bwtpk[l0 / 16 + i])
                                 : *reinterpret_cast<const uint4 *>(a.bwt + r0);
    } else {
      lv[r] = make_uint4(0, 0, 0, 0);
      bv[r] = lv[r];
    }
  }
  uint4 ev[4];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const uint32_t e = (uint32_t) lane + 64u * r;
    ev[r] = e < n ? *reinterpret_cast<const uint4 *>(&a.llv[lo + e]) : make_uint4(0, 0, 0, 0);
  }
  uint32_t nff = 0;
#pragma unroll
  for (int r = 0; r < 3; r++) {
    const int i = lane + 64 * r;
    if (r == 2 && i >= SMAX_NCHUNK) break;
    *reinterpret_cast<uint4 *>(&W->L[16 * i]) = lv[r];
    *reinterpret_cast<uint4 *>(&W->B[16 * i]) = bv[r];
    nff += seg_ffcount(lv[r]);
    const int64_t gr = (int64_t) wb + 16 * i;                     // global row of the chunk
    const uint32_t w[4] = {lv[r].x, lv[r].y, lv[r].z, lv[r].w};
    const bool inner = gr >= 1 && gr + 16 <= (int64_t) a.N;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      uint4 x;
      uint32_t *xe = &x.x;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int64_t g = gr + 4 * k + q;
        const uint32_t byte = (w[k] >> (8 * q)) & 0xffu;
        xe[q] = (inner || (g >= 1 && g < (int64_t) a.N)) ? byte : 0u;
      }
      *reinterpret_cast<uint4 *>(&W->X[16 * i + 4 * k]) = x;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  // .llv values over their 255 bytes (entries of [g0-LH, g0+TILE+RH)); the
  // record is {u64 position, u64 value}: x,y = position, z = value low dword
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const uint32_t e = (uint32_t) lane + 64u * r;
    const uint64_t pos = ((uint64_t) ev[r].y << 32) | ev[r].x;
    const uint64_t o = pos - wb;
    if (e < n && o < SMAX_LDSB && pos < a.N) W->X[o] = ev[r].z;
  }
  // dense windows (the static list's): 12 entries per lane per batch, so a
  // full window (<= 2080 entries) costs at most 3 dependent load rounds
  // instead of 8 (the window load was half of a K1b tile's time)
  for (uint32_t e0 = 256; e0 < n; e0 += 768) {
    uint2 pv[12];
    uint32_t vv[12];
#pragma unroll
    for (int r = 0; r < 12; r++) {
      const uint32_t e = e0 + (uint32_t) lane + 64u * r;
      const uint32_t *rec = reinterpret_cast<const uint32_t *>(&a.llv[lo + (e < n ? e : 0)]);
      pv[r] = make_uint2(rec[0], rec[1]);
      vv[r] = rec[2];
    }
#pragma unroll
    for (int r = 0; r < 12; r++) {
      const uint32_t e = e0 + (uint32_t) lane + 64u * r;
      const uint64_t pos = ((uint64_t) pv[r].y << 32) | pv[r].x;
      const uint64_t o = pos - wb;
      if (e < n && o < SMAX_LDSB && pos < a.N) W->X[o] = vv[r];
    }
  }
  uint32_t tot;
  (void) wave_excl(nff, &tot);
  // every 255 byte of [1, N) in the window has its entry (rows < 1 or >= N
  // hold 0 bytes in a consistent index)
  if (tot != n && lane == 0) atomicOr(a.err, SMAX_ERR_LLV);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// The boundary head from the exact window of the shard's first tile (the
// run of LCP == LCP[begin]); runs leaving the window take compute_head.
__device__ static void head_from_window(const SmaxScanArgs &a, const SmaxWindowX *W, uint64_t g0) {
  if ((threadIdx.x & 63) != 0) return;
  const uint64_t wb = g0 - SMAX_LH;
  uint64_t o = a.begin - wb;
  const uint32_t v = W->X[o];
  Seen s = {0, 0, 0, 0};
  uint64_t dup = 0, f = UINT64_MAX, nxt = 0;
  if (v >= a.minlen && a.begin < a.end) {
    for (;;) {
      if (seen_add(s, W->B[o])) { dup = 1; break; }
      if (o + 1 >= SMAX_LDSB) { compute_head(a); return; }
      const uint32_t nx = W->X[o + 1];
      if (nx != v) { f = wb + o + 1; nxt = nx; break; }
      if (wb + o + 1 >= a.end) break;   // run covers the whole shard: passthrough
      o++;
    }
  } else {
    f = a.begin;
    nxt = v;
  }
  GtSmaxBoundary *b = a.bnd;
  b->shard_begin = a.begin;
  b->shard_end = a.end;
  b->head_v = v;
  b->head_f = f;
  b->head_next = nxt;
  b->head_div.seen[0] = s.w0; b->head_div.seen[1] = s.w1;
  b->head_div.seen[2] = s.w2; b->head_div.seen[3] = s.w3;
  b->head_div.dup = dup;
}

// Exact evaluation of the plateau start at tile row b (window W, LCP value
// cur); returns whether [c-1 .. j] is a supermaximal-repeat interval.
__device__ static bool eval_start_x(const SmaxScanArgs &a, const Win &t, const SmaxWindowX *W,
                                    uint64_t g0, uint32_t b, uint32_t *curo, uint64_t *jo) {
  const uint32_t o = b + SMAX_LH;
  const uint32_t cur = W->X[o];
  // plateau end: first row >= b whose successor differs
  uint32_t wi = b >> 6;
  uint64_t m = W->ne[wi] >> (b & 63);
  uint32_t jb = b;
  while (m == 0 && wi + 1 < SMAX_XSTEPS) {
    jb = (wi + 1) << 6;
    m = W->ne[++wi];
  }
  jb += (uint32_t) __builtin_ctzll(m);
  if (jb + SMAX_LH + 1 >= SMAX_LDSB) {
    // the plateau leaves the window: generic exact path (global reads)
    return eval_start(t, a, g0, W->L, b, 0, false, curo, jo);
  }
  *curo = cur;
  const uint64_t c = g0 + b, j = g0 + jb;
  *jo = j;
  if (j >= a.end) {
    // the plateau contains row `end`: pending, resolved by the stitch
    Seen sn = {0, 0, 0, 0};
    bool dup = false;
    for (uint64_t g = c - 1; g < a.end && !dup; g++) dup = seen_add(sn, W->B[g - g0 + SMAX_LH]);
    if (!dup) {
      GtSmaxBoundary *bd = a.bnd;
      bd->pend_c = c;
      bd->pend_lcp = cur;
      bd->pend_div.seen[0] = sn.w0; bd->pend_div.seen[1] = sn.w1;
      bd->pend_div.seen[2] = sn.w2; bd->pend_div.seen[3] = sn.w3;
      bd->pend_div.dup = 0;
      bd->pend_valid = 1;
    }
    return false;
  }
  if (W->X[jb + SMAX_LH + 1] > cur) return false;   // not a local maximum
  const uint32_t width = jb - b + 2;
  if (width <= 8 && o + 10 < SMAX_LDSB) return diverse8(lds_bytes8(W->B, o - 1), width);
  Seen sn = {0, 0, 0, 0};
  for (uint32_t q = o - 1; q <= jb + SMAX_LH; q++)
    if (seen_add(sn, W->B[q])) return false;
  return true;
}

// load_exact_window for a whole workgroup (TH threads): one 16-row chunk
// per thread and every .llv entry of the window (<= SMAX_LDSB) fetched in
// one round of at most 9 (256 threads) or 5 (512) per thread, instead of one
// wave doing 3 chunks per lane and up to 4 dependent .llv rounds.  *nff is
// a workgroup counter the caller zeroes.
template <int TH>
__device__ static void load_exact_window_wg(const SmaxScanArgs &a, uint64_t l0, uint2 info,
                                            SmaxWindowX *W, uint32_t *nff, uint64_t *tmark) {
  static_assert(TH >= SMAX_NCHUNK, "one window chunk per thread");
  const int tid = threadIdx.x;
  const uint64_t g0 = a.base + l0;
  const uint32_t lo = info.x, n = SMAX_WIN_N(info.y);
  const uint64_t wb = g0 - SMAX_LH;
  constexpr int EPT = (SMAX_LDSB + TH - 1) / TH;      // .llv entries per thread
  uint2 ep[EPT];
  uint32_t ev[EPT];
#pragma unroll
  for (int r = 0; r < EPT; r++) {
    const uint32_t e = (uint32_t) tid + (uint32_t) TH * r;
    const uint32_t *rec = reinterpret_cast<const uint32_t *>(&a.llv[lo + (e < n ? e : 0)]);
    const uint32_t r0 = __builtin_nontemporal_load(rec), r1 = __builtin_nontemporal_load(rec + 1);
    const uint32_t r2 = __builtin_nontemporal_load(rec + 2);
    ep[r] = e < n ? make_uint2(r0, r1) : make_uint2(0xffffffffu, 0xffffffffu);
    ev[r] = e < n ? r2 : 0u;
  }
  uint32_t f = 0;
  if (tid < SMAX_NCHUNK) {
    const int i = tid;
    const int64_t r0 = (int64_t) l0 - SMAX_LH + 16 * i;
    // the window is read once (K1 skipped it): non-temporal loads
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 lq = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(a.lcp + r0));
    const uint4 lv = make_uint4(lq.x, lq.y, lq.z, lq.w);
    const uint4 bv = a.bwtpk != nullptr ? pk_expand(__builtin_nontemporal_load(&a.bwtpk[l0 / 16 + i]))
                                        : *reinterpret_cast<const uint4 *>(a.bwt + r0);
    if (SMAX_DBG(a) & 524288u) {   // diagnostic stamp: every load of the thread has landed
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (*tmark == 0) *tmark = __builtin_readcyclecounter();
    }
    *reinterpret_cast<uint4 *>(&W->L[16 * i]) = lv;
    *reinterpret_cast<uint4 *>(&W->B[16 * i]) = bv;
    f = seg_ffcount(lv);
    const int64_t gr = (int64_t) wb + 16 * i;
    const uint32_t w[4] = {lv.x, lv.y, lv.z, lv.w};
    const bool inner = gr >= 1 && gr + 16 <= (int64_t) a.N;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      uint4 x;
      uint32_t *xe = &x.x;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int64_t g = gr + 4 * k + q;
        const uint32_t byte = (w[k] >> (8 * q)) & 0xffu;
        xe[q] = (inner || (g >= 1 && g < (int64_t) a.N)) ? byte : 0u;
      }
      *reinterpret_cast<uint4 *>(&W->X[16 * i + 4 * k]) = x;
    }
  }
  // the window's 255 bytes: one LDS atomic per wave (not per chunk)
  uint32_t ftot;
  (void) wave_excl(f, &ftot);
  if ((threadIdx.x & 63) == 0 && ftot) atomicAdd(nff, ftot);
  __syncthreads();
  if ((SMAX_DBG(a) & 1048576u) && *tmark == 0) *tmark = __builtin_readcyclecounter();
#pragma unroll
  for (int r = 0; r < EPT; r++) {
    const uint32_t e = (uint32_t) tid + (uint32_t) TH * r;
    const uint64_t pos = ((uint64_t) ep[r].y << 32) | ep[r].x;
    const uint64_t o = pos - wb;
    if (e < n && o < SMAX_LDSB && pos < a.N) W->X[o] = ev[r];
  }
  __syncthreads();
  // every 255 byte of [1, N) in the window has its entry
  if (tid == 0 && *nff != n) atomicOr(a.err, SMAX_ERR_LLV);
}

// K1b, one workgroup per tile (the combined placement's kernel): a K1b
// launch covers few tiles (the static list and K1's rare deferrals; about
// 300 per shard of an 8-way C3 split), so its time is the slowest tile's,
// and one wave per tile left three of every four waves idle.  Here the
// whole workgroup loads the exact window (load_exact_window_wg), the NW
// waves share the ballot steps, and each takes one round of 2048 / NW rows'
// starts: evaluated once into LDS (value, width, accepted), the rounds'
// record counts are scanned across the waves and the records written in
// row order.  NW = 4 (one tile in 24k cycles, 5 workgroups per CU) or, when
// the launch fits one generation of them, NW = 8 (two per CU, a tile's
// ballots and evaluation split twice as fine).
template <int NW>
struct SmaxDeferWG {
  static constexpr int XQ = SMAX_TILE / NW;   // rows per wave's round
  SmaxWindowX win;
  uint16_t list[NW][XQ];            // per wave: its round's starts (row order)
  // per wave: its accepted records, compacted (a round of XQ rows holds at
  // most XQ / 2: consecutive accepted starts are >= 2 rows apart) -- half
  // the LDS of per-start results (27 KB per workgroup; registers, not LDS,
  // hold the 4-wave kernel at 5 workgroups per CU: forcing more spilled to
  // scratch and measured slower, profiles/r02v_k1b_variants.txt)
  uint2 rec[NW][XQ / 2];            // {LCP value, width}
  uint16_t row[NW][XQ / 2];         // start row in the tile
  uint32_t cnt[NW];
  uint32_t nff;                     // 255 bytes of the window (load_exact_window_wg)
  uint64_t off;                     // the tile's first record in the pool (~0: none)
};

template <int NW>
__global__ void __launch_bounds__(64 * NW)
smax_defer_wg_kernel(SmaxScanArgs a) {
  constexpr int XQ = SmaxDeferWG<NW>::XQ;
  __shared__ __attribute__((aligned(16))) SmaxDeferWG<NW> sD;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  SmaxWindowX *W = &sD.win;
  Win t;
  win_init(t, a);
  // the last bs_wgs workgroups: K3's block sums (K2's work, without its
  // launch), NW blocks each, from the counts K1 wrote; tiles K1 left
  // to K1b hold the wide bit and are added by their K1b workgroup below.
  // Both add into the run's zeroed buffer (K3 clears the other one).
  const uint32_t tile_wgs = gridDim.x - a.bs_wgs;
  if (blockIdx.x >= tile_wgs) {
    // wave w sums block b0 + w (4 counts per lane), one atomic per block;
    // the workgroup's NW blocks share a superblock: one atomic for it
    // (atomics are issued at about one wave-instruction per 50 ns per CU:
    // one per wave and block instead of per wave, block and level)
    static_assert(SMAX_SBB % NW == 0, "a block per wave, one superblock per workgroup");
    const uint32_t nb = (a.num_tiles + SMAX_CPB - 1) / SMAX_CPB;
    const uint32_t b0 = (blockIdx.x - tile_wgs) * NW, b = b0 + (uint32_t) wave;
    uint32_t v[SMAX_CPB / 64];
#pragma unroll
    for (int u = 0; u < SMAX_CPB / 64; u++) {
      const uint32_t tt = b * SMAX_CPB + 64u * u + lane;
      v[u] = b < nb && tt < a.num_tiles ? a.tile_count[tt] : 0u;
    }
    uint32_t c = 0;
#pragma unroll
    for (int u = 0; u < SMAX_CPB / 64; u++) c += (v[u] & SMAX_SLOT_WIDE) ? 0u : v[u];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
    if (lane == 0) {
      if (c != 0 && b < nb) atomicAdd(&a.block_sum[b], c);
      sD.cnt[wave] = b < nb ? c : 0u;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t sc = 0;
#pragma unroll
      for (int w = 0; w < NW; w++) sc += sD.cnt[w];
      if (sc != 0) atomicAdd(&a.block_sum[nb + b0 / SMAX_SBB], sc);   // their superblock
    }
    return;
  }
  // workgroup 0 computes the boundary head: dispatched first, so its window
  // load overlaps the tiles' (as the last workgroup it waited for a free slot)
  if (a.k1b_head && blockIdx.x == 0) {
    if (wave == 0) {
      const uint64_t l0 = a.tile_first * (uint64_t) SMAX_TILE;
      load_exact_window(a, l0, W);
      head_from_window(a, W, a.base + l0);
    }
    return;
  }
  const uint32_t n = *a.defer_count;
  const uint64_t ltm = lanemask_lt();
  for (uint32_t i = blockIdx.x - a.k1b_head; i < n; i += tile_wgs - a.k1b_head) {
    // the list entry and its llv_win words in one round (no dependent load
    // of llv_win[tile] before the window's .llv loads)
    const uint64_t tile = a.defer_list[i];
    const uint2 info = a.defer_info[i];
    const uint64_t l0 = (a.tile_first + tile) * (uint64_t) SMAX_TILE;
    const uint64_t g0 = a.base + l0;
    if (threadIdx.x == 0) sD.nff = 0;
    __syncthreads();
    // diagnostic (GT_SMAX_DEBUG 32768): the tile's cycles / 16 instead of its
    // count; |65536 stops the clock after the window load, |131072 after the
    // ballots, |262144 after the evaluation; inside the load: |524288 when the
    // loads of thread 0 have landed, |1048576 after the LDS writes
    const uint64_t t0 = (SMAX_DBG(a) & 32768u) ? __builtin_readcyclecounter() : 0;
    uint64_t tmark = 0;
    load_exact_window_wg<64 * NW>(a, l0, info, W, &sD.nff, &tmark);
    if (SMAX_DBG(a) & 65536u) tmark = __builtin_readcyclecounter();
    t.g0 = g0;
    t.L = to_lds<uint8_t>(W->L);
    t.B = to_lds<uint8_t>(W->B);
    t.P = nullptr;
    t.rank = nullptr;
    t.val = nullptr;
    t.val16 = nullptr;
    t.nval = -1;
    // ballots: the waves take every NW-th 64-row step
    for (uint32_t st = (uint32_t) wave; st < SMAX_XSTEPS; st += NW) {
      const uint32_t b = st * 64 + lane, o = b + SMAX_LH;
      bool ne = true, sm = false;
      if (o + 1 < SMAX_LDSB) {
        const uint32_t c = W->X[o], nx = W->X[o + 1], pv = W->X[o - 1];
        const uint64_t g = g0 + b;
        ne = nx != c;
        sm = b < SMAX_TILE && c > pv && c >= a.minlen && g >= a.begin && g < a.end;
      }
      const uint64_t nem = __ballot(ne), stm = __ballot(sm);
      if (lane == 0) {
        W->ne[st] = nem;
        if (st < SMAX_TILE / 64) W->st[st] = stm;
      }
    }
    __syncthreads();
    if ((SMAX_DBG(a) & 131072u) && tmark == 0) tmark = __builtin_readcyclecounter();
    // wave w: the starts of rows [XQ w, XQ w + XQ), evaluated; accepted
    // records compacted into LDS in row order
    const uint32_t q0 = (uint32_t) wave * XQ;
    uint32_t ns = 0;
    for (uint32_t s2 = q0 / 64; s2 < (q0 + XQ) / 64; s2++) {
      const uint64_t m = W->st[s2];
      if ((m >> lane) & 1u) sD.list[wave][ns + (uint32_t) __popcll(m & ltm)] = (uint16_t) (s2 * 64 + lane);
      ns += (uint32_t) __popcll(m);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    uint32_t wc = 0;
    for (uint32_t i0 = 0; i0 < ns; i0 += 64) {
      const uint32_t k = i0 + (uint32_t) lane;
      bool acc = false;
      uint32_t cur = 0, b = 0;
      uint64_t j = 0;
      if (k < ns) {
        b = sD.list[wave][k];
        acc = eval_start_x(a, t, W, g0, b, &cur, &j);
      }
      const uint64_t am = __ballot(acc);
      const uint32_t w = wc + (uint32_t) __popcll(am & ltm);
      if (acc && w < XQ / 2) {
        sD.rec[wave][w] = make_uint2(cur, (uint32_t) (j - (g0 + b) + 2));
        sD.row[wave][w] = (uint16_t) b;
      }
      wc += (uint32_t) __popcll(am);
    }
    if (wc > XQ / 2) {   // impossible in a consistent index (see SmaxDeferWG)
      if (lane == 0) atomicOr(a.err, SMAX_ERR_LLV);
      wc = XQ / 2;
    }
    if (lane == 0) sD.cnt[wave] = wc;
    __syncthreads();
    if ((SMAX_DBG(a) & 262144u) && tmark == 0) tmark = __builtin_readcyclecounter();
    uint32_t total = 0, base = 0;
#pragma unroll
    for (int w = 0; w < NW; w++) {
      const uint32_t cw = sD.cnt[w];
      base += w < wave ? cw : 0u;
      total += cw;
    }
    const bool nowrite = (SMAX_DBG(a) & (4096u | 32768u)) != 0;
    if (threadIdx.x == 0) {
      // the tile's records: list entry i owns wide slot wide_slot0 + i (a
      // tile has at most SMAX_TILE / 2 records), else a run from the pool
      uint64_t off = ~0ull;
      const uint32_t wslot = a.wide_slot0 + i;
      if (!nowrite) {
        if (wslot < a.wide_cap) {
          off = (uint64_t) wslot * (SMAX_TILE / 2);
        } else if (total > 0) {
          off = atomicAdd(a.pool_cursor, (unsigned long long) total);
          if (off + total > a.pool_cap) off = ~0ull;   // pool full: the host re-plans
        }
        a.tile_off[tile] = off;
      }
      sD.off = off;
      if (SMAX_DBG(a) & 32768u)
        a.tile_count[tile] = (uint32_t) (((tmark ? tmark : __builtin_readcyclecounter()) - t0) >> 4);
      else if (!(SMAX_DBG(a) & 4096u))
        a.tile_count[tile] = total | SMAX_SLOT_WIDE;   // 16-byte records
      if (a.bs_wgs && total != 0) {
        const uint32_t nb = (a.num_tiles + SMAX_CPB - 1) / SMAX_CPB;
        atomicAdd(&a.block_sum[tile / SMAX_CPB], total);
        atomicAdd(&a.block_sum[nb + tile / SMAX_CPB / SMAX_SBB], total);
      }
    }
    __syncthreads();
    const uint64_t off = sD.off;
    if (off != ~0ull) {
      GtSmaxRecord *wdst = a.pool + off + base;
      for (uint32_t k = (uint32_t) lane; k < wc; k += 64) {
        const uint2 r = sD.rec[wave][k];
        GtSmaxRecord rec;
        rec.lb = g0 + sD.row[wave][k] - 1;
        rec.lcp = r.x;
        rec.width = r.y;
        wdst[k] = rec;
      }
    }
    __syncthreads();   // window and lists reused by the next tile
  }
}

// K1 instantiations, selected by the plan (plan_run_scan):
//   smax_scan_kernel_b2[_dense][_nt]  2-plane BWT window stream (0.25 B/row of
//       BWT; windows with a special BWT row go to the static K1b list), the
//       production kernels, 6 waves/SIMD (SmaxWindowB2; against 5 with the
//       packed window: C3 step -2.6 %, 3/8 shard -2.1 %, profiles/r04g/); _dense: the 255-after-255 relations of a segment
//       resolved vectorised (ffp_resolve), chosen above SMAX_FFPV_DENSITY .llv
//       entries per row (C5, the 12 Gbp plant genome at 0.94 %: step 6.21 ->
//       5.72 ms; C3 at 0.39 %: 1.7 % slower with it); _nt: non-temporal
//       window loads (GtSmaxPlan::nt: 8- and 4-way shards of C3)
//   smax_scan_kernel[_dense]  the u64 packed groups (0.5 B/row of BWT,
//       specials included; 5 waves/SIMD): shards where special BWT rows would send more
//       than 1/256 of the windows to K1b (read sets)
//   smax_scan_kernel_diag     the 2-plane kernel with the GT_SMAX_DEBUG
//       ablation switches and GT_SMAX_STAMPS section stamps (diagnostics only)
//   smax_scan_kernel_bytes    byte BWT windows (any alphabet), 4 waves/SIMD
__global__ void __launch_bounds__(SMAX_K1_THREADS, 5) smax_scan_kernel(SmaxScanArgs a) {
  smax_scan_body<SmaxWindowPk, false>(a);
}
__global__ void __launch_bounds__(SMAX_K1_THREADS, 5) smax_scan_kernel_dense(SmaxScanArgs a) {
  smax_scan_body<SmaxWindowPk, false, true>(a);
}
__global__ void __launch_bounds__(SMAX_K1_THREADS, 6) smax_scan_kernel_b2(SmaxScanArgs a) {
  smax_scan_body<SmaxWindowB2, false, false, false, true>(a);
}
__global__ void __launch_bounds__(SMAX_K1_THREADS, 6) smax_scan_kernel_b2_dense(SmaxScanArgs a) {
  smax_scan_body<SmaxWindowB2, false, true, false, true>(a);
}
__global__ void __launch_bounds__(SMAX_K1_THREADS, 6) smax_scan_kernel_b2_nt(SmaxScanArgs a) {
  smax_scan_body<SmaxWindowB2, false, false, true, true>(a);
}
__global__ void __launch_bounds__(SMAX_K1_THREADS, 6) smax_scan_kernel_b2_dense_nt(SmaxScanArgs a) {
  smax_scan_body<SmaxWindowB2, false, true, true, true>(a);
}
#ifdef GT_SMAX_DIAG
__global__ void __launch_bounds__(SMAX_K1_THREADS, 6) smax_scan_kernel_diag(SmaxScanArgs a) {
  smax_scan_body<SmaxWindowB2, true, false, false, true>(a);
}
#endif
__global__ void __launch_bounds__(SMAX_K1_THREADS, 4) smax_scan_kernel_bytes(SmaxScanArgs a) {
  smax_scan_body<SmaxWindow, false>(a);
}

// ------------------------------------------------------------ BWT packing

// Plan-time packing of a DNA shard's BWT for K1's windows: group gi holds
// local rows 16(gi-1) .. 16(gi-1)+15 as two code bit planes + a special
// mask (see pk_sym).  Sets *flag when a row of [0, local_len) holds a symbol in
// [4, 254), i.e. the alphabet is not DNA (K1 then keeps byte BWT windows).
__global__ void __launch_bounds__(256)
smax_pack_bwt_kernel(const uint8_t *bwt, uint64_t local_len, uint64_t ngroups, uint64_t *pk,
                     uint32_t *flag) {
  const uint64_t gi = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (gi >= ngroups) return;
  const int64_t r0 = ((int64_t) gi - 1) * 16;
  const uint4 v = *reinterpret_cast<const uint4 *>(bwt + r0);
  uint32_t code = 0, sp = 0;
  bool other = false;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const uint32_t w = k < 4 ? v.x : k < 8 ? v.y : k < 12 ? v.z : v.w;
    const uint32_t b = (w >> (8 * (k & 3))) & 0xffu;
    const int64_t row = r0 + k;
    if (b >= 254) sp |= 1u << k;
    else code |= ((b & 1u) << k) | (((b >> 1) & 1u) << (16 + k));   // bit planes
    if (b > 3 && b < 254 && row >= 0 && (uint64_t) row < local_len) other = true;
  }
  pk[gi] = (uint64_t) code | ((uint64_t) sp << 32);
  if (other) atomicOr(flag, 1u);
}

// ------------------------------------------------------------ K3: compact

struct SmaxNextRun {                  // the next run's resets, done by K3
  uint32_t *defer_count, *defer_last;
  unsigned long long *pool_cursor;
  uint32_t defer_base;
  unsigned long long pool_start;
};

// One workgroup per SMAX_CPB consecutive tile slots: the slots' counts are
// scanned in LDS, then all 256 threads copy the slots' records to their final
// positions (slot found by binary search in the LDS prefix), consecutive
// threads on consecutive output records -> ascending lb overall, coalesced.
// Also publishes the total.  With split > 1, `split` workgroups share one
// block: each scans the block's counts and copies its share of the records
// (small shards: a few hundred blocks leave most SIMDs without a wave and
// the copy latency-bound).
__global__ void __launch_bounds__(256)
smax_compact_kernel(const uint64_t *slots, const uint32_t *slot_count,
                    const uint32_t *block_sum, uint64_t nslots, const GtSmaxRecord *pool,
                    uint64_t pool_cap, const uint64_t *tile_off, GtSmaxRecord *out,
                    uint64_t capacity, uint64_t *count, uint64_t g00, SmaxNextRun nr,
                    uint32_t *bs_clear, uint32_t split) {
  const uint32_t blk = blockIdx.x / split, part = blockIdx.x - blk * split;
  const uint32_t nblocks = (uint32_t) ((nslots + SMAX_CPB - 1) / SMAX_CPB);
  // block sums added up in K1b's launch: this block's entries (and its
  // superblock's, by the superblock's first block) of the next run's buffer
  // start at zero
  if (part == 0 && threadIdx.x == 0) {
    bs_clear[blk] = 0;
    if (blk % SMAX_SBB == 0) bs_clear[nblocks + blk / SMAX_SBB] = 0;
  }
  // the next run's resets: K1b, the last reader of the deferral count and
  // pool cursor, has finished
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    *nr.defer_last = *nr.defer_count;
    *nr.defer_count = nr.defer_base;
    *nr.pool_cursor = nr.pool_start;
  }
  __shared__ uint32_t sPre[SMAX_CPB + 1];
  __shared__ uint32_t sWave[4];
  __shared__ uint8_t sWide[SMAX_CPB];
  __shared__ uint64_t sRed[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t s0 = blk * (uint64_t) SMAX_CPB;
  // this workgroup's output offset: the record counts of all earlier
  // workgroups (summed per SMAX_CPB tiles by K1 / K1b)
  // (a separate one-workgroup prefix kernel over the block sums instead
  // measured 0.5 % longer at C3 and 2 % longer on an 8-way shard: the extra
  // launch costs more than these loads, profiles/r03j_k2b_ab.txt)
  // this block's counts: loaded first, in flight beside the block-sum loads
  // (independent of them)
  const uint32_t cw = s0 + tid < nslots ? slot_count[s0 + tid] : 0u;
  uint64_t bs = 0;
  {
    // two-level prefix (K1b's launch also sums superblocks of SMAX_SBB
    // blocks): the earlier superblocks, then the earlier blocks of this
    // one -- a flat loop over every earlier block costs O(blocks^2) loads
    // over the launch (22.7 k blocks at C5: up to 89 per thread)
    // (both levels' loads issued before either is summed: one round trip)
    const uint32_t sb = blk / SMAX_SBB;
    const uint32_t b = sb * SMAX_SBB + tid;
    const uint32_t x0 = (uint32_t) tid < sb ? block_sum[nblocks + tid] : 0u;
    const uint32_t x1 = tid < SMAX_SBB && b < blk ? block_sum[b] : 0u;
    for (uint32_t k = tid + 256; k < sb; k += 256) bs += block_sum[nblocks + k];   // > 256 superblocks
    bs += (uint64_t) x0 + x1;
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) bs += __shfl_xor(bs, d, 64);
  if (lane == 0) sRed[wave] = bs;
  const uint32_t c = cw & ~SMAX_SLOT_WIDE;
  sWide[tid] = (cw & SMAX_SLOT_WIDE) ? 1 : 0;
  uint32_t incl = c;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(incl, d, 64);
    if (lane >= d) incl += o;
  }
  if (lane == 63) sWave[wave] = incl;
  __syncthreads();
  uint32_t wo = 0;
  for (int w = 0; w < wave; w++) wo += sWave[w];
  sPre[tid + 1] = wo + incl;
  if (tid == 0) sPre[0] = 0;
  __syncthreads();
  const uint32_t total = sPre[SMAX_CPB];
  const uint64_t base = sRed[0] + sRed[1] + sRed[2] + sRed[3];
  if (tid == 0 && part == 0 && s0 + SMAX_CPB >= nslots) *count = base + total;
  const uint32_t rlo = (uint32_t) ((uint64_t) total * part / split);
  const uint32_t rhi = (uint32_t) ((uint64_t) total * (part + 1) / split);
  // four records per thread per round: their slot searches and loads are
  // independent, so their latencies overlap (one record at a time left the
  // kernel latency-bound: 28 us for the 2.5 M records of an 8-way C3 shard)
  constexpr int U = 4;
  static_assert(SMAX_CPB == 256, "8 halvings find a slot among SMAX_CPB");
  for (uint32_t r0 = rlo + tid; r0 < rhi; r0 += 256 * U) {
    uint32_t los[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t r = r0 + 256u * u;
      uint32_t lo = 0, hi = SMAX_CPB;        // largest j with sPre[j] <= r
#pragma unroll
      for (int st = 0; st < 8; st++) {       // SMAX_CPB = 256: 8 halvings
        const uint32_t mid = (lo + hi) >> 1;
        if (sPre[mid] <= r) lo = mid; else hi = mid;
      }
      los[u] = lo;
    }
    uint64_t v[U];
    bool wide[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t r = r0 + 256u * u, lo = los[u];
      wide[u] = sWide[lo] != 0;
      v[u] = (r < rhi && !wide[u]) ? slots[(s0 + lo) * (uint64_t) SMAX_SSLOT + (r - sPre[lo])] : 0;
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t r = r0 + 256u * u, lo = los[u];
      if (r >= rhi || base + r >= capacity) continue;
      const uint64_t tile = s0 + lo;
      if (wide[u]) {
        // K1b tile: its run in the pool (absent if the pool was full, which
        // only happens when the records exceed the capacity: re-planned)
        const uint64_t off = tile_off[tile];
        if (off <= pool_cap && off + (r - sPre[lo]) < pool_cap) out[base + r] = pool[off + (r - sPre[lo])];
      } else {
        GtSmaxRecord rec;
        rec.lb = g00 + tile * (uint64_t) SMAX_TILE + (v[u] & 0x7ffu) - 1;   // g00: global row of tile 0
        rec.width = (uint32_t) (v[u] >> 11) & SMAX_PK_WMAX;
        rec.lcp = (uint32_t) (v[u] >> 32);
        out[base + r] = rec;
      }
    }
  }
}

// ------------------------------------------------------------ BWT groups

// Packed BWT groups from their code planes and the special rows (the host
// runtime stages 4 B per 16 rows over PCIe instead of 8 B):
// groups[g] = planes[g], then each (group << 16 | mask) word of spec sets
// its group's special plane (one word per group: no atomics)
__global__ void __launch_bounds__(256)
smax_groups_planes_kernel(uint64_t *groups, const uint32_t *planes, uint64_t ng) {
  const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
  for (uint64_t g = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; g < ng; g += stride)
    groups[g] = planes[g];
}
__global__ void __launch_bounds__(256)
smax_groups_spec_kernel(uint64_t *groups, uint64_t ng, const uint64_t *spec, uint64_t nspec) {
  const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
  for (uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; i < nspec; i += stride) {
    const uint64_t w = spec[i], g = w >> 16;
    if (g < ng) groups[g] |= (w & 0xffffull) << 32;
  }
}

hipError_t smax_groups_from_planes(uint64_t *groups, const uint32_t *planes, uint64_t ngroups,
                                   const uint64_t *spec, uint64_t nspec, hipStream_t stream) {
  if (ngroups == 0) return hipSuccess;
  const unsigned grid = (unsigned) std::min<uint64_t>((ngroups + 255) / 256, 65536);
  hipLaunchKernelGGL(smax_groups_planes_kernel, dim3(grid), dim3(256), 0, stream, groups, planes,
                     ngroups);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || nspec == 0) return e;
  const unsigned g2 = (unsigned) std::min<uint64_t>((nspec + 255) / 256, 65536);
  hipLaunchKernelGGL(smax_groups_spec_kernel, dim3(g2), dim3(256), 0, stream, groups, ngroups,
                     spec, nspec);
  return hipGetLastError();
}

// ------------------------------------------------------------ llv index

// K1's 2-plane window stream from the packed BWT, one pass over the groups:
// bwt2[g] = the code planes of group g, and the groups of [g_lo, g_hi) (the
// plan's windows) holding a special row counted in *nspec and listed in
// spec[] (the first spec_cap of them; one atomic per wave).  The plan picks
// the 2-plane stream from the count and then flags the listed groups'
// windows (smax_spec_mark_kernel).  Replaced a counting pass plus a
// conversion pass over the 1.5 GB of groups (268 + 437 us at C3).
__global__ void __launch_bounds__(256)
smax_bwt2_kernel(const uint64_t *pk, uint64_t ngroups, uint32_t *bwt2, uint64_t g_lo,
                 uint64_t g_hi, uint32_t *nspec, uint64_t *spec, uint32_t spec_cap) {
  const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
  const uint32_t lane = threadIdx.x & 63u;
  // wave-uniform trip count (the ballot below needs the whole wave)
  for (uint64_t g0 = blockIdx.x * (uint64_t) blockDim.x; g0 < ngroups; g0 += stride) {
    const uint64_t g = g0 + threadIdx.x;
    bool sp = false;
    if (g < ngroups) {
      const uint64_t w = pk[g];
      bwt2[g] = (uint32_t) w;
      sp = g >= g_lo && g < g_hi && ((w >> 32) & 0xffffull) != 0;
    }
    const uint64_t m = __ballot(sp);
    if (m == 0) continue;
    uint32_t base = 0;
    if (lane == (uint32_t) __builtin_ctzll(m)) base = atomicAdd(nspec, (uint32_t) __popcll(m));
    base = __shfl(base, __builtin_ctzll(m), 64);
    if (sp) {
      const uint32_t k = base + (uint32_t) __popcll(m & ((1ull << lane) - 1ull));
      if (k < spec_cap) spec[k] = g;
    }
  }
}

// Flags for the static K1b list every K1 window reading a group with a
// special row (tile i's window: groups L/16 .. L/16 + 129, L = (tile_first +
// i) * TILE): the listed groups, or (list == NULL: more special groups than
// the list holds, the 2-plane stream forced by GT_SMAX_BW2 or the diagnostic
// kernel) every group of [0, n) read again
__device__ __forceinline__ void smax_spec_mark(uint64_t g, uint2 *llv_win, uint64_t tile_first,
                                               uint64_t num_tiles) {
  constexpr uint64_t GPT = SMAX_TILE / 16;                      // groups per tile
  const uint64_t t_hi = g / GPT;                                 // L/16 <= g
  const uint64_t t_lo = g >= 129 ? (g - 129 + GPT - 1) / GPT : 0; // g <= L/16 + 129
  for (uint64_t t = t_lo; t <= t_hi; t++)
    if (t >= tile_first && t - tile_first < num_tiles)
      atomicOr(&llv_win[t - tile_first].y, SMAX_WIN_STATIC);
}

__global__ void __launch_bounds__(256)
smax_spec_mark_kernel(const uint64_t *list, const uint64_t *pk, uint64_t n, uint2 *llv_win,
                      uint64_t tile_first, uint64_t num_tiles) {
  const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
  for (uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; i < n; i += stride) {
    if (list != NULL) smax_spec_mark(list[i], llv_win, tile_first, num_tiles);
    else if ((pk[i] >> 32) & 0xffffull) smax_spec_mark(i, llv_win, tile_first, num_tiles);
  }
}

// u16 copies of the .llv values (larger values are flagged per tile by the
// index kernels; those windows never read this array)
__global__ void __launch_bounds__(256)
smax_llv16_kernel(const GtSmaxLlv *llv, uint64_t numllv, uint16_t *out) {
  const uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (i < numllv) out[i] = (uint16_t) llv[i].value;
}

// .llv window index (plan time).  Tile t's window stages the entries with
// positions in [K_lo(t), K_hi(t)) -- K_lo = g0 - LH (0 below), K_hi = g0 +
// TILE + RH, g0 = base + (tile_first + t) * TILE -- and counts those below
// g0 (its left halo).  Each bound is a lower_bound over the sorted
// positions, found without a search: the keys of consecutive tiles are
// TILE apart, so for an entry at position p the number of tiles whose key
// is <= p is arithmetic, c(p); the entry lies below key(t) exactly for
// t >= c(p), so lower_bound(key(t)) = #{entries : c <= t} = the first entry
// with c > t: a max-scan over the tiles of where each run of equal c
// starts (smax_llv_hist_kernel, then the three scan launches below).  One
// pass over the entries instead of two dependent binary searches per tile
// (815 us at C3: 1.45 M tiles, 11.7 M entries, 24 dependent loads a
// search).
struct SmaxLlvKeys {
  int64_t a_lo, a_hi, a_g0;   // key(t) = a + t * TILE (K_lo clamped at 0)
  uint32_t num_tiles;
};

// #{t in [0, nt) : max(a + t * TILE, 0) <= p}
__device__ __forceinline__ uint32_t smax_tiles_le(int64_t a, uint64_t p, uint32_t nt) {
  const int64_t d = (int64_t) p - a;
  if (d < 0) return 0u;
  const uint64_t c = (uint64_t) d / SMAX_TILE + 1;
  return c < nt ? (uint32_t) c : nt;
}

// Pass 1, one thread per entry e (and one past the last): c is
// nondecreasing in e, so the tiles whose lower bound is e are [c(e-1), c(e))
// and A[c(e-1)] = e marks where that run starts -- one plain store, and no
// other entry writes that word; lower_bound(key(t)) = max of A over [0, t],
// a max-scan.  A[t].w: the tile's window holds a value >= 2^16 (K1 stages
// u16).  err bit 1: a value >= 2^32, bit 2: positions not strictly
// increasing.  (A histogram of c with one atomic per run of equal c cost
// 434 us at C3: 7 M atomics on neighbouring words.)
__global__ void __launch_bounds__(256)
smax_llv_hist_kernel(const GtSmaxLlv *llv, uint64_t numllv, SmaxLlvKeys k, uint4 *A,
                     uint32_t *err) {
  const uint64_t e = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
  if (e > numllv) return;
  uint32_t c[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, cp[3] = {0u, 0u, 0u}, bad = 0;
  uint64_t pos = 0, v = 0;
  if (e < numllv) {
    pos = llv[e].position;
    v = llv[e].value;
    c[0] = smax_tiles_le(k.a_lo, pos, k.num_tiles);
    c[1] = smax_tiles_le(k.a_hi, pos, k.num_tiles);
    c[2] = smax_tiles_le(k.a_g0, pos, k.num_tiles);
    if (v > 0xffffffffull) bad |= 1u;
  }
  if (e > 0) {
    const uint64_t pp = llv[e - 1].position;
    cp[0] = smax_tiles_le(k.a_lo, pp, k.num_tiles);
    cp[1] = smax_tiles_le(k.a_hi, pp, k.num_tiles);
    cp[2] = smax_tiles_le(k.a_g0, pp, k.num_tiles);
    if (e < numllv && pos <= pp) bad |= 2u;
  }
#pragma unroll
  for (int q = 0; q < 3; q++)
    if (c[q] > cp[q] && cp[q] < k.num_tiles)
      reinterpret_cast<uint32_t *>(A)[4 * (uint64_t) cp[q] + q] = (uint32_t) e;
  // the windows holding p: K_lo(t) <= p < K_hi(t), i.e. c_hi <= t < c_lo
  if (e < numllv && v > 0xffffull)
    for (uint32_t t = c[1]; t < c[0]; t++)
      atomicOr(reinterpret_cast<uint32_t *>(A) + 4 * (uint64_t) t + 3, 1u);
  if (bad) atomicOr(err, bad);
}

// The max-scan of A over the tiles, in three launches of this module (a
// library scan's first call cost ~3 ms of one-time setup in a fresh
// process): per-block maxima of 1024 tiles, one workgroup scanning them,
// then each block's scan from its prefix, which also assembles the tiles'
// llv_win words.
#define SMAX_IDX_PER 4
#define SMAX_IDX_BLK (256 * SMAX_IDX_PER)

__device__ __forceinline__ uint3 smax_u3max(uint3 a, uint3 b) {
  return make_uint3(a.x > b.x ? a.x : b.x, a.y > b.y ? a.y : b.y, a.z > b.z ? a.z : b.z);
}

// exclusive prefix maximum over the 256 threads of one uint3 each (0 for
// thread 0); *total = the maximum
__device__ __forceinline__ uint3 smax_block_excl3(uint3 v, uint3 *total) {
  __shared__ uint3 sW[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint3 inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint3 o = make_uint3(__shfl_up(inc.x, d, 64), __shfl_up(inc.y, d, 64), __shfl_up(inc.z, d, 64));
    if (lane >= d) inc = smax_u3max(inc, o);
  }
  if (lane == 63) sW[wave] = inc;
  __syncthreads();
  uint3 wo = make_uint3(0u, 0u, 0u);
  for (int w = 0; w < wave; w++) wo = smax_u3max(wo, sW[w]);
  // the thread's exclusive value: its lane predecessor's inclusive one
  uint3 ex = make_uint3(__shfl_up(inc.x, 1, 64), __shfl_up(inc.y, 1, 64), __shfl_up(inc.z, 1, 64));
  if (lane == 0) ex = make_uint3(0u, 0u, 0u);
  *total = smax_u3max(smax_u3max(sW[0], sW[1]), smax_u3max(sW[2], sW[3]));
  __syncthreads();   // sW before a next use
  return smax_u3max(wo, ex);
}

__global__ void __launch_bounds__(256)
smax_llv_bsum_kernel(const uint4 *hist, uint32_t nt, uint3 *bsum) {
  const uint64_t t0 = blockIdx.x * (uint64_t) SMAX_IDX_BLK + threadIdx.x * (uint64_t) SMAX_IDX_PER;
  uint3 s = make_uint3(0u, 0u, 0u);
#pragma unroll
  for (int q = 0; q < SMAX_IDX_PER; q++)
    if (t0 + q < nt) {
      const uint4 h = hist[t0 + q];
      s = smax_u3max(s, make_uint3(h.x, h.y, h.z));
    }
  uint3 tot;
  (void) smax_block_excl3(s, &tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

// one workgroup: bsum[0..nb) -> exclusive prefixes, in place
__global__ void __launch_bounds__(256) smax_llv_btop_kernel(uint3 *bsum, uint32_t nb) {
  uint3 run = make_uint3(0u, 0u, 0u);
  for (uint64_t c0 = 0; c0 < nb; c0 += SMAX_IDX_BLK) {
    const uint64_t b0 = c0 + threadIdx.x * (uint64_t) SMAX_IDX_PER;
    uint3 v[SMAX_IDX_PER], s = make_uint3(0u, 0u, 0u);
#pragma unroll
    for (int q = 0; q < SMAX_IDX_PER; q++) {
      v[q] = b0 + q < nb ? bsum[b0 + q] : make_uint3(0u, 0u, 0u);
      s = smax_u3max(s, v[q]);
    }
    uint3 tot;
    uint3 o = smax_u3max(run, smax_block_excl3(s, &tot));
#pragma unroll
    for (int q = 0; q < SMAX_IDX_PER; q++)
      if (b0 + q < nb) {
        bsum[b0 + q] = o;
        o = smax_u3max(o, v[q]);
      }
    run = smax_u3max(run, tot);
  }
}

// each tile's three lower bounds (the inclusive scan at the tile) and its
// llv_win word
__global__ void __launch_bounds__(256)
smax_llv_win_kernel(const uint4 *hist, const uint3 *bsum, uint32_t nt, uint64_t g0_first,
                    uint64_t begin, uint64_t end, uint2 *win_out, uint32_t all_static) {
  const uint64_t t0 = blockIdx.x * (uint64_t) SMAX_IDX_BLK + threadIdx.x * (uint64_t) SMAX_IDX_PER;
  uint4 h[SMAX_IDX_PER];
  uint3 s = make_uint3(0u, 0u, 0u);
#pragma unroll
  for (int q = 0; q < SMAX_IDX_PER; q++) {
    h[q] = t0 + q < nt ? hist[t0 + q] : make_uint4(0u, 0u, 0u, 0u);
    s = smax_u3max(s, make_uint3(h[q].x, h[q].y, h[q].z));
  }
  uint3 tot;
  uint3 run = smax_u3max(bsum[blockIdx.x], smax_block_excl3(s, &tot));
#pragma unroll
  for (int q = 0; q < SMAX_IDX_PER; q++) {
    const uint64_t t = t0 + q;
    run = smax_u3max(run, make_uint3(h[q].x, h[q].y, h[q].z));
    if (t >= nt) continue;
    const uint64_t g0 = g0_first + t * (uint64_t) SMAX_TILE;
    const uint32_t lo = run.x, wn = run.y - run.x;   // <= SMAX_LDSB rows
    const uint32_t halo = run.z - run.x;             // entries in the left halo [g0 - LH, g0)
    const bool wide = h[q].w != 0;                   // K1 stages values as u16
    // g0 < begin: the shard's first tile when begin is not tile-aligned (K1
    // assumes every row of its tiles is owned)
    // all_static (GT_SMAX_ALL_STATIC, a test hook): every tile through K1b's
    // exact path
    const bool stat = g0 < SMAX_LH || g0 < begin || g0 + SMAX_TILE + SMAX_RH > end || wide ||
                      wn + (lo & 7u) > SMAX_LLV_CAP || all_static;
    const uint32_t nl8 = wn == 0 ? 0u : (wn + (lo & 7u) + 7u) / 8u;
    const uint32_t nl = nl8 < SMAX_LLV_CAP / 8 ? nl8 : SMAX_LLV_CAP / 8;
    static_assert(SMAX_LLV_CAP / 8 < 64, "lane count fits SMAX_WIN_LANES");
    win_out[t] = make_uint2(lo, wn | (halo << 12) | (nl << 17) | (stat ? SMAX_WIN_STATIC : 0u));
  }
}

// the plan's host-side scalars in one copy: the static list's length and
// the first and last tiles' llv_win words
__global__ void smax_plan_probe_kernel(const uint32_t *static_count, const uint2 *llv_win,
                                       uint32_t num_tiles, uint32_t *out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  out[0] = *static_count;
  const uint2 w0 = num_tiles ? llv_win[0] : make_uint2(0u, 0u);
  const uint2 w1 = num_tiles ? llv_win[num_tiles - 1] : make_uint2(0u, 0u);
  out[1] = w0.x;
  out[2] = w0.y;
  out[3] = w1.x;
  out[4] = w1.y;
}

// ------------------------------------------------------------ stitch

__host__ __device__ static int stitch_resolve(const GtSmaxBoundary *all,
                                              int nshards, int idx,
                                              unsigned int minlen,
                                              GtSmaxRecord *rec) {
  const GtSmaxBoundary *me = &all[idx];
  if (!me->pend_valid) return 0;
  const uint64_t l = me->pend_lcp;
  uint64_t seen[4] = {me->pend_div.seen[0], me->pend_div.seen[1],
                      me->pend_div.seen[2], me->pend_div.seen[3]};
  (void) minlen;
  for (int r = idx + 1; r < nshards; r++) {
    const GtSmaxBoundary *h = &all[r];
    if (h->head_v != l) return 0;          // cannot happen: LCP[end] == l
    if (h->head_div.dup) return 0;
    for (int w = 0; w < 4; w++) {
      if (seen[w] & h->head_div.seen[w]) return 0;
      seen[w] |= h->head_div.seen[w];
    }
    if (h->head_f != UINT64_MAX) {
      if (h->head_next >= l) return 0;     // not a local maximum
      const uint64_t lb = me->pend_c - 1, rb = h->head_f - 1;
      rec->lb = lb;
      rec->lcp = (uint32_t) l;
      rec->width = (uint32_t) (rb - lb + 1);
      return 1;
    }
  }
  return 0;   // last shard always ends the run (LCP[N] == 0)
}

__global__ void smax_stitch_kernel(const GtSmaxBoundary *all, int nshards,
                                   int idx, unsigned int minlen,
                                   GtSmaxRecord *out, uint64_t capacity,
                                   uint64_t *count) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  GtSmaxRecord rec;
  if (stitch_resolve(all, nshards, idx, minlen, &rec)) {
    const uint64_t c = *count;
    if (c < capacity) out[c] = rec;
    *count = c + 1;
  }
}

// ============================================================ host side

static void seterr(char *errbuf, size_t errlen, const char *fmt, ...) {
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

#define SMAX_PLAN_STREAMS 4
struct GtSmaxPlan {
  GtSmaxDevShard shard;
  unsigned int minlen;
  uint64_t capacity;
  uint32_t num_tiles;
  uint64_t tile_first;
  uint32_t grid, compact_grid;
  uint32_t sched_n;                               // K1's tile schedule (plan_size_grid)
  uint32_t sched_blk[SMAX_SCHED_MAX + 1], sched_tile[SMAX_SCHED_MAX + 1];
  uint4 *sched_wg;                                // its per-workgroup entries (device)
  GtSmaxRecord *out;         // capacity records, ascending lb
  uint64_t *slots;           // num_tiles * SMAX_SSLOT packed records (K1)
  GtSmaxRecord *pool;        // wide_cap wide slots + capacity records (K1b tiles' runs)
  uint32_t wide_cap;
  unsigned long long *pool_cursor;
  uint64_t *tile_off;        // num_tiles
  uint32_t *tile_count;      // num_tiles
  uint32_t *block_sum;       // two buffers of block + superblock record sums (K3's offsets)
  uint64_t *count;
  GtSmaxBoundary *bnd;
  uint2 *llv_win;
  uint64_t *bwtpk;           // packed BWT (DNA shards), else null
  bool pk, pk_owned;          // packed windows; bwtpk allocated by the plan
  uint32_t *bwt2;            // its code planes alone (K1's 2-plane window stream), or null
  bool bw2;                  // K1 streams bwt2 (windows with a special BWT row: static K1b)
  uint16_t *llv16;           // .llv values as u16 (numllv + 2)
  uint32_t *defer_list;      // K1 -> K1b tile list (num_tiles) + count
  uint2 *defer_info;         // beside each entry: the tile's llv_win words
  uint32_t *defer_count;
  uint32_t *defer_last;      // K1's last count (K3 resets the live one for the next run)
  uint32_t *static_list;     // plan-time K1b list (edges, wide .llv windows) + count
  uint32_t *static_count;
  uint32_t n_static;
  bool dense;                // .llv entries per row above SMAX_FFPV_DENSITY: smax_scan_kernel*_dense
  bool nt;                   // window stream with the non-temporal policy (smax_scan_kernel_b2*_nt)
  uint32_t k1b_grid;         // K1b's tile workgroups (+1: the boundary head)
  uint32_t bs_wgs;           // block-sum workgroups appended to K1b's grid
  uint32_t k1b_nw;           // waves per K1b workgroup (4 or 8)
  uint32_t k3_split;         // K3 workgroups per block of 256 tiles (GT_SMAX_K3_SPLIT)
  bool part1_pending;        // part 0 enqueued, its part 1 not yet (the next part 0 must wait)
  uint32_t *err;
  uint32_t dbg;              // GT_SMAX_DEBUG (diagnostic build only; 0 otherwise)
  bool all_static;           // GT_SMAX_ALL_STATIC: every tile through K1b (test hook)
  bool byte_windows;         // GT_SMAX_BYTE_WINDOWS: byte BWT windows, never packed (test hook)
  uint32_t dev_cus;
  // streams this plan's work was enqueued on (the fence of its buffers at
  // delete: a freed block is reused only after that work,
  // smax_dev_free_fenced); more than SMAX_PLAN_STREAMS distinct ones: the
  // device is synchronised.  The events are recorded at delete (and waited
  // on in plan_sync) on these handles, so every stream passed to the plan
  // must outlive it (gt_smax_hip.h): an event recorded behind every run
  // instead cost one event packet per step, +0.7 % of the C3 step
  // (profiles/r6/, bench_c3 against the round-5 build)
  hipStream_t streams[SMAX_PLAN_STREAMS];
  int nstreams;
  bool streams_overflow;
  // optional K1 timing: event pairs recorded around the scan kernel
  hipEvent_t *ev;
  unsigned long long *stamps;    // GT_SMAX_STAMPS: K1 section cycles (diag build)
  int nslots;
  int tstride;               // K1 events on every tstride-th run (gt_smax_plan_timing_stride)
  uint64_t runs;             // runs since the timing was (re)configured (event slots)
  uint32_t bs_buf;           // block-sum buffer (0/1) of the next run: flipped only by
                             // plan_run_compact (its K3 clears the other buffer), never by
                             // the timing calls, so a pass always adds into a cleared one
};

static SmaxScanArgs plan_args(GtSmaxPlan *p);

// plan buffers come from the runtime's per-device cache (smax_internal.h)
template <typename T>
static hipError_t dalloc(T **p, size_t bytes) {
  return smax_dev_alloc(reinterpret_cast<void **>(p), bytes);
}

extern "C" int gt_smax_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

extern "C" void gt_smax_free(void *ptr) { free(ptr); }

#ifndef GT_SMAX_BUILD_ID
#define GT_SMAX_BUILD_ID "unknown"
#endif
extern "C" const char *gt_smax_build_id(void) { return GT_SMAX_BUILD_ID; }

extern "C" int gt_smax_dev_alloc_table(int device, uint64_t len,
                                       uint8_t **table, char *errbuf,
                                       size_t errlen) {
  // the table starts SMAX_TABLE_SHIFT bytes past a 128-byte line (smax_internal.h)
  uint8_t *p = NULL;
  HIPCHK(hipSetDevice(device));
  HIPCHK(hipMalloc(&p, len + SMAX_TABLE_SHIFT + GT_SMAX_PAD_FRONT + GT_SMAX_PAD_BACK));
  HIPCHK(hipMemset(p, 0, SMAX_TABLE_SHIFT + GT_SMAX_PAD_FRONT));
  HIPCHK(hipMemset(p + SMAX_TABLE_SHIFT + GT_SMAX_PAD_FRONT + len, 0, GT_SMAX_PAD_BACK));
  *table = p + SMAX_TABLE_SHIFT + GT_SMAX_PAD_FRONT;
  return 0;
fail:
  if (p) (void) hipFree(p);
  return -1;
}

extern "C" int gt_smax_dev_free_table(int device, uint8_t *table) {
  if (table == NULL) return 0;
  if (hipSetDevice(device) != hipSuccess) return -1;
  return hipFree(table - GT_SMAX_PAD_FRONT - SMAX_TABLE_SHIFT) == hipSuccess ? 0 : -1;
}

// tiles of the local grid [first, last] that hold owned rows [begin, end)
static uint32_t plan_tiles(const GtSmaxDevShard *s, uint64_t *first) {
  const uint64_t lo = (s->begin - s->base) / SMAX_TILE;
  const uint64_t hi = s->end > s->begin ? (s->end - 1 - s->base) / SMAX_TILE : lo;
  *first = lo;
  return (uint32_t) (hi - lo + 1);
}


// Warms the runtime's caching allocator for a plan over `shard` (every
// buffer gt_smax_plan_create will take, at its size -- K1b's record pool at
// an upper estimate, the cache serves a block of up to twice the request)
// and loads the scan kernels' code object, so that a plan created right
// after costs no cold hipMalloc: the host-table entry point runs this on a
// helper thread beside the staged upload of the shard's tables.
hipError_t smax_plan_reserve(const GtSmaxDevShard *shard, uint64_t capacity) {
  if (shard->begin < 1 || shard->begin > shard->end) return hipSuccess;
  uint64_t first = 0;
  const uint64_t nt = plan_tiles(shard, &first);
  if (capacity == 0) capacity = (shard->end - shard->begin) / 64 + 4096;
  const uint64_t cg = (nt + SMAX_CPB - 1) / SMAX_CPB;
  const uint64_t ngroups = GT_SMAX_PK_GROUPS(shard->local_len);
  const uint64_t wide_est = nt / 256 + std::max<uint64_t>(256u, nt / 256u);
  const size_t sizes[] = {
      sizeof (GtSmaxRecord) * capacity, sizeof (uint64_t) * SMAX_SSLOT * nt,
      sizeof (unsigned long long), sizeof (uint64_t) * nt, sizeof (uint32_t) * nt,
      sizeof (uint32_t) * (2 * smax_bs_stride(cg) + 1), sizeof (uint64_t), sizeof (GtSmaxBoundary),
      sizeof (uint2) * (nt + 2), sizeof (uint32_t), sizeof (uint32_t) * (2 * nt + 1),
      sizeof (uint2) * (2 * nt + 1), sizeof (uint32_t), sizeof (uint32_t), sizeof (uint32_t) * 8,
      sizeof (uint16_t) * (shard->numllv + 16), sizeof (uint4) * nt,
      sizeof (uint3) * ((nt + SMAX_IDX_BLK - 1) / SMAX_IDX_BLK + 1), sizeof (uint32_t) * ngroups,
      sizeof (uint64_t) * (std::max<uint64_t>(nt / 256u, 64u) / 2u + 1u),
      64 * nt, sizeof (uint32_t) * (nt + 1), sizeof (uint32_t)};
  // (not K1b's record pool: its size depends on the static list, an
  // estimate parked a block of up to ~2x the plan's need in the cache)
  (void) wide_est;
  constexpr size_t K = sizeof sizes / sizeof sizes[0];
  void *blk[K] = {};
  hipError_t e = hipSuccess;
  for (size_t i = 0; i < K && e == hipSuccess; i++) e = smax_dev_alloc(&blk[i], sizes[i]);
  for (size_t i = 0; i < K; i++) smax_dev_free(blk[i]);   // no work was enqueued on them
  int per_cu = 0;   // loads the code object (the first query or launch of a kernel does)
  if (e == hipSuccess)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, smax_scan_kernel_b2, SMAX_K1_THREADS, 0);
  return e;
}

typedef void (*SmaxScanFn)(SmaxScanArgs);

// The K1 variant a plan launches (its choices: packed or byte windows,
// 2-plane or u64-group stream, dense .llv, non-temporal) and its name
static SmaxScanFn plan_scan_fn(const GtSmaxPlan *p, const char **name) {
  const char *nm;
  SmaxScanFn f;
  if (!p->pk) { nm = "smax_scan_kernel_bytes"; f = smax_scan_kernel_bytes; }
#ifdef GT_SMAX_DIAG
  else if (p->dbg) { nm = "smax_scan_kernel_diag"; f = smax_scan_kernel_diag; }
#endif
  else if (p->bw2 && p->dense && p->nt) { nm = "smax_scan_kernel_b2_dense_nt"; f = smax_scan_kernel_b2_dense_nt; }
  else if (p->bw2 && p->dense) { nm = "smax_scan_kernel_b2_dense"; f = smax_scan_kernel_b2_dense; }
  else if (p->bw2 && p->nt) { nm = "smax_scan_kernel_b2_nt"; f = smax_scan_kernel_b2_nt; }
  else if (p->bw2) { nm = "smax_scan_kernel_b2"; f = smax_scan_kernel_b2; }
  else if (p->dense) { nm = "smax_scan_kernel_dense"; f = smax_scan_kernel_dense; }
  else { nm = "smax_scan_kernel"; f = smax_scan_kernel; }
  if (name) *name = nm;
  return f;
}

// K1's grid: generations of resident workgroups of the launched variant --
// the dispatcher hands a finished slot the next workgroup, which balances
// tiles of uneven cost (measured 9 % faster than one persistent generation
// on repeat-rich input).  The guided schedule (SMAX_K1_GUIDED) gives each
// generation 2/3 of the tiles left, so the launch ends on workgroups of one
// or two tiles (C3 -1.4 %, 1/8 shards -2.2 to -2.6 %, C5 -2.7 % against 8-16
// equal generations, profiles/s5/guided_ab_*; 1/2 and 3/4 measured in
// guided_fraction_ab_*).  Without it (or under GT_SMAX_GRID): 8 equal
// generations, up to 16 for tables of more than ~18 tiles per wave of one
// generation (profiles/r03i_*)
// The schedule table's second entry per workgroup: the llv_win words of its
// first tile and of the one after (the last of its range if none)
__global__ void __launch_bounds__(256)
smax_sched_info_kernel(uint4 *wg, uint32_t grid, const uint2 *llv_win) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= grid) return;
  const uint4 e = wg[2 * (size_t) b];
  const uint32_t t1 = e.x + e.y <= e.z - 1 ? e.x + e.y : e.z - 1;
  const uint2 w0 = llv_win[e.x], w1 = llv_win[t1];
  wg[2 * (size_t) b + 1] = make_uint4(w0.x, w0.y, w1.x, w1.y);
}

// The guided schedule of num_tiles tiles over `resident` workgroup slots:
// generation g = workgroups [blk[g], blk[g+1]) over tiles [tile[g],
// tile[g+1]), each taking ceil(2R / 3W) of the R tiles left per workgroup
// (the rest in one generation once that is below 2, or at the last of
// SMAX_SCHED_MAX); returns the generation count.  Exported for the host
// tests (tests/test_host_logic.py): every tile once, in order, each
// generation at most `resident` workgroups.
extern "C" uint32_t gt_smax_k1_schedule(uint32_t num_tiles, uint32_t resident, uint32_t *blk,
                                        uint32_t *tile) {
  const uint64_t W = resident ? resident : 1;
  uint64_t R = num_tiles, t0 = 0, b0 = 0;
  uint32_t n = 0;
  while (R > 0 && n < SMAX_SCHED_MAX) {
    uint64_t c = (SMAX_GUIDE_NUM * R + SMAX_GUIDE_DEN * W - 1) / (SMAX_GUIDE_DEN * W);
    if (c < 2 || n + 1 == SMAX_SCHED_MAX) c = (R + W - 1) / W;   // the rest, in one generation
    const uint64_t w = std::min<uint64_t>(W, (R + c - 1) / c);
    const uint64_t take = std::min<uint64_t>(R, w * c);
    blk[n] = (uint32_t) b0;
    tile[n] = (uint32_t) t0;
    b0 += w;
    t0 += take;
    R -= take;
    n++;
  }
  blk[n] = (uint32_t) b0;
  tile[n] = (uint32_t) t0;
  return n;
}

static hipError_t plan_size_grid(GtSmaxPlan *p) {
  int per_cu = 0;
  const char *name = nullptr;
  const SmaxScanFn f = plan_scan_fn(p, &name);
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, SMAX_K1_THREADS, 0);
  if (e != hipSuccess) return e;
  if (per_cu < 1) per_cu = 1;
  const uint64_t resident = (uint64_t) p->dev_cus * (uint64_t) per_cu;
  uint64_t gens = resident ? (uint64_t) p->num_tiles / (resident * (SMAX_K1_THREADS / 64) * 18) : 8;
  gens = gens < 8 ? 8 : gens > 16 ? 16 : gens;
  uint64_t g = resident * gens;
  const char *gs = getenv("GT_SMAX_GRID");     // diagnostic / test override
  if (gs && strtoul(gs, NULL, 0) > 0) g = strtoul(gs, NULL, 0);
  const uint64_t wg = ((uint64_t) p->num_tiles + SMAX_K1_THREADS / 64 - 1) /
                      (SMAX_K1_THREADS / 64);                // workgroups with a tile per wave
  p->grid = (uint32_t) (g < wg ? g : wg);
  if (p->grid < 1) p->grid = 1;
  // one generation: every workgroup strides the whole tile range
  p->sched_n = 1;
  p->sched_blk[0] = 0;
  p->sched_blk[1] = p->grid;
  p->sched_tile[0] = 0;
  p->sched_tile[1] = p->num_tiles;
#if SMAX_K1_GUIDED
  // guided: generation g of resident workgroups takes 2/3 of the tiles left
  // (ceil(2R / 3W) per wave), the last ones a tile or two each, so the
  // launch ends on short workgroups instead of a generation of equal ones
  // started late
  if (!(gs && strtoul(gs, NULL, 0) > 0) && resident > 0 && p->num_tiles > 0 &&
      SMAX_K1_THREADS == 64) {
    p->sched_n = gt_smax_k1_schedule(p->num_tiles, (uint32_t) resident, p->sched_blk, p->sched_tile);
    p->grid = p->sched_blk[p->sched_n];
  }
#endif
  if (getenv("GT_SMAX_VERBOSE")) {
    fprintf(stderr, "gt_smax: K1 %s, %u CUs x %d blocks/CU -> grid %u, %u tiles, schedule", name,
            p->dev_cus, per_cu, p->grid, p->num_tiles);
    for (uint32_t k = 0; k < p->sched_n; k++)
      fprintf(stderr, " [%u wgs: %u tiles]", p->sched_blk[k + 1] - p->sched_blk[k],
              p->sched_tile[k + 1] - p->sched_tile[k]);
    fprintf(stderr, "\n");
  }
  return hipSuccess;
}

static void plan_note_stream(GtSmaxPlan *p, hipStream_t s) {
  for (int i = 0; i < p->nstreams; i++)
    if (p->streams[i] == s) return;
  if (p->nstreams < SMAX_PLAN_STREAMS) p->streams[p->nstreams++] = s;
  else p->streams_overflow = true;
}

// waits for the work this plan enqueued (its streams), not for the device
static hipError_t plan_sync(GtSmaxPlan *p) {
  hipError_t e = hipSetDevice(p->shard.device);
  if (e == hipSuccess && p->streams_overflow) return hipDeviceSynchronize();
  for (int i = 0; e == hipSuccess && i < p->nstreams; i++) e = hipStreamSynchronize(p->streams[i]);
  return e;
}

extern "C" int gt_smax_plan_create(GtSmaxPlan **planp,
                                   const GtSmaxDevShard *shard,
                                   unsigned int minlen, uint64_t capacity,
                                   char *errbuf, size_t errlen) {
  GtSmaxPlan *p = (GtSmaxPlan *) calloc(1, sizeof *p);
  uint32_t *derr = NULL;
  uint32_t probe[5] = {0u, 0u, 0u, 0u, 0u};
  // plan-time scratch, returned once a blocking copy has passed its users
  uint4 *ihist = NULL;
  uint3 *ibsum = NULL;
  uint64_t *spec = NULL;
  *planp = NULL;
  if (p == NULL) { seterr(errbuf, errlen, "out of memory"); return -1; }
  if (minlen == 0) { seterr(errbuf, errlen, "minlen must be >= 1"); free(p); return -1; }
  if (shard->begin < 1 || shard->begin > shard->end ||
      shard->end > shard->nonspecials || shard->base + 1 > shard->begin ||
      shard->base + shard->local_len <= shard->end) {
    seterr(errbuf, errlen,
           "bad shard: base=%lu len=%lu begin=%lu end=%lu N=%lu",
           (unsigned long) shard->base, (unsigned long) shard->local_len,
           (unsigned long) shard->begin, (unsigned long) shard->end,
           (unsigned long) shard->nonspecials);
    free(p);
    return -1;
  }
  if (((uintptr_t) shard->lcp_dev & 15) || ((uintptr_t) shard->bwt_dev & 15) ||
      ((uintptr_t) shard->bwtpk_dev & 15)) {
    seterr(errbuf, errlen, "device tables must be 16-byte aligned");
    free(p);
    return -1;
  }
  if (shard->lcp_dev == NULL || (shard->bwt_dev == NULL && shard->bwtpk_dev == NULL)) {
    seterr(errbuf, errlen, "shard without an LCP or BWT table");
    free(p);
    return -1;
  }
  p->shard = *shard;
  p->minlen = minlen;
  p->num_tiles = plan_tiles(shard, &p->tile_first);
  if (capacity == 0) capacity = (shard->end - shard->begin) / 64 + 4096;
  p->capacity = capacity;
  p->dbg = 0;
#ifdef GT_SMAX_DIAG
  {
    const char *d = getenv("GT_SMAX_DEBUG");
    p->dbg = d ? (uint32_t) strtoul(d, NULL, 0) : 0u;
    // section stamps need the diagnostic kernel (a no-op ablation bit selects it)
    if (getenv("GT_SMAX_STAMPS")) p->dbg |= 1u << 30;
  }
#endif
  {
    const char *v = getenv("GT_SMAX_ALL_STATIC");
    p->all_static = (v && strtol(v, NULL, 0) != 0) || (p->dbg & 64u);
    v = getenv("GT_SMAX_BYTE_WINDOWS");
    p->byte_windows = (v && strtol(v, NULL, 0) != 0) || (p->dbg & 8192u);
  }
  double tpc = smax_phase_clock();
  HIPCHK(hipSetDevice(shard->device));
  plan_note_stream(p, nullptr);   // plan-time kernels: the null stream
  {
    int dev_cus = 0;
    HIPCHK(hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount,
                                 shard->device));
    // packed BWT: the caller's (ESA builder, host staging), or packed here
    // from the byte table when the shard's alphabet is DNA ({0..3} plus
    // specials) -- a plan-time pass over the .bwt bytes
    if (shard->bwtpk_dev != NULL && !(p->byte_windows && shard->bwt_dev != NULL)) {
      p->bwtpk = const_cast<uint64_t *>(shard->bwtpk_dev);
      p->pk = true;
      p->pk_owned = false;
    } else if (shard->bwt_dev == NULL) {
      seterr(errbuf, errlen, "byte BWT windows requested (GT_SMAX_BYTE_WINDOWS) but the shard has none");
      goto fail;
    } else {
      p->pk_owned = true;
      const uint64_t ngroups = GT_SMAX_PK_GROUPS(shard->local_len);
      uint32_t *flag = NULL, hflag = 0;
      HIPCHK(dalloc(&p->bwtpk, sizeof (uint64_t) * ngroups));
      HIPCHK(dalloc(&flag, sizeof (uint32_t)));
      HIPCHK(hipMemset(flag, 0, sizeof (uint32_t)));
      hipLaunchKernelGGL(smax_pack_bwt_kernel, dim3((unsigned) ((ngroups + 255) / 256)), dim3(256),
                         0, 0, shard->bwt_dev, shard->local_len, ngroups, p->bwtpk, flag);
      HIPCHK(hipGetLastError());
      HIPCHK(hipMemcpy(&hflag, flag, sizeof hflag, hipMemcpyDeviceToHost));
      smax_dev_free(flag);
      smax_phase_mark(" pack_bwt", &tpc);
      p->pk = hflag == 0 && !p->byte_windows;
      if (!p->pk) { smax_dev_free(p->bwtpk); p->bwtpk = NULL; }
    }
    p->dev_cus = (uint32_t) (dev_cus > 0 ? dev_cus : 256);
    p->compact_grid = (uint32_t) (((uint64_t) p->num_tiles + SMAX_CPB - 1) / SMAX_CPB);
    {
      // K3: each block of 256 tiles split over two workgroups (each copies
      // a share of its block's records), more until there are 8 workgroups
      // per CU (at most 8 per block).  Measured (profiles/r03zc/):
      // C3 (5,663 blocks) split 2 -0.8 % against 1 and -1 % against 4; a 3/8
      // shard (708 blocks) split 4 -3.3 % against 1, -0.6 % against 8; C2
      // (191 blocks, 3,365 records) +3 % with 8 -- tables of fewer than 256
      // blocks keep one.  GT_SMAX_K3_SPLIT overrides.
      const char *ks = getenv("GT_SMAX_K3_SPLIT");
      uint32_t sp = 1;
      if (ks) {
        sp = (uint32_t) strtoul(ks, NULL, 0);
      } else if (p->compact_grid >= 256) {
        sp = 2;
        while (sp < 8 && (uint64_t) p->compact_grid * sp < (uint64_t) dev_cus * 8u) sp *= 2;
      }
      p->k3_split = sp < 1 ? 1u : sp > 64 ? 64u : sp;
    }
  }
  smax_phase_mark(" occupancy", &tpc);
  HIPCHK(dalloc(&p->out, sizeof (GtSmaxRecord) * capacity));
  smax_phase_mark(" out_alloc", &tpc);
  HIPCHK(dalloc(&p->slots, sizeof (uint64_t) * SMAX_SSLOT * (uint64_t) p->num_tiles));
  // K1b's records: a wide slot per list entry for the static list and the
  // first num_tiles/256 runtime deferrals, then a pool for the rest
  p->wide_cap = 0;   // set once the static list is known (below)
  p->pool = NULL;
  HIPCHK(dalloc(&p->pool_cursor, sizeof (unsigned long long)));
  HIPCHK(dalloc(&p->tile_off, sizeof (uint64_t) * (uint64_t) p->num_tiles));
  smax_phase_mark(" slot_alloc", &tpc);
  HIPCHK(dalloc(&p->tile_count, sizeof (uint32_t) * (uint64_t) p->num_tiles));

  // two buffers: with the block sums added up in K1b's launch, run r adds
  // into buffer r % 2 and its K3 clears the other
  HIPCHK(dalloc(&p->block_sum, sizeof (uint32_t) * (2 * smax_bs_stride(p->compact_grid) + 1)));
  HIPCHK(hipMemset(p->block_sum, 0, sizeof (uint32_t) * (2 * smax_bs_stride(p->compact_grid) + 1)));

  HIPCHK(dalloc(&p->count, sizeof (uint64_t)));
  HIPCHK(hipMemset(p->count, 0, sizeof (uint64_t)));
  HIPCHK(dalloc(&p->bnd, sizeof (GtSmaxBoundary)));
  HIPCHK(hipMemset(p->bnd, 0, sizeof (GtSmaxBoundary)));
  // + 2 zeroed entries: the dummy .llv record of K1's unconditional loads
  HIPCHK(dalloc(&p->llv_win, sizeof (uint2) * (p->num_tiles + 2)));
  HIPCHK(hipMemset(p->llv_win, 0, sizeof (uint2) * (p->num_tiles + 2)));
  HIPCHK(dalloc(&p->err, sizeof (uint32_t)));
  HIPCHK(hipMemset(p->err, 0, sizeof (uint32_t)));
#ifdef GT_SMAX_DIAG
  if (getenv("GT_SMAX_STAMPS")) {
    HIPCHK(dalloc(&p->stamps, sizeof (unsigned long long) * 8));
    HIPCHK(hipMemset(p->stamps, 0, sizeof (unsigned long long) * 8));
  }
#endif
  // K1's runtime list; in the combined placement (mode 4) the static list is
  // copied to its front and K1 appends behind it
  HIPCHK(dalloc(&p->defer_list, sizeof (uint32_t) * (2 * (uint64_t) p->num_tiles + 1)));
  HIPCHK(dalloc(&p->defer_info, sizeof (uint2) * (2 * (uint64_t) p->num_tiles + 1)));
  HIPCHK(dalloc(&p->defer_count, sizeof (uint32_t)));
  HIPCHK(hipMemset(p->defer_count, 0, sizeof (uint32_t)));
  HIPCHK(dalloc(&p->defer_last, sizeof (uint32_t)));
  HIPCHK(hipMemset(p->defer_last, 0, sizeof (uint32_t)));
  // plan-time scalars read back by the host: [0] the .llv errors, [1] the
  // special groups in the windows' range, [2..6] smax_plan_probe_kernel's
  HIPCHK(dalloc(&derr, sizeof (uint32_t) * 8));
  HIPCHK(hipMemset(derr, 0, sizeof (uint32_t) * 8));
  if (shard->numllv > 0xffffffffull) {
    seterr(errbuf, errlen, "more than 2^32 .llv entries in one shard");
    goto fail;
  }
  {
    // the .llv window index: run starts of the entries over the tiles' keys,
    // max-scanned (smax_llv_hist_kernel)
    HIPCHK(dalloc(&p->llv16, sizeof (uint16_t) * (shard->numllv + 16)));
    HIPCHK(hipMemset(p->llv16 + shard->numllv, 0, sizeof (uint16_t) * 16));
    if (shard->numllv)
      hipLaunchKernelGGL(smax_llv16_kernel, dim3((unsigned) ((shard->numllv + 255) / 256)),
                         dim3(256), 0, 0, shard->llv_dev, shard->numllv, p->llv16);
    HIPCHK(hipGetLastError());
    if (p->num_tiles > 0) {
      const uint64_t nt = p->num_tiles;
      const int64_t g0f = (int64_t) (shard->base + p->tile_first * (uint64_t) SMAX_TILE);
      SmaxLlvKeys k;
      k.a_lo = g0f - SMAX_LH;
      k.a_hi = g0f + SMAX_TILE + SMAX_RH;
      k.a_g0 = g0f;
      k.num_tiles = p->num_tiles;
      const uint32_t nb = (uint32_t) ((nt + SMAX_IDX_BLK - 1) / SMAX_IDX_BLK);
      HIPCHK(dalloc(&ihist, sizeof (uint4) * nt));
      HIPCHK(dalloc(&ibsum, sizeof (uint3) * nb));
      HIPCHK(hipMemset(ihist, 0, sizeof (uint4) * nt));
      hipLaunchKernelGGL(smax_llv_hist_kernel, dim3((unsigned) ((shard->numllv + 1 + 255) / 256)),
                         dim3(256), 0, 0, shard->llv_dev, shard->numllv, k, ihist, derr);
      hipLaunchKernelGGL(smax_llv_bsum_kernel, dim3(nb), dim3(256), 0, 0, ihist, p->num_tiles, ibsum);
      hipLaunchKernelGGL(smax_llv_btop_kernel, dim3(1), dim3(256), 0, 0, ibsum, nb);
      hipLaunchKernelGGL(smax_llv_win_kernel, dim3(nb), dim3(256), 0, 0, ihist, ibsum, p->num_tiles,
                         (uint64_t) g0f, shard->begin, shard->end, p->llv_win,
                         p->all_static ? 1u : 0u);
      HIPCHK(hipGetLastError());
    } else if (shard->numllv) {
      // no tiles: only the entries' checks
      const SmaxLlvKeys k = {0, 0, 0, 0u};
      hipLaunchKernelGGL(smax_llv_hist_kernel, dim3((unsigned) ((shard->numllv + 1 + 255) / 256)),
                         dim3(256), 0, 0, shard->llv_dev, shard->numllv, k, (uint4 *) NULL, derr);
      HIPCHK(hipGetLastError());
    }
  }
  smax_phase_mark(" llv_index", &tpc);
  // K1's 2-plane window stream: the packed BWT without its special plane
  // (0.25 B per row instead of 0.5); a window that holds a special BWT row
  // goes to the static K1b list, which reads the full packed form.  The plan
  // picks it unless that list would grow by more than 1/256 of the tiles
  // (read sets: a separator every few hundred rows puts a special BWT row in
  // most windows, and a K1b tile costs ~14 K1 tiles; K1 then streams the u64
  // groups, specials and all).  GT_SMAX_BW2=0/1 overrides; the diagnostic
  // kernel is a 2-plane one.  The planes are written in the same pass that
  // counts the special groups, and dropped when the plan does not take them.
  {
    uint32_t h[2] = {0u, 0u};
    uint32_t spec_cap = 0;
    if (p->pk) {
      const uint64_t ngroups = GT_SMAX_PK_GROUPS(shard->local_len);
      const uint64_t g_lo = p->tile_first * (SMAX_TILE / 16);     // groups the windows read
      const uint64_t g_hi = std::min<uint64_t>(g_lo + (uint64_t) p->num_tiles * (SMAX_TILE / 16) + 2,
                                               ngroups);
      spec_cap = std::max<uint32_t>(p->num_tiles / 256u, 64u) / 2u + 1u;
      HIPCHK(dalloc(&p->bwt2, sizeof (uint32_t) * ngroups));
      HIPCHK(dalloc(&spec, sizeof (uint64_t) * spec_cap));
      hipLaunchKernelGGL(smax_bwt2_kernel, dim3((unsigned) std::min<uint64_t>((ngroups + 255) / 256, 1u << 20)),
                         dim3(256), 0, 0, p->bwtpk, ngroups, p->bwt2, g_lo, g_hi, derr + 1, spec,
                         spec_cap);
      HIPCHK(hipGetLastError());
    }
    HIPCHK(hipMemcpy(h, derr, sizeof h, hipMemcpyDeviceToHost));   // the index kernels are done
    smax_phase_mark(" index+bwt2", &tpc);
    smax_dev_free(ibsum);
    smax_dev_free(ihist);
    ibsum = NULL;
    ihist = NULL;
    if (h[0] & 1u) { seterr(errbuf, errlen, "lcp value >= 2^32 in .llv"); goto fail; }
    if (h[0] & 2u) { seterr(errbuf, errlen, ".llv positions not strictly increasing"); goto fail; }
    if (p->pk) {
      const char *b2 = getenv("GT_SMAX_BW2");
      const uint32_t nsp = h[1];
      // a special group flags at most two windows
      // (the diagnostic kernel streams the 2-plane form: bw2 whatever
      // GT_SMAX_BW2 says while GT_SMAX_DEBUG/STAMPS select it)
      p->bw2 = p->dbg != 0 ? true
             : b2 ? strtol(b2, NULL, 0) != 0
                  : 2ull * nsp <= std::max<uint32_t>(p->num_tiles / 256u, 64u);
      if (p->bw2 && nsp > 0) {
        const uint64_t ngroups = GT_SMAX_PK_GROUPS(shard->local_len);
        const bool listed = nsp <= spec_cap;
        const uint64_t n = listed ? nsp : ngroups;
        hipLaunchKernelGGL(smax_spec_mark_kernel, dim3((unsigned) std::min<uint64_t>((n + 255) / 256, 1u << 20)),
                           dim3(256), 0, 0, listed ? spec : (const uint64_t *) NULL, p->bwtpk, n,
                           p->llv_win, p->tile_first, (uint64_t) p->num_tiles);
        HIPCHK(hipGetLastError());
      }
      if (!p->bw2) {
        smax_dev_free(p->bwt2);
        p->bwt2 = NULL;
      }
    }
  }
  // static K1b list (needs llv_win), copied to the front of K1b's list: one
  // K1b launch after K1 runs the static tiles, then K1's deferrals (a second
  // stream beside K1 cost a fork/join event pair per step, ~25 us,
  // DESIGN.md §4)
  HIPCHK(dalloc(&p->static_list, sizeof (uint32_t) * ((uint64_t) p->num_tiles + 1)));
  HIPCHK(dalloc(&p->static_count, sizeof (uint32_t)));
  HIPCHK(hipMemset(p->static_count, 0, sizeof (uint32_t)));
  {
    SmaxScanArgs a = plan_args(p);
    if (p->num_tiles > 0)
      hipLaunchKernelGGL(smax_static_defer_kernel, dim3((p->num_tiles + 255) / 256), dim3(256), 0, 0,
                       a, p->static_list, p->static_count);
    hipLaunchKernelGGL(smax_plan_probe_kernel, dim3(1), dim3(64), 0, 0, p->static_count,
                       (const uint2 *) p->llv_win, p->num_tiles, derr + 2);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpy(probe, derr + 2, sizeof probe, hipMemcpyDeviceToHost));
    p->n_static = probe[0];
    smax_phase_mark(" static_list", &tpc);
    smax_dev_free(spec);   // the marking kernel is done
    spec = NULL;
    p->wide_cap = p->n_static + std::max<uint32_t>(256u, p->num_tiles / 256u);
    HIPCHK(dalloc(&p->pool, sizeof (GtSmaxRecord) *
                                ((uint64_t) p->wide_cap * (SMAX_TILE / 2) + capacity)));
    if (p->n_static) {
      HIPCHK(hipMemcpy(p->defer_list, p->static_list, sizeof (uint32_t) * p->n_static,
                       hipMemcpyDeviceToDevice));
      hipLaunchKernelGGL(smax_defer_info_kernel, dim3((p->n_static + 255) / 256), dim3(256), 0, 0,
                         p->defer_list, p->n_static, p->llv_win, p->defer_info);
      HIPCHK(hipGetLastError());
    }
  }
  smax_phase_mark(" static_k1b", &tpc);
  {
    // density over the plan's own tiles (a shard plan over full tables
    // sees every .llv entry): first entry of the first window to the end
    // of the last one
    const char *dv = getenv("GT_SMAX_DENSE");   // diagnostic override: 0 / 1
    const uint2 w0 = make_uint2(probe[1], probe[2]), w1 = make_uint2(probe[3], probe[4]);
    const uint64_t inrange = (uint64_t) w1.x + SMAX_WIN_N(w1.y) - w0.x;
    const uint64_t rows = (uint64_t) p->num_tiles * SMAX_TILE;
    p->dense = dv ? strtol(dv, NULL, 0) != 0
                  : rows > 0 && (double) inrange > SMAX_FFPV_DENSITY * (double) rows;
  }
  {
    // non-temporal window stream where it measured faster: the shard's
    // stream (1.5 B per row) larger than the 256 MB MALL -- a smaller one
    // is served from it on repeated passes, which nt gives up -- and at
    // most 2^19 tiles (the 4- and 8-way C3 splits; the whole 3 Gbp table
    // measured slower).  2-plane windows only.  GT_SMAX_NT=0/1 overrides.
    const char *ntv = getenv("GT_SMAX_NT");
    const uint64_t stream_bytes = (uint64_t) p->num_tiles * SMAX_TILE * 3 / 2;
    p->nt = p->bw2 && (ntv ? strtol(ntv, NULL, 0) != 0
                           : stream_bytes > (256ull << 20) && p->num_tiles <= (1u << 19));
  }
  // K1's grid, from the occupancy of the variant this plan launches (the
  // u64-group kernels hold 5 waves per SIMD, the 2-plane ones 6)
  smax_phase_mark(" pool", &tpc);
  HIPCHK(plan_size_grid(p));
  if (p->sched_n > 1) {
    // the schedule's per-workgroup entries: {first tile, stride, end, 0},
    // then the llv_win words of the workgroup's first two tiles (filled on
    // the device from llv_win): a workgroup's prologue is one scalar load
    // and its first window DMA, not three dependent round trips
    std::vector<uint4> wg(2 * (size_t) p->grid, make_uint4(0u, 0u, 0u, 0u));
    for (uint32_t g = 0; g < p->sched_n; g++) {
      const uint32_t b0 = p->sched_blk[g], w = p->sched_blk[g + 1] - b0;
      for (uint32_t j = 0; j < w; j++)
        wg[2 * (size_t) (b0 + j)] = make_uint4(p->sched_tile[g] + j, w, p->sched_tile[g + 1], 0u);
    }
    HIPCHK(dalloc(&p->sched_wg, sizeof (uint4) * wg.size()));
    HIPCHK(hipMemcpy(p->sched_wg, wg.data(), sizeof (uint4) * wg.size(), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(smax_sched_info_kernel, dim3((p->grid + 255) / 256), dim3(256), 0, 0,
                       p->sched_wg, p->grid, (const uint2 *) p->llv_win);
    HIPCHK(hipGetLastError());
  }
  {
    // K1b: a workgroup per tile -- the static list plus K1's deferrals
    // (about one tile in 10^4) -- in one generation on all CUs where they fit;
    // the first workgroup computes the boundary head
    int ncu = 256;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, shard->device) !=
            hipSuccess || ncu < 1)
      ncu = 256;
    p->k1b_grid = std::min<uint32_t>(p->n_static + p->num_tiles / SMAX_K1B_SLACK + 64u, (uint32_t) ncu * 8u) + 1;
    // 8 waves per tile (each tile's ballots and evaluation split twice as
    // fine) when the launch -- tiles, the head and the block-sum workgroups
    // -- fits one generation of the 8-wave kernel (two per CU), else 4 (five
    // per CU).  GT_SMAX_K1B_WAVES=4/8 overrides.
    {
      int per8 = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per8, smax_defer_wg_kernel<8>, 512, 0) !=
          hipSuccess)
        per8 = 0;
      const uint64_t need8 = (uint64_t) p->k1b_grid + (p->compact_grid + 7u) / 8u;
      const char *kw = getenv("GT_SMAX_K1B_WAVES");
      p->k1b_nw = kw ? (strtol(kw, NULL, 0) == 8 ? 8u : 4u)
                     : (per8 > 0 && need8 <= (uint64_t) per8 * (uint64_t) ncu ? 8u : 4u);
    }
    // K3's block sums in the same launch (K2's work without its launch):
    // K1b's last workgroups, one block per wave (measured against a separate
    // block-sum kernel: C3 step -0.3 %, 3/8 shard -1.4 %, C2 -4.2 %,
    // profiles/r03zb/fuse_bs_*.txt)
    p->bs_wgs = (p->compact_grid + p->k1b_nw - 1) / p->k1b_nw;
    // the first run's state (later runs: reset by the previous run's K3)
    const unsigned long long pc = (unsigned long long) p->wide_cap * (SMAX_TILE / 2);
    HIPCHK(hipMemcpy(p->defer_count, &p->n_static, sizeof (uint32_t), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(p->pool_cursor, &pc, sizeof pc, hipMemcpyHostToDevice));
  }
  smax_phase_mark(" schedule", &tpc);
  smax_dev_free(derr);   // past the blocking copies above
  *planp = p;
  return 0;
fail:
  (void) hipStreamSynchronize(nullptr);   // plan-time kernels (null stream) may still use the scratch
  smax_dev_free(derr);
  smax_dev_free(ibsum);
  smax_dev_free(ihist);
  smax_dev_free(spec);
  gt_smax_plan_delete(p);
  return -1;
}

extern "C" void gt_smax_plan_delete(GtSmaxPlan *p) {
  if (p == NULL) return;
  (void) hipSetDevice(p->shard.device);
  void *bufs[] = {p->out, p->slots, p->pool, p->pool_cursor, p->tile_off, p->tile_count, p->block_sum, p->count, p->bnd, p->defer_last, p->stamps, p->bwt2, p->sched_wg,
                  p->llv_win, p->err, p->pk_owned ? p->bwtpk : NULL, p->llv16, p->defer_list, p->defer_info,
                  p->defer_count, p->static_list, p->static_count};
  // stream-ordered: the buffers go back to the cache behind events on the
  // streams this plan's work ran on (a plan closed right after run() must
  // not hand them to the next allocation while K1..K3 still write them);
  // nothing here waits, and no other stream of the device is involved
  SmaxFence *fence = smax_fence_create(p->streams, p->streams_overflow ? -1 : p->nstreams);
  for (size_t i = 0; i < sizeof bufs / sizeof bufs[0]; i++)
    if (bufs[i]) smax_dev_free_fenced(bufs[i], fence);
  smax_fence_release(fence);
  for (int i = 0; i < 2 * p->nslots; i++) (void) hipEventDestroy(p->ev[i]);
  free(p->ev);
  free(p);
}

static SmaxScanArgs plan_args(GtSmaxPlan *p) {
  SmaxScanArgs a;
  a.lcp = p->shard.lcp_dev;
  a.bwt = p->shard.bwt_dev;
  a.bwtpk = p->pk ? p->bwtpk : nullptr;
  a.bwt2 = p->bw2 ? p->bwt2 : nullptr;
  a.llv16 = p->llv16;
  a.llv = p->shard.llv_dev;
  a.numllv = p->shard.numllv;
  a.llv_win = p->llv_win;
  a.base = p->shard.base;
  a.begin = p->shard.begin;
  a.end = p->shard.end;
  a.N = p->shard.nonspecials;
  a.local_len = p->shard.local_len;
  a.err = p->err;
  a.tile_first = p->tile_first;
  a.minlen = p->minlen;
  a.num_tiles = p->num_tiles;
  a.slots = p->slots;
  a.pool = p->pool;
  a.pool_cap = (uint64_t) p->wide_cap * (SMAX_TILE / 2) + p->capacity;
  a.wide_cap = p->wide_cap;
  a.wide_slot0 = 0;               // K1b's list: the static entries, then K1's
  a.defer_base = p->n_static;
  a.pool_cursor = p->pool_cursor;
  a.tile_off = p->tile_off;
  a.tile_count = p->tile_count;
  a.block_sum = p->block_sum + p->bs_buf * smax_bs_stride(p->compact_grid);
  a.bs_wgs = p->bs_wgs;
  a.bnd = p->bnd;
  a.defer_list = p->defer_list;
  a.defer_info = p->defer_info;
  a.defer_count = p->defer_count;
  a.k1b_head = 0;
  a.k1_reset = 0;
  a.dbg = p->dbg;
  a.stamps = p->stamps;
  a.sched_wg = p->sched_n > 1 ? p->sched_wg : nullptr;
  return a;
}

static int plan_run_scan(GtSmaxPlan *p, hipStream_t s);
static int plan_run_compact(GtSmaxPlan *p, hipStream_t s);

// parts: bit 0 = the scan (K1 and K1b; the boundary record is final after
// it), bit 1 = the ordered compaction (K3).  gt_smax_plan_run
// enqueues both; a sharded caller can enqueue part 0, start the boundary
// all-gather on its communication stream, then part 1 beside it.
static int plan_run_parts(GtSmaxPlan *p, hipStream_t s, unsigned parts) {
  char *errbuf = NULL;
  size_t errlen = 0;
  HIPCHK(hipSetDevice(p->shard.device));
  plan_note_stream(p, s);
  // K3 of part 1 resets the deferral list and pool cursor the next part 0's
  // K1/K1b start from: a second part 0 before that part 1 would run on stale
  // state (and part 1 without a part 0 would compact stale tiles)
  if ((parts & 1u) && p->part1_pending) {
    fprintf(stderr, "gt_smax: gt_smax_plan_run_part(0) called again before part 1\n");
    return -1;
  }
  if (parts == 2u && !p->part1_pending) {
    fprintf(stderr, "gt_smax: gt_smax_plan_run_part(1) without a pending part 0\n");
    return -1;
  }
  if (p->shard.begin >= p->shard.end) {
    p->part1_pending = (parts == 1u);
    if (parts & 1u) return plan_run_scan(p, s);
    return 0;
  }
  if ((parts & 1u) && plan_run_scan(p, s) != 0) return -1;
  p->part1_pending = true;
  if ((parts & 2u) && plan_run_compact(p, s) != 0) return -1;
  if (parts & 2u) p->part1_pending = false;
  return 0;
fail:
  return -1;
}

extern "C" int gt_smax_plan_run(GtSmaxPlan *p, void *stream) {
  return plan_run_parts(p, (hipStream_t) stream, 3u);
}

extern "C" int gt_smax_plan_run_part(GtSmaxPlan *p, int part, void *stream) {
  if (part != 0 && part != 1) return -1;
  return plan_run_parts(p, (hipStream_t) stream, 1u << part);
}

static int plan_run_scan(GtSmaxPlan *p, hipStream_t s) {
  char *errbuf = NULL;
  size_t errlen = 0;
  SmaxScanArgs a = plan_args(p);
  if (p->shard.begin >= p->shard.end) {
    // empty shard: K0 alone (the boundary head, the per-run resets)
    hipLaunchKernelGGL(smax_head_kernel, dim3(1), dim3(64), 0, s, a);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemsetAsync(p->count, 0, sizeof (uint64_t), s));
    return 0;
  }
  // no K0: K1 clears the pending-plateau slot, the previous run's K3 reset
  // the deferral count and the pool cursor
  a.k1_reset = 1u;
  {
    const uint64_t ts = p->tstride > 1 ? (uint64_t) p->tstride : 1u;
    const int slot = p->nslots && p->runs % ts == 0 ? (int) ((p->runs / ts) % (uint64_t) p->nslots)
                                                    : -1;
    if (slot >= 0) HIPCHK(hipEventRecord(p->ev[2 * slot], s));
    const dim3 g(p->grid), b(SMAX_K1_THREADS);
    void *kargs_[] = {&a};
    HIPCHK(hipLaunchKernel(reinterpret_cast<const void *>(plan_scan_fn(p, nullptr)), g, b, kargs_, 0, s));
    HIPCHK(hipGetLastError());
    if (slot >= 0) HIPCHK(hipEventRecord(p->ev[2 * slot + 1], s));
  }
  {
    // K1b over the static list and K1's deferrals, one launch; its first
    // workgroup computes the boundary head, its last ones the block sums
    SmaxScanArgs c = a;
    c.k1b_head = 1;
    if (p->k1b_nw == 8)
      hipLaunchKernelGGL(smax_defer_wg_kernel<8>, dim3(p->k1b_grid + p->bs_wgs), dim3(512), 0, s, c);
    else
      hipLaunchKernelGGL(smax_defer_wg_kernel<4>, dim3(p->k1b_grid + p->bs_wgs), dim3(256), 0, s, c);
    HIPCHK(hipGetLastError());
  }
  return 0;
fail:
  return -1;
}

static int plan_run_compact(GtSmaxPlan *p, hipStream_t s) {
  char *errbuf = NULL;
  size_t errlen = 0;
  {
    // block sums added up in K1b's launch into this run's buffer; K3 clears
    // the other one for the next run and resets the deferral state K1b was
    // the last to read
    uint32_t *bs = p->block_sum + p->bs_buf * smax_bs_stride(p->compact_grid);
    uint32_t *bs_clear = p->block_sum + (p->bs_buf ^ 1u) * smax_bs_stride(p->compact_grid);
    SmaxNextRun nr;
    nr.defer_count = p->defer_count;
    nr.defer_last = p->defer_last;
    nr.pool_cursor = p->pool_cursor;
    nr.defer_base = p->n_static;
    nr.pool_start = (unsigned long long) p->wide_cap * (SMAX_TILE / 2);
    hipLaunchKernelGGL(smax_compact_kernel, dim3(p->compact_grid * p->k3_split), dim3(256), 0, s,
                       p->slots, p->tile_count, bs, (uint64_t) p->num_tiles,
                       p->pool, (uint64_t) p->wide_cap * (SMAX_TILE / 2) + p->capacity,
                       p->tile_off, p->out, p->capacity, p->count,
                       p->shard.base + p->tile_first * (uint64_t) SMAX_TILE, nr, bs_clear,
                       p->k3_split);
    HIPCHK(hipGetLastError());
  }
  p->bs_buf ^= 1u;
  p->runs++;
  return 0;
fail:
  return -1;
}

extern "C" GtSmaxRecord *gt_smax_plan_records(GtSmaxPlan *p) { return p->out; }
extern "C" uint64_t *gt_smax_plan_count_dev(GtSmaxPlan *p) { return p->count; }
extern "C" GtSmaxBoundary *gt_smax_plan_boundary_dev(GtSmaxPlan *p) { return p->bnd; }
extern "C" uint64_t gt_smax_plan_capacity(GtSmaxPlan *p) { return p->capacity; }
extern "C" uint64_t gt_smax_plan_num_tiles(GtSmaxPlan *p) { return p->num_tiles; }

extern "C" int gt_smax_plan_stitch(GtSmaxPlan *p, const GtSmaxBoundary *all_dev,
                                   int nshards, int shard_index, void *stream) {
  char *errbuf = NULL;
  size_t errlen = 0;
  HIPCHK(hipSetDevice(p->shard.device));
  plan_note_stream(p, (hipStream_t) stream);
  hipLaunchKernelGGL(smax_stitch_kernel, dim3(1), dim3(64), 0,
                     (hipStream_t) stream, all_dev, nshards, shard_index,
                     p->minlen, p->out, p->capacity, p->count);
  HIPCHK(hipGetLastError());
  return 0;
fail:
  return -1;
}

extern "C" int gt_smax_stitch_host(const GtSmaxBoundary *all, int nshards,
                                   int shard_index, unsigned int minlen,
                                   GtSmaxRecord *rec) {
  return stitch_resolve(all, nshards, shard_index, minlen, rec);
}

extern "C" int gt_smax_plan_timing_stride(GtSmaxPlan *p, int stride) {
  if (stride < 1) return -1;
  p->tstride = stride;
  p->runs = 0;
  return 0;
}

extern "C" int gt_smax_plan_timing(GtSmaxPlan *p, int nslots) {
  char *errbuf = NULL;
  size_t errlen = 0;
  HIPCHK(hipSetDevice(p->shard.device));
  for (int i = 0; i < 2 * p->nslots; i++) (void) hipEventDestroy(p->ev[i]);
  free(p->ev);
  p->ev = NULL;
  p->nslots = 0;
  p->runs = 0;
  if (nslots <= 0) return 0;
  p->ev = (hipEvent_t *) calloc((size_t) (2 * nslots), sizeof (hipEvent_t));
  if (p->ev == NULL) return -1;
  p->nslots = nslots;
  for (int i = 0; i < 2 * nslots; i++) HIPCHK(hipEventCreate(&p->ev[i]));
  return 0;
fail:
  return -1;
}

extern "C" int gt_smax_plan_timing_read(GtSmaxPlan *p, double *sum_ms, int *nread) {
  char *errbuf = NULL;
  size_t errlen = 0;
  double acc = 0.0;
  const uint64_t ts = p->tstride > 1 ? (uint64_t) p->tstride : 1u;
  const uint64_t timed = (p->runs + ts - 1) / ts;
  const int n = (int) (timed < (uint64_t) p->nslots ? timed : (uint64_t) p->nslots);
  HIPCHK(hipSetDevice(p->shard.device));
  for (int i = 0; i < n; i++) {
    float ms = 0.0f;
    HIPCHK(hipEventSynchronize(p->ev[2 * i + 1]));
    HIPCHK(hipEventElapsedTime(&ms, p->ev[2 * i], p->ev[2 * i + 1]));
    acc += ms;
  }
  *sum_ms = acc;
  *nread = n;
  return 0;
fail:
  return -1;
}

extern "C" int gt_smax_plan_copy_boundary(GtSmaxPlan *p, void *dst_dev, void *stream) {
  char *errbuf = NULL;
  size_t errlen = 0;
  HIPCHK(hipSetDevice(p->shard.device));
  plan_note_stream(p, (hipStream_t) stream);
  HIPCHK(hipMemcpyAsync(dst_dev, p->bnd, sizeof (GtSmaxBoundary),
                        hipMemcpyDeviceToDevice, (hipStream_t) stream));
  return 0;
fail:
  return -1;
}

extern "C" int gt_smax_plan_fetch_count(GtSmaxPlan *p, uint64_t *count) {
  char *errbuf = NULL;
  size_t errlen = 0;
  uint32_t e = 0;
  HIPCHK(plan_sync(p));
  HIPCHK(hipMemcpy(count, p->count, sizeof (uint64_t), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(&e, p->err, sizeof e, hipMemcpyDeviceToHost));
  if (e != 0) {
    fprintf(stderr, "gt_smax: inconsistent index (device error bits 0x%x)\n", e);
    return -1;
  }
  return 0;
fail:
  return -1;
}


extern "C" int gt_smax_plan_fetch_triples(GtSmaxPlan *p, uint64_t *lcp_lb_rb, uint64_t capacity,
                                          uint64_t *count) {
  char *errbuf = NULL;
  size_t errlen = 0;
  uint64_t c = 0;
  if (gt_smax_plan_fetch_count(p, &c)) return -1;
  *count = c;
  if (c > p->capacity || c > capacity) return -1;   // caller re-plans / enlarges
  HIPCHK(smax_d2h_triples(lcp_lb_rb, p->out, c, 0));
  return 0;
fail:
  return -1;
}

extern "C" uint32_t gt_smax_plan_deferred_tiles(GtSmaxPlan *p) {
  uint32_t n = 0;
  if (hipSetDevice(p->shard.device) != hipSuccess) return 0xffffffffu;
  // K3 resets the live count; its last value is kept
  if (hipMemcpy(&n, p->defer_last, sizeof n, hipMemcpyDeviceToHost) != hipSuccess)
    return 0xffffffffu;
  return n - p->n_static;   // K1's deferrals only
}

extern "C" int gt_smax_plan_debug_tiles(GtSmaxPlan *p, uint32_t *counts, uint32_t *deferred,
                                        uint32_t *ndeferred) {
  if (plan_sync(p) != hipSuccess) return -1;
  if (counts && hipMemcpy(counts, p->tile_count, sizeof (uint32_t) * (uint64_t) p->num_tiles,
                          hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  if (counts && !(p->dbg & 32768u))
    for (uint64_t i = 0; i < p->num_tiles; i++) counts[i] &= ~SMAX_SLOT_WIDE;   // slot-format flag
  uint32_t n = 0;
  if (hipMemcpy(&n, p->defer_last, sizeof n, hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  const uint32_t base = p->n_static;   // K1b's list: K1's part follows the static entries
  n -= base;
  if (ndeferred) *ndeferred = n;
  if (deferred && n && hipMemcpy(deferred, p->defer_list + base, sizeof (uint32_t) * n,
                                 hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return 0;
}

extern "C" int gt_smax_plan_debug_windows(GtSmaxPlan *p, uint32_t *words) {
  if (plan_sync(p) != hipSuccess) return -1;
  if (p->num_tiles && hipMemcpy(words, p->llv_win, sizeof (uint2) * (uint64_t) p->num_tiles,
                                hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return 0;
}

// diagnostic: K1's per-section cycle sums (GT_SMAX_STAMPS plans; 8 values:
// wait, flush+issue, filter, classify+queue, exact starts, output, staging,
// tiles); -1 if the plan has none
extern "C" uint32_t gt_smax_plan_k1b_waves(const GtSmaxPlan *p) { return p->k1b_nw; }

extern "C" const char *gt_smax_plan_scan_kernel(const GtSmaxPlan *p) {
  // the selection of plan_run_scan
  const char *name = nullptr;
  (void) plan_scan_fn(p, &name);
  return name;
}

extern "C" int gt_smax_plan_stamps(GtSmaxPlan *p, unsigned long long *out8) {
  if (p->stamps == nullptr) return -1;
  if (plan_sync(p) != hipSuccess) return -1;
  return hipMemcpy(out8, p->stamps, sizeof (unsigned long long) * 8, hipMemcpyDeviceToHost) ==
                 hipSuccess ? 0 : -1;
}

extern "C" uint32_t gt_smax_plan_error_bits(GtSmaxPlan *p) {
  uint32_t e = 0;
  if (hipSetDevice(p->shard.device) != hipSuccess) return 0xffffffffu;
  if (hipMemcpy(&e, p->err, sizeof e, hipMemcpyDeviceToHost) != hipSuccess) return 0xffffffffu;
  return e;
}
