/*
 * gt_smax_hip.h -- C-ABI of the MI355X supermaximal-repeat (smax) layer.
 *
 * Drop-in boundary for the smax hot path of GenomeTools.
 * Plain C types only: a C host (the gt repfind runner, esa_linsmax.c, the
 * repo's own CLI) links libgtsmax_hip.so and never sees HIP or torch types.
 *
 * Each entry point names the reference interface it replaces:
 *
 *  gt_smax_hip_enumerate          replaces the bottom-up traversal driving a
 *                                 GtESAVisitor lcp-interval callback:
 *                                 gt_esa_bottomup(ssar, visitor, err)
 *                                   src/match/esa-bottomup.h:31-33,
 *                                   src/match/esa-bottomup.c:116-273
 *                                 visit_lcp_interval(lcp, lb, rb)
 *                                   src/match/esa_visitor_rep.h:46-51
 *                                 and the maxpairs driver pattern
 *                                 gt_callenummaxpairs
 *                                   src/match/esa-maxpairs.c:476-520
 *                                 Intervals arrive in ascending lb, the order
 *                                 in which the bottom-up traversal pops
 *                                 leaf-only intervals.
 *  gt_smax_hip_enumerate_to_buffer  same, returning a malloc'd array.
 *  GtSmaxInput                    the mapped tables of Suffixarray
 *                                   src/match/sarr-def.h:101-126
 *                                 as exposed by
 *                                   gt_suffixarraySequentialsuffixarrayreader
 *                                   src/match/esa-seqread.h:238-239
 *  GtSmaxLlv                      Largelcpvalue {position,value} on LP64
 *                                   src/match/lcpoverflow.h:23-30
 *
 * The gt_smax_dev_* functions are the device-resident form used when the
 * tables already live in HBM (one process per GPU under torch.distributed):
 * they enqueue work on a caller-provided HIP stream and never synchronise
 * except where documented.
 *
 * Conventions follow GenomeTools: 0 = success, -1 = error with a message in
 * errbuf (the gt shim copies it into GtError via gt_error_set, as
 * src/match/esa-maxpairs.c:443 returns haserr ? -1 : 0).  A non-zero return
 * from the interval callback stops the enumeration and is propagated as -1
 * (src/match/esa-bottomup.c:147-157).  Input pointers are borrowed for the
 * duration of the call only; every device and pinned buffer is owned by this
 * layer (cached across calls, see gt_smax_release_cache).
 */
#ifndef GT_SMAX_HIP_H
#define GT_SMAX_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  uint64_t position, value;
} GtSmaxLlv;

typedef struct {
  const uint8_t *lcptab;     /* .lcp, totallength+1 bytes, 255 = overflow  */
  const GtSmaxLlv *llvtab;   /* .llv, sorted by position                   */
  uint64_t numllv;
  const uint8_t *bwttab;     /* .bwt, totallength+1 bytes                  */
  const void *suftab;        /* .suf (optional for enumeration)            */
  int suftab_bytes;          /* 4, 8, or 0 when suftab is NULL             */
  uint64_t totallength;      /* n  (.prj totallength)                      */
  uint64_t nonspecials;      /* N = n - specialcharacters                  */
} GtSmaxInput;

/* visit_lcp_interval analogue: one supermaximal-repeat interval
 * [lb..rb] of lcp-value lcp (occurrences are suftab[lb..rb]). */
typedef int (*GtSmaxIntervalFunc)(void *data, uint64_t lcp, uint64_t lb,
                                  uint64_t rb);

/* Device output record: interval [lb .. lb+width-1] with lcp-value lcp.
 *
 * Width limits (the reference carries GtUword lcp values,
 * src/match/lcpoverflow.h:26-30, src/match/esa_visitor_rep.h:46-51): an
 * lcp-value must be below 2^32 and one shard may hold at most 2^32 - 1 .llv
 * entries.  Tables beyond either are REFUSED, never truncated: the plan and
 * the host-table entry points return -1 with "lcp value >= 2^32 in .llv" or
 * "more than 2^32 .llv entries in one shard" (tests/test_smax_gpu.py::
 * test_width_limits_are_refused).  A longest repeat of 4 Gbp would need a
 * multi-Gbp duplication inside one genome; more .llv entries per shard than
 * 2^32 are split by a larger num_gpus (shards) first. */
typedef struct {
  uint64_t lb;
  uint32_t lcp;
  uint32_t width;
} GtSmaxRecord;

int gt_smax_hip_enumerate(const GtSmaxInput *in, unsigned int minlen,
                          int num_gpus, GtSmaxIntervalFunc cb, void *data,
                          char *errbuf, size_t errlen);

/* *lcp_lb_rb receives 3*count uint64 (lcp,lb,rb triples, ascending lb),
 * allocated with malloc; free with gt_smax_free. */
int gt_smax_hip_enumerate_to_buffer(const GtSmaxInput *in,
                                    unsigned int minlen, int num_gpus,
                                    uint64_t **lcp_lb_rb, uint64_t *count,
                                    char *errbuf, size_t errlen);

void gt_smax_free(void *ptr);

/* The host-table entry points keep device memory (a per-device cache of
 * table and plan buffers) and pinned staging buffers for the process, so a
 * second call does not pay multi-GB allocations again; this returns all of
 * it (GT_SMAX_NO_CACHE=1 in the environment frees before every return).
 * num_gpus > 1 splits the suffix rows into num_gpus shards over the visible
 * devices, the calling thread's current device first and then the next ones
 * (contiguous blocks of shards per device, one host thread each; the
 * caller's current device is current again on return);
 * the shards' boundary records are exchanged with one RCCL all-gather over
 * those devices (communicators created by the library and cached), or by
 * device-to-device copies when one device holds all shards. */
void gt_smax_release_cache(void);

/* Warm-up for the first host-table call of a process, asynchronous: returns
 * at once and, on a helper thread, initialises the HIP runtime, creates the
 * device contexts and pinned staging ring of the devices a call with
 * num_gpus would use, starts the staging workers, loads the scan kernels and
 * puts the device buffers of an index with this totallength / nonspecials
 * into the cache.  The next host-table call (or gt_smax_release_cache)
 * waits for it to finish.  A `gt repfind -smax` runner issues it as soon as
 * it has read the index's .prj (src/match/esa-map.c:331-342: the sizes are known
 * before the tables are mapped), so the warm-up overlaps reading the
 * .lcp/.llv/.bwt files.  Returns 0, or -1 when no thread can be started.
 * Optional: without it the first call does the same work itself. */
int gt_smax_hip_prepare(uint64_t totallength, uint64_t nonspecials, int num_gpus);

/* Number of HIP devices visible (0 if the runtime has none). */
int gt_smax_device_count(void);

/* Identity of the scan kernels' build: a hash of the K1..K3 sources and the
 * gfx950 compile flags (set by the Makefile).  Profiles of the kernels
 * (profiles/pmc_*.json) carry it, so a measurement can be matched to the
 * code object it was taken on.  Static string. */
const char *gt_smax_build_id(void);

/* -------------------------------------------------- device-resident API */

/*
 * A shard owns the suffix-array rows whose plateau starts c = lb+1 lie in
 * [begin, end) of [1, nonspecials).  Its device tables cover global indices
 * [base, base+local_len): lcp_dev[i] is LCP[base+i], bwt_dev[i] is
 * BWT[base+i], with base <= begin-1 and base+local_len > end (the shard needs
 * LCP[begin-1 .. end] and BWT[begin-1 .. end-1]).  Both device buffers must
 * be readable GT_SMAX_PAD_FRONT bytes before and GT_SMAX_PAD_BACK bytes after
 * their local_len bytes (use gt_smax_dev_alloc_table).  llv_dev holds the
 * .llv entries with base <= position < base+local_len (global positions).
 */
#define GT_SMAX_PAD_FRONT 256
#define GT_SMAX_PAD_BACK 32768

/*
 * Packed BWT (DNA alphabets: symbols 0..3 plus the specials >= 254), the
 * form the scan streams: 0.5 B per row instead of the .bwt file's 1 B.
 * u64 group gi (0 <= gi < GT_SMAX_PK_GROUPS(local_len)) holds local rows
 * r = 16*(gi-1) + q, q = 0..15: bit q = bit 0 and bit 16+q = bit 1 of the
 * row's symbol, bit 32+q = the row holds a special symbol (>= 254: WILDCARD,
 * SEPARATOR or the undefined BWT character; its code bits are 0); rows
 * outside [0, local_len) are all-zero.  Group 0 is the front halo.
 * Producers: the GPU ESA builder (gt_smax_esa_build), gt_smax_pack_bwt on the
 * host (the host-table entry points pack while staging), or the plan itself
 * from bwt_dev (a plan-time pass over the byte table).  Specials are unique
 * for left diversity, so the packed form loses nothing the smax predicate
 * reads (src/match/esa-maxpairs.c:24-31).
 */
#define GT_SMAX_PK_GROUPS(local_len) ((local_len) / 16 + 134)

typedef struct {
  const uint8_t *lcp_dev;
  const uint8_t *bwt_dev;    /* byte BWT, or NULL when bwtpk_dev is given  */
  const GtSmaxLlv *llv_dev;
  uint64_t numllv;
  uint64_t base, local_len;
  uint64_t begin, end;
  uint64_t nonspecials;      /* global N: LCP[0] = LCP[N] = 0 */
  int device;                /* HIP device ordinal */
  /* packed BWT (GT_SMAX_PK_GROUPS(local_len) u64, 16-byte aligned), or NULL:
   * the plan then packs bwt_dev itself when its alphabet is DNA */
  const uint64_t *bwtpk_dev;
} GtSmaxDevShard;

/* Host packing of a DNA BWT: writes GT_SMAX_PK_GROUPS(len) groups of
 * bwt[0 .. len) to pk.  Returns 0, or 1 (pk incomplete) when a symbol in
 * [4, 254) shows that the alphabet is not DNA. */
int gt_smax_pack_bwt(const uint8_t *bwt, uint64_t len, uint64_t *pk);

/* Diversity of a run of BWT rows: set of symbols < 254 seen, dup flag. */
typedef struct {
  uint64_t seen[4];
  uint64_t dup;
} GtSmaxDiv;

/* Fixed-size boundary record exchanged by the all-gather. */
typedef struct {
  /* tail: plateau owned by this shard that runs into the next shard */
  uint64_t pend_valid, pend_c, pend_lcp;
  GtSmaxDiv pend_div;
  /* head: the run of LCP == LCP[begin] at the start of this shard */
  uint64_t head_v;           /* exact LCP[begin]                         */
  uint64_t head_f;           /* first t>begin... with LCP[t] != head_v,   */
                             /* or UINT64_MAX if the run covers the shard */
  uint64_t head_next;        /* exact LCP[head_f]                         */
  GtSmaxDiv head_div;        /* diversity of BWT[begin .. head_f-1]       */
  uint64_t shard_begin, shard_end;
} GtSmaxBoundary;

typedef struct GtSmaxPlan GtSmaxPlan;

/* Allocate a device table of len bytes with the required padding; returns
 * the usable pointer (free with gt_smax_dev_free_table). */
int gt_smax_dev_alloc_table(int device, uint64_t len, uint8_t **table,
                            char *errbuf, size_t errlen);
int gt_smax_dev_free_table(int device, uint8_t *table);

/* Creates a plan for one shard: output capacity (records), look-back state
 * and the per-tile .llv index.  capacity==0 picks a default. */
int gt_smax_plan_create(GtSmaxPlan **plan, const GtSmaxDevShard *shard,
                        unsigned int minlen, uint64_t capacity,
                        char *errbuf, size_t errlen);
/* Frees the plan; its device buffers return to the runtime's cache only
 * after the device has finished the work already enqueued (safe right after
 * an asynchronous gt_smax_plan_run).  Nothing here waits: the fence is made
 * of events recorded here on the streams the plan's work was enqueued on,
 * so every stream passed to the plan (run, run_part, stitch,
 * copy_boundary) must stay alive until gt_smax_plan_delete -- a per-run
 * event would cost every pass an event packet.  (The F2 / F3 plans record
 * theirs when they enqueue: their callers' streams may go first.) */
void gt_smax_plan_delete(GtSmaxPlan *plan);

/* Enqueue one smax pass (scan + ordered compaction + boundary record) on
 * stream (a hipStream_t, NULL = default stream).  Asynchronous. */
int gt_smax_plan_run(GtSmaxPlan *plan, void *stream);

/* The same pass in two parts (plan_run == part 0 then part 1 on one stream):
 * part 0 = the scan, after which the shard's boundary record is final
 * (gt_smax_plan_copy_boundary may follow); part 1 = the ordered compaction
 * into the record array.  A sharded caller enqueues part 0, the boundary
 * copy and its all-gather (on the collective's stream), then part 1 beside
 * the all-gather, and the stitch once both are done.  -1 for another part.
 * Order: part 1 must follow every part 0 before the next part 0 (its
 * compaction resets the deferral state the next scan starts from); a second
 * part 0, or a part 1 with no part 0 pending, returns -1 and enqueues
 * nothing.  gt_smax_plan_run is refused likewise while a part 1 is pending. */
int gt_smax_plan_run_part(GtSmaxPlan *plan, int part, void *stream);

/* Device pointers owned by the plan. */
GtSmaxRecord *gt_smax_plan_records(GtSmaxPlan *plan);
uint64_t *gt_smax_plan_count_dev(GtSmaxPlan *plan);   /* 1 x uint64 */
GtSmaxBoundary *gt_smax_plan_boundary_dev(GtSmaxPlan *plan);
uint64_t gt_smax_plan_capacity(GtSmaxPlan *plan);
uint64_t gt_smax_plan_num_tiles(GtSmaxPlan *plan);

/* After all shards' boundary records are gathered (in rank order) into
 * all_dev (nshards records, device memory), append this shard's stitched
 * interval, if any, to its records.  Asynchronous on stream. */
int gt_smax_plan_stitch(GtSmaxPlan *plan, const GtSmaxBoundary *all_dev,
                        int nshards, int shard_index, void *stream);

/* Pure host form of the stitch: resolves the pending plateau of shard
 * shard_index against the following heads.  Returns 1 and fills *rec if an
 * interval results, 0 otherwise. */
int gt_smax_stitch_host(const GtSmaxBoundary *all, int nshards,
                        int shard_index, unsigned int minlen,
                        GtSmaxRecord *rec);

/* K1 timing: record hipEvents around the scan kernel of the next runs into
 * nslots ring slots (0 disables); read sums the elapsed time of the slots
 * filled so far (synchronising on them). */
int gt_smax_plan_timing(GtSmaxPlan *plan, int nslots);
int gt_smax_plan_timing_read(GtSmaxPlan *plan, double *sum_ms, int *nread);
/* Events on every stride-th run only (default 1; resets the run count): each
 * timed run pays the two event records (~1 % of a C3 step, ~3 % of an
 * 8-way shard's). */
int gt_smax_plan_timing_stride(GtSmaxPlan *plan, int stride);

/* Copies this shard's boundary record to dst_dev (device memory) on stream,
 * e.g. into the send buffer of an all-gather. */
int gt_smax_plan_copy_boundary(GtSmaxPlan *plan, void *dst_dev, void *stream);

/* Synchronises the plan's device and copies the record count to the host;
 * -1 if the kernels flagged an inconsistent index (see error bits). */
int gt_smax_plan_fetch_count(GtSmaxPlan *plan, uint64_t *count);

/* Synchronises and copies the plan's records (after run / stitch) to host
 * memory as (lcp, lb, rb) triples, ascending lb: 3*capacity uint64 at
 * lcp_lb_rb.  *count receives the record count; -1 when it exceeds the
 * plan's or the caller's capacity (nothing copied), or on a device error. */
int gt_smax_plan_fetch_triples(GtSmaxPlan *plan, uint64_t *lcp_lb_rb,
                               uint64_t capacity, uint64_t *count);

/* Sticky device error bits: 1 = an .lcp byte 255 without its .llv entry,
 * 2 = a table read outside the shard's rows. */
uint32_t gt_smax_plan_error_bits(GtSmaxPlan *plan);

/* Diagnostic: with GT_SMAX_STAMPS set when the plan was created, K1 runs its
 * diagnostic build and sums s_memtime cycles per section over all waves:
 * out8 = {window wait, flush + next DMA issue, segment filter,
 * classification + exact queue, exact starts, record output, staging, tiles}
 * accumulated over the plan's runs.  -1 for a plan without stamps. */
int gt_smax_plan_stamps(GtSmaxPlan *plan, unsigned long long *out8);

/* Name of the K1 variant the plan's runs launch (smax_scan_kernel,
 * _b2 = 2-plane BWT window stream, _dense = vectorised 255-after-255
 * relations, _nt = non-temporal window loads, _diag = GT_SMAX_DEBUG,
 * _bytes = byte BWT windows); a static string. */
const char *gt_smax_plan_scan_kernel(const GtSmaxPlan *plan);

/* Waves per workgroup of the plan's K1b launch (4, or 8 when the launch
 * fits one generation of the 8-wave kernel; GT_SMAX_K1B_WAVES overrides). */
uint32_t gt_smax_plan_k1b_waves(const GtSmaxPlan *plan);

/* Diagnostic: tiles the last run handed from K1 to the generic kernel K1b
 * (shard edges and tiles with more exact-evaluation starts than K1 queues). */
uint32_t gt_smax_plan_deferred_tiles(GtSmaxPlan *plan);

/* Diagnostic: copies the last run's per-tile record counts (num_tiles
 * entries; with GT_SMAX_DEBUG bit 32768 the deferred tiles hold K1b cycle
 * stamps instead) and the deferred-tile list (capacity num_tiles) to host
 * buffers (either may be NULL).  0 on success, -1 on a HIP error. */
int gt_smax_plan_debug_tiles(GtSmaxPlan *plan, uint32_t *counts, uint32_t *deferred,
                             uint32_t *ndeferred);

/* Diagnostic: copies the plan's per-tile .llv window words -- the plan-time
 * index K1 reads, num_tiles pairs {first entry of the window, entries |
 * left-halo entries << 12 | DMA lanes << 17 | static-K1b flag << 31} -- to a
 * host buffer of 2 * num_tiles words.  0 on success, -1 on a HIP error. */
int gt_smax_plan_debug_windows(GtSmaxPlan *plan, uint32_t *words);

#ifdef __cplusplus
}
#endif

#endif
