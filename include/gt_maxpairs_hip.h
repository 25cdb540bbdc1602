/*
 * gt_maxpairs_hip.h -- C-ABI of the MI355X maximal-pairs layer
 * (`gt repfind -l N` without -smax) and of the
 * on-device position formatting (§8(f) F4).
 *
 * Same conventions as gt_smax_hip.h: plain C types, 0 = success, -1 = error
 * with the message in errbuf, input pointers borrowed for the call only, a
 * non-zero callback return stops the enumeration and yields -1.
 *
 *  gt_maxpairs_hip_enumerate      replaces gt_enumeratemaxpairs /
 *                                 gt_callenummaxpairs
 *                                   src/match/esa-maxpairs.h:45-63,
 *                                   src/match/esa-maxpairs.c:476-520
 *                                 i.e. the bottom-up traversal
 *                                   src/match/esa-bottomup-maxpairs.inc:136-264
 *                                 with the leaf/branching-edge cartesian
 *                                 products of src/match/esa-maxpairs.c:181-360.
 *                                 The callback has the argument meaning of
 *                                 GtProcessmaxpairs (src/match/esa-maxpairs.h:38-43):
 *                                 (len, pos1, pos2).  Pairs, their order AND
 *                                 the order of pos1/pos2 in each call are
 *                                 the reference's: the callback sees exactly
 *                                 the calls the traversal makes (a leaf edge
 *                                 passes the new leaf first, a branching
 *                                 edge the father's position first,
 *                                 src/match/esa-maxpairs.c:127-157,259-261,
 *                                 349-351); gt_simpleexactselfmatchoutput
 *                                 swaps them into pos1 < pos2 itself
 *                                 (src/tools/gt_repfind.c:60-65).
 *  gt_maxpairs_hip_enumerate_to_buffer  same, malloc'd (len,pos1,pos2) triples.
 *
 * A maximal pair of length L >= minlen is a pair of suffix-array rows
 * i < j with L = min LCP[i+1..j] (the depth of their lowest common
 * lcp-interval, so the two suffixes branch right after L symbols) whose
 * left contexts differ: not (BWT[i] == BWT[j] < 254).  BWT >= 254 (wildcard,
 * separator, or the undefined left context of position 0, the reference's
 * INITIALCHAR) is unique, as in ISLEFTDIVERSE (src/match/esa-maxpairs.c:24-31).
 */
#ifndef GT_MAXPAIRS_HIP_H
#define GT_MAXPAIRS_HIP_H

#include <stddef.h>
#include <stdint.h>

#include "gt_smax_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* GtProcessmaxpairs analogue (without the encseq / GtError arguments). */
typedef int (*GtMaxpairsFunc)(void *data, uint64_t len, uint64_t pos1, uint64_t pos2);

/* in->suftab is required (4 or 8 bytes per entry).  The host-table entry
 * points run on the calling thread's current HIP device and leave it
 * current; the tables are staged through the library's pinned ring into its
 * caching allocator (released by gt_smax_release_cache). */
int gt_maxpairs_hip_enumerate(const GtSmaxInput *in, unsigned int minlen,
                              GtMaxpairsFunc cb, void *data,
                              char *errbuf, size_t errlen);

/* *len_pos1_pos2 receives 3*count uint64 (malloc'd; free with gt_smax_free). */
int gt_maxpairs_hip_enumerate_to_buffer(const GtSmaxInput *in, unsigned int minlen,
                                        uint64_t **len_pos1_pos2, uint64_t *count,
                                        char *errbuf, size_t errlen);

/* -------------------------------------------------- device-resident API */

/* Tables in HBM, global rows 0..N (lcp_dev/bwt_dev as for GtSmaxDevShard
 * with base 0; suftab entries of suf_bytes = 4 or 8 bytes). */
typedef struct {
  const uint8_t *lcp_dev;
  const uint8_t *bwt_dev;
  const GtSmaxLlv *llv_dev;
  uint64_t numllv;
  const void *suf_dev;
  int suf_bytes;
  uint64_t nonspecials;      /* N */
  int device;
} GtMaxpairsDevInput;

typedef struct GtMaxpairsPlan GtMaxpairsPlan;

/* Expands the exact LCP values (u32 per row, .llv applied) once. */
int gt_maxpairs_plan_create(GtMaxpairsPlan **plan, const GtMaxpairsDevInput *in,
                            unsigned int minlen, char *errbuf, size_t errlen);
/* The same on stream (a hipStream_t, NULL = default stream): waits on that
 * stream only, for the candidate count that sizes the lists.  Every plan
 * call orders itself after the plan's earlier work on other streams (events
 * recorded at enqueue time); none synchronises the device. */
int gt_maxpairs_plan_create_stream(GtMaxpairsPlan **plan, const GtMaxpairsDevInput *in,
                                   unsigned int minlen, void *stream, char *errbuf,
                                   size_t errlen);
/* Frees the plan; its device buffers return to the runtime's cache behind
 * the plan's enqueued work (nothing waits; the caller's streams may already
 * be destroyed). */
void gt_maxpairs_plan_delete(GtMaxpairsPlan *plan);

/* Enqueue the counting pass (pairs per row + exclusive scan) on stream. */
int gt_maxpairs_plan_count(GtMaxpairsPlan *plan, void *stream);

/* Waits for the plan's own work (not the device) and returns the number of
 * pairs of the last count pass. */
int gt_maxpairs_plan_total(GtMaxpairsPlan *plan, uint64_t *total);

/* Candidate rows of the plan (rows j >= 1 with LCP[j] >= minlen: the rows
 * whose walk is not empty -- the rows the reference's traversal pushes into
 * an lcp-interval of depth >= minlen, src/match/esa-bottomup-maxpairs.inc:
 * 155-243); fixed at plan creation (the tables are immutable). */
uint64_t gt_maxpairs_plan_candidates(const GtMaxpairsPlan *plan);

/* Enqueue the emission pass: out_dev receives 3*total uint64
 * (len, pos1 < pos2) triples in suffix-array row order (by the later row,
 * then descending earlier row); capacity is in triples (pairs beyond it are
 * dropped).  Requires a preceding count pass. */
int gt_maxpairs_plan_emit(GtMaxpairsPlan *plan, uint64_t *out_dev, uint64_t capacity,
                          void *stream);

/* The emission pass in the reference's order (the order of
 * gt_maxpairs_hip_enumerate's callbacks, with the reference's pos1/pos2
 * argument order): the pairs are written with their event/row sort keys and
 * permuted by stable radix sorts.  Synchronises the
 * stream (the pair count sizes its temporary buffers, ~80 bytes per pair);
 * capacity must be >= the count, else -1.  Requires a preceding count pass. */
int gt_maxpairs_plan_emit_ordered(GtMaxpairsPlan *plan, uint64_t *out_dev, uint64_t capacity,
                                  void *stream);

/* F4: on-device sequence mapping of position pairs, the seqnum/relpos step
 * of gt_querymatch_fill / gt_encseq_seqnum (src/match/querymatch.c:47-67,
 * src/core/encseq.c:3815-3885): for each (len, pos1, pos2) triple with
 * pos1 < pos2, writes (len, seqnum1, relpos1, seqnum2, relpos2) given the
 * sorted separator positions sep_dev[0..nsep).  Asynchronous on stream. */
int gt_seqpos_map_dev(const uint64_t *sep_dev, uint64_t nsep, const uint64_t *pairs_dev,
                      uint64_t count, uint64_t *out_dev, int device, void *stream);

/* F4: gt repfind output lines formatted on the GPU
 * ("len seqnum1 relpos1 F len seqnum2 relpos2\n", gt_simpleexactselfmatchoutput
 * + gt_querymatch_output, src/tools/gt_repfind.c:49-84,
 * src/match/querymatch.c:130-190; pos1/pos2 swapped into ascending order,
 * seqnum/relpos from the sorted separator positions).  The text arrives in
 * chunks (whole lines, <= 2^22 pairs each) through the callback, in pair
 * order; a non-zero return stops and yields -1. */
typedef int (*GtRepfindTextFunc)(void *data, const char *text, uint64_t bytes);

/* device (len, pos1, pos2) triples (e.g. gt_maxpairs_plan_emit_ordered's)
 * and device separators -> lines, on `device` (the caller's current device is
 * restored on return) */
int gt_repfind_pairs_lines_dev(const uint64_t *pairs_dev, uint64_t count, const uint64_t *sep_dev,
                               uint64_t nsep, int device, GtRepfindTextFunc cb, void *data,
                               char *errbuf, size_t errlen);

/* `gt repfind -l N` (maximal pairs) as lines: gt_maxpairs_hip_enumerate's
 * pairs, in its (the reference's) order, formatted without leaving HBM. */
int gt_repfind_maxpairs_lines(const GtSmaxInput *in, unsigned int minlen, const uint64_t *sep,
                              uint64_t nsep, GtRepfindTextFunc cb, void *data, char *errbuf,
                              size_t errlen);

/* `gt repfind -smax` as lines: record r's occurrences are
 * occpos[rec[r].lb .. rec[r].lb + rec[r].width) (text positions in
 * suffix-array row order); every pair a < b of them, a outer, becomes one
 * line of length rec[r].lcp -- the order bin/gt-repfind prints them in.
 * The pairs are generated on the GPU from the records (none stored), on the
 * caller's current HIP device (left current on return). */
int gt_repfind_smax_lines(const GtSmaxRecord *rec, uint64_t nrec, const uint64_t *occpos,
                          uint64_t nocc, const uint64_t *sep, uint64_t nsep,
                          GtRepfindTextFunc cb, void *data, char *errbuf, size_t errlen);

#ifdef __cplusplus
}
#endif

#endif
