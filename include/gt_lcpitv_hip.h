/*
 * gt_lcpitv_hip.h -- C-ABI of the MI355X generic bottom-up lcp-interval
 * traversal: the lcp-interval tree of an enhanced
 * suffix array computed on the GPU, replayed as GtESAVisitor events.
 *
 * Same conventions as gt_smax_hip.h (plain C types, 0 / -1 + errbuf, input
 * pointers borrowed for the call, a non-zero callback return stops the
 * traversal and yields -1, src/match/esa-bottomup.c:147-157).
 *
 *  gt_esa_bottomup_hip            replaces gt_esa_bottomup(ssar, visitor, err)
 *                                   src/match/esa-bottomup.h:31-33,
 *                                   src/match/esa-bottomup.c:116-273
 *                                 with the GtESAVisitor callbacks
 *                                   src/match/esa_visitor_rep.h:25-67
 *                                 (leaf edge, branching edge, lcp-interval;
 *                                 NULL callbacks are skipped as in
 *                                 src/match/esa_visitor.c:90-146).  The event
 *                                 sequence -- order, firstsucc flags, father
 *                                 depth/lb, child depth/lb/rb, leaf numbers
 *                                 -- is the reference traversal's, exactly.
 *  gt_esa_bottomup_info_hip       the same with the per-node GtESAVisitorInfo
 *                                 of every callback (info_new / info_delete
 *                                 per stack slot, as the reference's stack).
 *  gt_lcpitv_hip_enumerate_to_buffer  every lcp-interval of depth > 0 with
 *                                 its father, in bottom-up (pop) order:
 *                                 (lcp, lb, rb, father lcp, father lb).
 *
 * Device form: the tree comes from the strict previous-smaller values of
 * the exact LCP array (ANSV per 2048-row tile in LDS, a 64-ary min
 * hierarchy across tiles): the reference's stack after each row is the
 * previous-smaller chain from it, so the intervals popped there are read
 * off that chain; no stack walk, no sort.  The device-resident API (gt_lcpitv_plan_*) keeps the tree in
 * HBM and writes the whole visitor event stream there, every event at its
 * position in the reference's order; the host entry points above are built
 * on it (events downloaded in chunks, callbacks on the calling thread).
 */
#ifndef GT_LCPITV_HIP_H
#define GT_LCPITV_HIP_H

#include <stddef.h>
#include <stdint.h>

#include "gt_smax_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* GtESAVisitor analogue; any callback may be NULL. */
typedef struct {
  /* visit_leaf_edge(firstsucc, fatherdepth, fatherlb, leafnumber) */
  int (*leaf_edge)(void *data, int firstsucc, uint64_t fd, uint64_t flb, uint64_t leafnumber);
  /* visit_branching_edge(firstsucc, fd, flb, childdepth, childlb, childrb) */
  int (*branching_edge)(void *data, int firstsucc, uint64_t fd, uint64_t flb, uint64_t sd,
                        uint64_t slb, uint64_t srb);
  /* visit_lcp_interval(lcp, lb, rb) */
  int (*lcp_interval)(void *data, uint64_t lcp, uint64_t lb, uint64_t rb);
} GtLcpitvVisitor;

/* in->suftab is required when v->leaf_edge is set (leaf numbers).  Like
 * every host-table entry point here: runs on the calling thread's current
 * HIP device and leaves it current; tables staged through the library's
 * pinned ring into its caching allocator. */
int gt_esa_bottomup_hip(const GtSmaxInput *in, const GtLcpitvVisitor *v, void *data,
                        char *errbuf, size_t errlen);

/* GtESAVisitor with its per-node state (src/match/esa_visitor_rep.h:25-67):
 * every callback also receives the GtESAVisitorInfo of the interval(s) it
 * concerns, created by info_new and released by info_delete exactly as
 * gt_esa_bottomup does (src/match/esa-bottomup.c:20-110,116-273): one info
 * per stack slot, allocated 32 at a time as the stack grows, reused by the
 * intervals that occupy the slot, deleted slot by slot after the traversal;
 * a father pushed right after its first child's pop occupies that child's
 * slot, so its branching edge passes soninfo NULL with fatherinfo == the
 * child's info (the reference's hand-over of the child's state).  The
 * callbacks and their order are gt_esa_bottomup_hip's; info_new is required,
 * the other callbacks may be NULL. */
typedef struct {
  int (*leaf_edge)(void *data, int firstsucc, uint64_t fd, uint64_t flb, void *finfo,
                   uint64_t leafnumber);
  int (*branching_edge)(void *data, int firstsucc, uint64_t fd, uint64_t flb, void *finfo,
                        uint64_t sd, uint64_t slb, uint64_t srb, void *sinfo);
  int (*lcp_interval)(void *data, uint64_t lcp, uint64_t lb, uint64_t rb, void *info);
  void *(*info_new)(void *data);
  void (*info_delete)(void *info, void *data);
} GtLcpitvInfoVisitor;

/* gt_esa_bottomup(ssar, visitor, err) for visitors with per-node state
 * (esa-bottomup.h:31-33 with the GtESAVisitorInfo arguments of
 * esa_visitor.h:30-51). */
int gt_esa_bottomup_info_hip(const GtSmaxInput *in, const GtLcpitvInfoVisitor *v, void *data,
                             char *errbuf, size_t errlen);

/* *itv receives 5*count uint64: (lcp, lb, rb, fatherlcp, fatherlb) per
 * lcp-interval of depth > 0, bottom-up order (rb ascending, then lcp
 * descending).  malloc'd; free with gt_smax_free. */
int gt_lcpitv_hip_enumerate_to_buffer(const GtSmaxInput *in, uint64_t **itv, uint64_t *count,
                                      char *errbuf, size_t errlen);

/* -------------------------------------------------- device-resident API */

/* Tables in HBM, global rows 0..N (as GtMaxpairsDevInput); suf_dev may be
 * NULL (leaf numbers are then written as 0). */
typedef struct {
  const uint8_t *lcp_dev;
  const GtSmaxLlv *llv_dev;
  uint64_t numllv;
  const void *suf_dev;
  int suf_bytes;             /* 4 or 8 */
  uint64_t nonspecials;      /* N */
  int device;
} GtLcpitvDevInput;

typedef struct GtLcpitvPlan GtLcpitvPlan;

/* Builds the lcp-interval tree in HBM (synchronous). */
int gt_lcpitv_plan_create(GtLcpitvPlan **plan, const GtLcpitvDevInput *in, char *errbuf,
                          size_t errlen);
/* The same, enqueued on stream (a hipStream_t, NULL = default stream): it
 * waits on that stream once, for the interval count that sizes the records,
 * and returns with the records still being written there.  Reading them
 * (gt_lcpitv_plan_intervals) on another stream needs that stream ordered
 * after `stream`; gt_lcpitv_plan_events orders itself. */
int gt_lcpitv_plan_create_stream(GtLcpitvPlan **plan, const GtLcpitvDevInput *in, void *stream,
                                 char *errbuf, size_t errlen);
/* Frees the plan; its device buffers return to the runtime's cache behind
 * events recorded where its work was enqueued (nothing waits; the caller's
 * streams may already be destroyed). */
void gt_lcpitv_plan_delete(GtLcpitvPlan *plan);

/* Number of lcp-intervals of depth > 0; *itv_dev = their device records,
 * 5 uint64 each (lcp, lb, rb, fatherlcp, fatherlb), pop order. */
uint64_t gt_lcpitv_plan_intervals(const GtLcpitvPlan *plan, const uint64_t **itv_dev);

/* N + 2 * intervals: one leaf edge per row, an lcp-interval and a
 * branching-edge event per interval. */
uint64_t gt_lcpitv_plan_num_events(const GtLcpitvPlan *plan);

/* Enqueues the event stream of gt_esa_bottomup (7 uint64 per event, in the
 * reference's order) into events_dev (gt_lcpitv_plan_num_events entries;
 * 16-byte aligned, else -1: the records are stored as 16-byte pieces) on
 * stream, after the plan's construction (on whatever stream it ran):
 *   (0, firstsucc, fd, flb, leafnumber, 0, 0)   visit_leaf_edge
 *   (1, firstsucc, fd, flb, sd, slb, srb)       visit_branching_edge
 *   (2, 0, lcp, lb, rb, 0, 0)                   visit_lcp_interval  */
int gt_lcpitv_plan_events(GtLcpitvPlan *plan, uint64_t *events_dev, void *stream);

#ifdef __cplusplus
}
#endif

#endif
