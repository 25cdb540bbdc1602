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
 *                                 The per-node GtESAVisitorInfo state is not
 *                                 modelled (visitors that need it keep their
 *                                 own, keyed by the father's lb).
 *  gt_lcpitv_hip_enumerate_to_buffer  every lcp-interval of depth > 0 with
 *                                 its father, in bottom-up (pop) order:
 *                                 (lcp, lb, rb, father lcp, father lb).
 *
 * Device form: the tree comes from all-nearest-smaller-value searches over
 * the exact LCP array (a 64-ary min hierarchy), one thread per row; no
 * stack walk.
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

/* in->suftab is required when v->leaf_edge is set (leaf numbers). */
int gt_esa_bottomup_hip(const GtSmaxInput *in, const GtLcpitvVisitor *v, void *data,
                        char *errbuf, size_t errlen);

/* *itv receives 5*count uint64: (lcp, lb, rb, fatherlcp, fatherlb) per
 * lcp-interval of depth > 0, bottom-up order (rb ascending, then lcp
 * descending).  malloc'd; free with gt_smax_free. */
int gt_lcpitv_hip_enumerate_to_buffer(const GtSmaxInput *in, uint64_t **itv, uint64_t *count,
                                      char *errbuf, size_t errlen);

#ifdef __cplusplus
}
#endif

#endif
