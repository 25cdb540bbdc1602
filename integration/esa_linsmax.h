/*
 * esa_linsmax.h -- GenomeTools-side binding of the MI355X smax layer.
 *
 * This file belongs in the reference tree as src/match/esa_linsmax.h (next to
 * esa-maxpairs.h); it is compiled against the reference headers by
 * integration/check_shim.sh.  The two entry points have the signature of
 * gt_callenummaxpairs (src/match/esa-maxpairs.h:57-63, body at
 * src/match/esa-maxpairs.c:476-520) plus the GPU count, so the repfind
 * runner (src/tools/gt_repfind.c:553-562) can call them with its own
 * GtProcessmaxpairs output function (gt_simpleexactselfmatchoutput,
 * src/tools/gt_repfind.c:49-84).
 */
#ifndef ESA_LINSMAX_H
#define ESA_LINSMAX_H

#include <stdbool.h>
#include "core/error_api.h"
#include "core/logger_api.h"
#include "match/esa-maxpairs.h"
#include "match/esa-seqread.h"
#include "match/esa_visitor.h"

/* gt repfind -smax: every occurrence pair of every supermaximal repeat of
   length >= userdefinedleastlength, passed to processmaxpairs in ascending
   lb (interval) and occurrence-row order.  0 on success, -1 with err set. */
int gt_callenumsupermaxrepeats(const char *indexname,
                               unsigned int userdefinedleastlength,
                               bool scanfile,
                               int num_gpus,
                               GtProcessmaxpairs processmaxpairs,
                               void *processmaxpairsinfo,
                               GtLogger *logger,
                               GtError *err);

/* gt repfind -l N (default -f) on the GPU: the maximal pairs of
   gt_callenummaxpairs, same output function. */
int gt_callenummaxpairs_hip(const char *indexname,
                            unsigned int userdefinedleastlength,
                            bool scanfile,
                            GtProcessmaxpairs processmaxpairs,
                            void *processmaxpairsinfo,
                            GtLogger *logger,
                            GtError *err);

/* gt_esa_bottomup (src/match/esa-bottomup.h:31-33) on the GPU: any
   GtESAVisitor -- the reference's own visitors included -- receives its
   leaf-edge, branching-edge and lcp-interval calls with their
   GtESAVisitorInfo objects (created with gt_esa_visitor_info_new, one per
   stack slot, and deleted after the traversal, as esa-bottomup.c:20-110) in
   the reference's order, from the lcp-interval tree built on the GPU
   (gt_esa_bottomup_info_hip).  Needs the mapped .lcp/.llv/.suf tables
   (a reader opened without scanfile).  0 on success, -1 with err set. */
int gt_esa_bottomup_gpu(Sequentialsuffixarrayreader *ssar, GtESAVisitor *ev,
                        GtError *err);

#endif
