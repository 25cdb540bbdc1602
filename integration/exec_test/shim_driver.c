/*
 * shim_driver.c -- runs the reference-side binding (integration/esa_linsmax.c)
 * the way the patched repfind runner calls it (integration/gt_repfind_smax.patch,
 * src/tools/gt_repfind.c:553-562), with an output function of the
 * GtProcessmaxpairs type (src/match/esa-maxpairs.h:38-43) that records every
 * (len, pos1, pos2) it receives, in order:
 *
 *   shim_exec INDEX MINLEN smax|maxpairs [-scan] [GPUS]
 *   shim_exec INDEX 0 bottomup
 *
 * prints one "len pos1 pos2" line per call; with bottomup, the reference's
 * gt_esa_bottomup entry point on the GPU (gt_esa_bottomup_gpu) drives a
 * recording GtESAVisitor (gt_stubs.c) -- one line per visitor call with its
 * GtESAVisitorInfo ids, one "D id" line per deleted info; exit 0, or 1 with
 * the GtError message on stderr.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "core/error_api.h"
#include "match/esa-maxpairs.h"
#include "match/esa_linsmax.h"

GtESAVisitor *stub_visitor_new(FILE *out);

struct GtError {
  char msg[4096];
  bool isset;
};

static int record_pair(void *info, const GtGenericEncseq *genericencseq, GtUword len,
                       GtUword pos1, GtUword pos2, GtError *err)
{
  FILE *out = info;
  (void) err;
  if (genericencseq == NULL || !genericencseq->hasencseq ||
      genericencseq->seqptr.encseq == NULL)
    return -1;                      /* the runner's output function needs the encseq */
  fprintf(out, "%lu %lu %lu\n", (unsigned long) len, (unsigned long) pos1,
          (unsigned long) pos2);
  return 0;
}

int main(int argc, char **argv)
{
  struct GtError err;
  bool scan = false, smax;
  int gpus = 1, rc, i;
  if (argc < 4) {
    fprintf(stderr, "usage: %s INDEX MINLEN smax|maxpairs [-scan] [GPUS]\n", argv[0]);
    return 2;
  }
  smax = strcmp(argv[3], "smax") == 0;
  for (i = 4; i < argc; i++) {
    if (strcmp(argv[i], "-scan") == 0) scan = true;
    else gpus = atoi(argv[i]);
  }
  memset(&err, 0, sizeof err);
  if (strcmp(argv[3], "bottomup") == 0) {
    Sequentialsuffixarrayreader *ssar =
      gt_newSequentialsuffixarrayreaderfromfile(argv[1], SARR_LCPTAB | SARR_SUFTAB | SARR_ESQTAB,
                                                false, NULL, &err);
    GtESAVisitor *ev = stub_visitor_new(stdout);
    rc = ssar == NULL ? -1 : gt_esa_bottomup_gpu(ssar, ev, &err);
    if (ssar != NULL) gt_freeSequentialsuffixarrayreader(&ssar);
    free(ev);
    if (rc != 0) {
      fprintf(stderr, "shim error: %s\n", err.isset ? err.msg : "(no message)");
      return 1;
    }
    return 0;
  }
  rc = smax ? gt_callenumsupermaxrepeats(argv[1], (unsigned) atoi(argv[2]), scan, gpus,
                                         record_pair, stdout, NULL, &err)
            : gt_callenummaxpairs_hip(argv[1], (unsigned) atoi(argv[2]), scan,
                                      record_pair, stdout, NULL, &err);
  if (rc != 0) {
    fprintf(stderr, "shim error: %s\n", err.isset ? err.msg : "(no message)");
    return 1;
  }
  return 0;
}
