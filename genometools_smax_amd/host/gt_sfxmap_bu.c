/*
 * gt_sfxmap_bu.c -- C host for `gt dev sfxmap -enumlcpitvtreeBU -esa IDX`
 * (src/tools/gt_sfxmap.c:295-299, runner src/match/esa-lcpintervals.c:
 * 195-236): the bottom-up lcp-interval tree enumeration over an enhanced
 * suffix array (.prj/.lcp/.llv/.suf; .bwt not needed), with the tree built
 * on the GPU (gt_esa_bottomup_hip).  Prints the lines of
 * the reference's lcpitvs visitor (src/match/esa_lcpintervals_visitor.c:
 * 30-61), in its order:
 *   "L <firstsucc 0|1> <fatherdepth> <fatherlb> <leafnumber>"
 *   "B <firstsucc 0|1> <fatherdepth> <fatherlb> <childdepth> <childlb>"
 * Options: -esa IDX (mandatory), -enumlcpitvtreeBU (required), -scan.
 * Errors: "gt sfxmap: error: <msg>" on stderr, exit status 1.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "esa_reader.h"
#include "gt_lcpitv_hip.h"

static int leaf_edge(void *data, int first, uint64_t fd, uint64_t flb, uint64_t leaf)
{
  (void) data;
  printf("L %c %llu %llu %llu\n", first ? '1' : '0', (unsigned long long) fd,
         (unsigned long long) flb, (unsigned long long) leaf);
  return 0;
}

static int branching_edge(void *data, int first, uint64_t fd, uint64_t flb, uint64_t sd,
                          uint64_t slb, uint64_t srb)
{
  (void) data;
  (void) srb;
  printf("B %c %llu %llu %llu %llu\n", first ? '1' : '0', (unsigned long long) fd,
         (unsigned long long) flb, (unsigned long long) sd, (unsigned long long) slb);
  return 0;
}

static int fail(const char *msg)
{
  fprintf(stderr, "gt sfxmap: error: %s\n", msg);
  return 1;
}

int main(int argc, char **argv)
{
  const char *indexname = NULL;
  int bu = 0, scan = 0, i;
  char errbuf[1024], msg[1200];
  static char outbuf[1 << 20];
  SmaxEsa esa;
  GtSmaxInput in;
  GtLcpitvVisitor v = {leaf_edge, branching_edge, NULL};

  for (i = 1; i < argc; i++) {
    if (strcmp(argv[i], "-enumlcpitvtreeBU") == 0) bu = 1;
    else if (strcmp(argv[i], "-scan") == 0) scan = 1;
    else if (strcmp(argv[i], "-esa") == 0) {
      if (i + 1 >= argc) return fail("missing argument to option \"-esa\"");
      indexname = argv[++i];
    } else if (strcmp(argv[i], "-help") == 0) {
      printf("Usage: gt dev sfxmap -enumlcpitvtreeBU -esa indexname [-scan]\n"
             "enumerate the lcp-interval tree (using a bottom-up strategy, GPU)\n");
      return 0;
    } else {
      snprintf(msg, sizeof msg, "unknown option: %s (-help shows a list of possible options)",
               argv[i]);
      return fail(msg);
    }
  }
  if (!bu) return fail("this build implements -enumlcpitvtreeBU only");
  if (indexname == NULL) return fail("option \"-esa\" is mandatory");
  setvbuf(stdout, outbuf, _IOFBF, sizeof outbuf);
  if (smax_esa_open_tables(&esa, indexname, 1, 0, scan, errbuf, sizeof errbuf) != 0)
    return fail(errbuf);
  smax_esa_input(&esa, &in);
  if (gt_esa_bottomup_hip(&in, &v, NULL, errbuf, sizeof errbuf) != 0) {
    fflush(stdout);
    smax_esa_close(&esa);
    return fail(errbuf);
  }
  fflush(stdout);
  smax_esa_close(&esa);
  return 0;
}
