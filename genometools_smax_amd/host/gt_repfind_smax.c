/*
 * gt_repfind_smax.c -- C host for the smax tool path: `gt repfind -smax`.
 *
 * Mirrors the reference tool's option surface and runner
 * (src/tools/gt_repfind.c:404-483 options, :498-623 runner) for the new
 * -smax branch:
 *   -smax      compute supermaximal repeats (this path; required here)
 *   -l N       minimum length (default 20, minimum 1, gt_repfind.c:415-418)
 *   -ii IDX    index name (mandatory)
 *   -scan      read the tables instead of mapping them (4-byte .suf allowed)
 *   -v         verbose: "# "-prefixed progress lines (logger, :469-473)
 *   -gpus N    number of GPUs / suffix-array shards (default 1)
 *   -intervals print "lcp lb rb" interval rows instead of pair lines
 * -smax excludes -r, -q, -spm, -samples, -extend as gt_option_exclude would.
 * Without -smax the tool computes maximal pairs (the reference's default -f
 * branch, gt_callenummaxpairs, src/tools/gt_repfind.c:553-562) on the GPU
 * (gt_maxpairs_hip_enumerate); -r, -q, -spm, -samples
 * and -extend are not part of this build.
 * Output: one line per occurrence pair of every supermaximal repeat (or per
 * maximal pair), in the format of gt_simpleexactselfmatchoutput
 * (src/tools/gt_repfind.c:49-84, src/match/querymatch.c:130-190):
 * "len seqnum1 relpos1 F len seqnum2 relpos2", formatted on the GPU
 * (gt_repfind_smax_lines / gt_repfind_maxpairs_lines, §8(f) F4) unless
 * -hostformat asks for the host printf path.  Maximal pairs come in the
 * reference's traversal order (the same lines in the same order).
 * Errors: "gt repfind: error: <msg>" on stderr, exit status 1 (gt_tool_run).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "esa_reader.h"
#include "gt_maxpairs_hip.h"
#include "gt_smax_hip.h"

typedef struct {
  const SmaxEsa *esa;
  const uint64_t *sep;
  uint64_t nsep;
  int intervals_only;
  uint64_t *occ;
  uint64_t occcap;
  uint64_t nintervals, npairs;
} OutState;

static uint64_t seqnum_of(const OutState *st, uint64_t p)
{
  uint64_t lo = 0, hi = st->nsep;
  while (lo < hi) {
    uint64_t mid = (lo + hi) / 2;
    if (st->sep[mid] < p) lo = mid + 1; else hi = mid;
  }
  return lo;
}

/* one pair line (gt_simpleexactselfmatchoutput: pos1 < pos2 after ordering,
 * filtered when both are in one sequence and relpos1 > relpos2) */
static void emit_pair(OutState *st, uint64_t len, uint64_t p1, uint64_t p2)
{
  uint64_t s1, s2, st1, st2;
  if (p1 > p2) { uint64_t t = p1; p1 = p2; p2 = t; }
  s1 = seqnum_of(st, p1);
  s2 = seqnum_of(st, p2);
  st1 = s1 == 0 ? 0 : st->sep[s1 - 1] + 1;
  st2 = s2 == 0 ? 0 : st->sep[s2 - 1] + 1;
  if (s1 == s2 && p1 - st1 > p2 - st2) return;
  printf("%llu %llu %llu F %llu %llu %llu\n", (unsigned long long) len,
         (unsigned long long) s1, (unsigned long long) (p1 - st1),
         (unsigned long long) len, (unsigned long long) s2,
         (unsigned long long) (p2 - st2));
  st->npairs++;
}

/* GtMaxpairsFunc (GtProcessmaxpairs analogue) */
static int emit_maxpair(void *data, uint64_t len, uint64_t pos1, uint64_t pos2)
{
  emit_pair((OutState *) data, len, pos1, pos2);
  return 0;
}

/* GtRepfindTextFunc: GPU-formatted lines (F4) to stdout */
static int write_lines(void *data, const char *text, uint64_t bytes)
{
  OutState *st = data;
  uint64_t k;
  if (fwrite(text, 1, bytes, stdout) != bytes) return -1;
  for (k = 0; k < bytes; k++) st->npairs += text[k] == '\n';
  return 0;
}

/* -smax lines: intervals from the GPU, their occurrence positions gathered
 * from the suffix array here, all pairs formatted on the GPU */
static int smax_lines(OutState *st, const GtSmaxInput *in, unsigned int minlen, int gpus,
                      char *errbuf, size_t errlen)
{
  uint64_t *trip = NULL, cnt = 0, nocc = 0, r, k;
  GtSmaxRecord *rec = NULL;
  uint64_t *occ = NULL;
  int rc = -1;
  if (gt_smax_hip_enumerate_to_buffer(in, minlen, gpus, &trip, &cnt, errbuf, errlen) != 0)
    return -1;
  st->nintervals = cnt;
  for (r = 0; r < cnt; r++) nocc += trip[3 * r + 2] - trip[3 * r + 1] + 1;
  rec = malloc(sizeof *rec * (cnt ? cnt : 1));
  occ = malloc(sizeof *occ * (nocc ? nocc : 1));
  if (rec == NULL || occ == NULL) {
    snprintf(errbuf, errlen, "out of memory (%llu occurrences)", (unsigned long long) nocc);
    goto done;
  }
  for (r = 0, nocc = 0; r < cnt; r++) {
    const uint64_t lb = trip[3 * r + 1], rb = trip[3 * r + 2];
    rec[r].lb = nocc;
    rec[r].lcp = (uint32_t) trip[3 * r];
    rec[r].width = (uint32_t) (rb - lb + 1);
    for (k = lb; k <= rb; k++) occ[nocc++] = smax_esa_suffix(st->esa, k);
  }
  rc = gt_repfind_smax_lines(rec, cnt, occ, nocc, st->sep, st->nsep, write_lines, st, errbuf,
                             errlen);
done:
  free(rec);
  free(occ);
  gt_smax_free(trip);
  return rc;
}

/* GtSmaxIntervalFunc: emits the pair lines of one interval (host format) */
static int emit_interval(void *data, uint64_t lcp, uint64_t lb, uint64_t rb)
{
  OutState *st = data;
  uint64_t w = rb - lb + 1, a, b;
  st->nintervals++;
  if (st->intervals_only) {
    printf("%llu %llu %llu\n", (unsigned long long) lcp, (unsigned long long) lb,
           (unsigned long long) rb);
    return 0;
  }
  if (w > st->occcap) {
    uint64_t *p = realloc(st->occ, sizeof (uint64_t) * w);
    if (p == NULL) return -1;
    st->occ = p;
    st->occcap = w;
  }
  for (a = 0; a < w; a++) st->occ[a] = smax_esa_suffix(st->esa, lb + a);
  for (a = 0; a < w; a++)
    for (b = a + 1; b < w; b++) emit_pair(st, lcp, st->occ[a], st->occ[b]);
  return 0;
}

static void usage(FILE *fp)
{
  fprintf(fp, "Usage: gt repfind [options] -ii indexname\n"
              "Compute maximal pairs (default) or supermaximal repeats (-smax).\n\n"
              "-f         compute maximal forward repeats (default)\n"
              "-smax      compute supermaximal repeats (MI355X)\n"
              "-l         Specify minimum length of repeats\n"
              "           default: 20\n"
              "-scan      scan index rather than mapping it to main memory\n"
              "-ii        Specify input index\n"
              "-v         be verbose\n"
              "-gpus      number of GPUs (suffix-array shards)\n"
              "-intervals print lcp-intervals \"lcp lb rb\" instead of pairs\n"
              "-hostformat format the pair lines on the host (default: on the GPU)\n"
              "-help      display help and exit\n");
}

static int fail(const char *msg)
{
  fprintf(stderr, "gt repfind: error: %s\n", msg);
  return 1;
}

static double now_s(void)
{
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int main(int argc, char **argv)
{
  const char *indexname = NULL;
  long minlen = 20;
  int smax = 0, scan = 0, verbose = 0, gpus = 1, intervals = 0, hostformat = 0, i;
  const char *excluded = NULL;
  char errbuf[1024], msg[1200];
  SmaxEsa esa;
  GtSmaxInput in;
  OutState st;
  double t0, t1;
  static char outbuf[1 << 20];

  for (i = 1; i < argc; i++) {
    const char *a = argv[i];
    if (strcmp(a, "-smax") == 0) smax = 1;
    else if (strcmp(a, "-scan") == 0) scan = 1;
    else if (strcmp(a, "-v") == 0) verbose = 1;
    else if (strcmp(a, "-intervals") == 0) intervals = 1;
    else if (strcmp(a, "-hostformat") == 0) hostformat = 1;
    else if (strcmp(a, "-help") == 0) { usage(stdout); return 0; }
    else if (strcmp(a, "-l") == 0 || strcmp(a, "-ii") == 0 || strcmp(a, "-gpus") == 0) {
      char *end = NULL;
      if (i + 1 >= argc) {
        snprintf(msg, sizeof msg, "missing argument to option \"%s\"", a);
        return fail(msg);
      }
      if (strcmp(a, "-ii") == 0) { indexname = argv[++i]; continue; }
      {
        long v = strtol(argv[++i], &end, 10);
        if (end == argv[i] || *end != '\0') {
          snprintf(msg, sizeof msg, "argument to option \"%s\" must be an integer", a);
          return fail(msg);
        }
        if (strcmp(a, "-l") == 0) {
          if (v < 1) return fail("argument to option \"-l\" must be an integer >= 1");
          minlen = v;
        } else {
          if (v < 1) return fail("argument to option \"-gpus\" must be an integer >= 1");
          gpus = (int) v;
        }
      }
    } else if (strcmp(a, "-r") == 0 || strcmp(a, "-q") == 0 ||
               strcmp(a, "-spm") == 0 || strcmp(a, "-samples") == 0 ||
               strcmp(a, "-extend") == 0 || strcmp(a, "-f") == 0) {
      if (strcmp(a, "-f") != 0) excluded = a;
      if ((strcmp(a, "-q") == 0 || strcmp(a, "-samples") == 0) && i + 1 < argc) i++;
    } else {
      snprintf(msg, sizeof msg, "unknown option: %s (-help shows a list of possible options)", a);
      return fail(msg);
    }
  }
  if (excluded != NULL) {
    if (smax)
      snprintf(msg, sizeof msg, "option \"-smax\" and option \"%s\" exclude each other", excluded);
    else
      snprintf(msg, sizeof msg, "option \"%s\" is not part of this build (maximal pairs -f "
               "and supermaximal repeats -smax only)", excluded);
    return fail(msg);
  }
  if (!smax && intervals) return fail("option \"-intervals\" requires option \"-smax\"");
  if (!smax && gpus > 1) return fail("option \"-gpus\" > 1 requires option \"-smax\"");
  if (indexname == NULL) return fail("option \"-ii\" is mandatory");

  setvbuf(stdout, outbuf, _IOFBF, sizeof outbuf);
  t0 = now_s();
  if (smax) {
    /* the device warm-up from the .prj sizes, beside the table reads and
     * the separator scan below (gt_smax_hip_prepare) */
    uint64_t pn = 0, pN = 0;
    if (smax_esa_sizes(indexname, &pn, &pN, errbuf, sizeof errbuf) == 0)
      (void) gt_smax_hip_prepare(pn, pN, gpus);
  }
  if (smax_esa_open(&esa, indexname, !intervals || !smax, scan, errbuf, sizeof errbuf) != 0)
    return fail(errbuf);
  smax_esa_input(&esa, &in);
  memset(&st, 0, sizeof st);
  st.esa = &esa;
  st.intervals_only = intervals;
  if (!intervals && smax_esa_separators(&esa, (uint64_t **) &st.sep, &st.nsep) != 0) {
    smax_esa_close(&esa);
    return fail("out of memory");
  }
  if (verbose) {
    printf("# totallength=%llu nonspecials=%llu largelcpvalues=%llu gpus=%d\n",
           (unsigned long long) esa.totallength, (unsigned long long) esa.nonspecials,
           (unsigned long long) esa.numllv, gpus);
  }
  if (intervals || hostformat
        ? (smax ? gt_smax_hip_enumerate(&in, (unsigned int) minlen, gpus, emit_interval, &st,
                                        errbuf, sizeof errbuf)
                : gt_maxpairs_hip_enumerate(&in, (unsigned int) minlen, emit_maxpair, &st,
                                            errbuf, sizeof errbuf)) != 0
        : (smax ? smax_lines(&st, &in, (unsigned int) minlen, gpus, errbuf, sizeof errbuf)
                : gt_repfind_maxpairs_lines(&in, (unsigned int) minlen, st.sep, st.nsep,
                                            write_lines, &st, errbuf, sizeof errbuf)) != 0) {
    fflush(stdout);
    free((void *) st.sep);
    free(st.occ);
    smax_esa_close(&esa);
    return fail(errbuf);
  }
  t1 = now_s();
  if (verbose && smax)
    printf("# smax intervals=%llu pairs=%llu time=%.3fs\n",
           (unsigned long long) st.nintervals, (unsigned long long) st.npairs, t1 - t0);
  else if (verbose)
    printf("# maximal pairs=%llu time=%.3fs\n", (unsigned long long) st.npairs, t1 - t0);
  fflush(stdout);
  free((void *) st.sep);
  free(st.occ);
  smax_esa_close(&esa);
  return 0;
}
