/*
 * gt_suffixerator_gpu.c -- `gt suffixerator` for the smax path, on the GPU
 * (SURVEY.md §8(f) F1).
 *
 * Mirrors the reference tool's options for the tables this path reads
 * (src/tools/gt_suffixerator.c, src/match/sfx-run.c:213-300):
 *   -db FILE        FASTA input (one file)
 *   -indexname IDX  index name (default: the FASTA file name)
 *   -dna -suf -lcp -bwt   accepted; .suf/.lcp/.llv/.bwt/.prj are always
 *                   written (the smax and maximal-pairs paths need all)
 *   -suftabuint     4-byte .suf (n+1 < 2^32), readable with -scan
 *   -device N       HIP device (default 0)
 *   -v              "# "-prefixed progress lines
 * The suffix array is built by gt_smax_esa64_build (any length, 64-bit
 * suffixes); files by gt_smax_esa64_write.  The encoded-sequence files
 * (.esq/.ssp/.des/.sds) are not written: this path derives sequence
 * boundaries from the .bwt separators.
 * Errors: "gt suffixerator: error: <msg>" on stderr, exit status 1.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "gt_smax_esa.h"

static int fail(const char *msg)
{
  fprintf(stderr, "gt suffixerator: error: %s\n", msg);
  return 1;
}

static double now(void)
{
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

int main(int argc, char **argv)
{
  const char *db = NULL, *indexname = NULL;
  int suftabuint = 0, verbose = 0, device = 0, i;
  char errbuf[1024] = "", msg[1200];
  FILE *fp;
  long long len;
  char *buf;
  uint8_t *text;
  uint64_t n = 0, numseq = 0;
  GtSmaxEsa64Dev esa;
  double t0 = now();
  for (i = 1; i < argc; i++) {
    if (!strcmp(argv[i], "-db") && i + 1 < argc) db = argv[++i];
    else if (!strcmp(argv[i], "-indexname") && i + 1 < argc) indexname = argv[++i];
    else if (!strcmp(argv[i], "-suftabuint")) suftabuint = 1;
    else if (!strcmp(argv[i], "-device") && i + 1 < argc) device = atoi(argv[++i]);
    else if (!strcmp(argv[i], "-v")) verbose = 1;
    else if (!strcmp(argv[i], "-dna") || !strcmp(argv[i], "-suf") || !strcmp(argv[i], "-lcp") ||
             !strcmp(argv[i], "-bwt") || !strcmp(argv[i], "-tis"))
      ;
    else {
      snprintf(msg, sizeof msg, "unknown option \"%s\"", argv[i]);
      return fail(msg);
    }
  }
  if (db == NULL) return fail("option \"-db\" is mandatory");
  if (indexname == NULL) indexname = db;
  fp = fopen(db, "rb");
  if (fp == NULL) {
    snprintf(msg, sizeof msg, "file \"%s\" does not exist", db);
    return fail(msg);
  }
  fseeko(fp, 0, SEEK_END);
  len = (long long) ftello(fp);
  fseeko(fp, 0, SEEK_SET);
  buf = malloc((size_t) len + 1);
  text = malloc((size_t) len + 1);
  if (buf == NULL || text == NULL) return fail("out of memory");
  if (len > 0 && fread(buf, 1, (size_t) len, fp) != (size_t) len) return fail("read error");
  fclose(fp);
  if (gt_smax_encode_fasta(buf, (uint64_t) len, text, &n, &numseq, errbuf, sizeof errbuf)) {
    snprintf(msg, sizeof msg, "%s: %s", db, errbuf);
    return fail(msg);
  }
  free(buf);
  if (verbose) printf("# %s: %llu symbols, %llu sequences (%.2f s)\n", db, (unsigned long long) n,
                      (unsigned long long) numseq, now() - t0);
  if (gt_smax_esa64_build(device, text, n, 0, 0, 1, 0, &esa, errbuf, sizeof errbuf)) return fail(errbuf);
  if (verbose) printf("# suffix array on device %d: %d batches, %d rounds, %llu .llv entries (%.2f s)\n",
                      device, esa.batches, esa.sort_rounds, (unsigned long long) esa.numllv, now() - t0);
  if (gt_smax_esa64_write(&esa, text, n, numseq, db, (uint64_t) len, indexname, suftabuint ? 4 : 8,
                          errbuf, sizeof errbuf)) {
    gt_smax_esa64_release(&esa);
    return fail(errbuf);
  }
  gt_smax_esa64_release(&esa);
  free(text);
  if (verbose) printf("# wrote %s.{suf,lcp,llv,bwt,prj} (%.2f s)\n", indexname, now() - t0);
  return 0;
}
