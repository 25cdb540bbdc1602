/*
 * gt_smax_e2e.c -- one-shot timing of the drop-in entry point in a fresh
 * process (bin/gt-smax-e2e), the way `gt repfind -smax` meets it: one
 * process per index (src/tools/gt_repfind.c:553-562), the HIP runtime not
 * yet initialised, nothing cached by the library.
 *
 *   gt-smax-e2e LCP BWT LLV TOTALLENGTH NONSPECIALS MINLEN CALLS GPUS [OUT]
 *
 * LCP / BWT: totallength+1 raw bytes each (.lcp / .bwt); LLV: raw GtSmaxLlv
 * records (.llv).  The tables are read into malloc'd memory before any timed
 * region (a mapped index pays its page faults inside gt's own reader, which
 * is not what is measured here).  Timed: gt_smax_device_count() (HIP runtime
 * initialisation), then CALLS calls of gt_smax_hip_enumerate_to_buffer; the
 * first is the cold call.  GT_SMAX_E2E_PREPARE=1 issues gt_smax_hip_prepare
 * at process start, before the tables are read (read_s: that read).  With
 * OUT, the first call's (lcp, lb, rb) triples are written there (raw uint64)
 * for the caller's parity check.  Prints one JSON line on stdout.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "gt_smax_hip.h"

static double now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double) ts.tv_sec + 1e-9 * (double) ts.tv_nsec;
}

static void *slurp(const char *path, uint64_t want, uint64_t *got) {
  FILE *fp = fopen(path, "rb");
  if (fp == NULL) return NULL;
  if (fseek(fp, 0, SEEK_END) != 0) { fclose(fp); return NULL; }
  const long sz = ftell(fp);
  rewind(fp);
  if (sz < 0 || (want && (uint64_t) sz < want)) { fclose(fp); return NULL; }
  uint8_t *buf = malloc(sz > 0 ? (size_t) sz : 1);
  if (buf == NULL) { fclose(fp); return NULL; }
  uint64_t off = 0;
  while (off < (uint64_t) sz) {
    const size_t r = fread(buf + off, 1, (size_t) sz - off, fp);
    if (r == 0) break;
    off += r;
  }
  fclose(fp);
  if (off != (uint64_t) sz) { free(buf); return NULL; }
  *got = (uint64_t) sz;
  return buf;
}

int main(int argc, char **argv) {
  if (argc < 9) {
    fprintf(stderr, "usage: %s LCP BWT LLV TOTALLENGTH NONSPECIALS MINLEN CALLS GPUS [OUT]\n",
            argv[0]);
    return 2;
  }
  const uint64_t n = strtoull(argv[4], NULL, 10), N = strtoull(argv[5], NULL, 10);
  const unsigned minlen = (unsigned) strtoul(argv[6], NULL, 10);
  const int calls = atoi(argv[7]), gpus = atoi(argv[8]);
  const char *out = argc > 9 ? argv[9] : NULL;
  /* GT_SMAX_E2E_PREPARE=1: the runner's warm-up (gt_smax_hip_prepare) at
   * process start, before the tables are read -- as a gt repfind runner
   * issues it once the .prj has given the sizes */
  const char *pv = getenv("GT_SMAX_E2E_PREPARE");
  const int prepared = pv != NULL && atoi(pv) != 0;
  const double tr = now();
  if (prepared && gt_smax_hip_prepare(n, N, gpus) != 0) {
    fprintf(stderr, "gt-smax-e2e: gt_smax_hip_prepare failed\n");
    return 1;
  }
  uint64_t lsz = 0, bsz = 0, vsz = 0;
  uint8_t *lcp = slurp(argv[1], n + 1, &lsz), *bwt = slurp(argv[2], n + 1, &bsz);
  GtSmaxLlv *llv = slurp(argv[3], 0, &vsz);
  const double t_read = now() - tr;
  if (lcp == NULL || bwt == NULL || llv == NULL || vsz % sizeof (GtSmaxLlv) != 0 || calls < 1) {
    fprintf(stderr, "gt-smax-e2e: cannot read the tables\n");
    return 1;
  }
  GtSmaxInput in;
  memset(&in, 0, sizeof in);
  in.lcptab = lcp;
  in.bwttab = bwt;
  in.llvtab = vsz ? llv : NULL;
  in.numllv = vsz / sizeof (GtSmaxLlv);
  in.totallength = n;
  in.nonspecials = N;
  char err[1024];
  const double t0 = now();
  const int ndev = gt_smax_device_count();
  const double t_init = now() - t0;
  if (ndev < 1) {
    fprintf(stderr, "gt-smax-e2e: no HIP device\n");
    return 1;
  }
  printf("{\"prepared\": %s, \"read_s\": %.6f, \"hip_init_s\": %.6f, \"calls_s\": [",
         prepared ? "true" : "false", t_read, t_init);
  uint64_t first_count = 0;
  for (int c = 0; c < calls; c++) {
    uint64_t *trip = NULL, count = 0;
    err[0] = 0;
    fprintf(stderr, "[gt_smax call] %d\n", c);   /* separates GT_SMAX_TIMING's phase lines */
    const double t1 = now();
    const int rc = gt_smax_hip_enumerate_to_buffer(&in, minlen, gpus, &trip, &count, err, sizeof err);
    const double dt = now() - t1;
    if (rc != 0) {
      fprintf(stderr, "gt-smax-e2e: call %d failed: %s\n", c, err);
      return 1;
    }
    printf("%s%.6f", c ? ", " : "", dt);
    fflush(stdout);
    if (c == 0) {
      first_count = count;
      if (out != NULL) {
        FILE *fp = fopen(out, "wb");
        if (fp == NULL || fwrite(trip, sizeof (uint64_t) * 3, count, fp) != count) {
          fprintf(stderr, "gt-smax-e2e: cannot write %s\n", out);
          return 1;
        }
        fclose(fp);
      }
    }
    gt_smax_free(trip);
  }
  printf("], \"count\": %lu, \"devices\": %d}\n", (unsigned long) first_count, ndev);
  free(lcp);
  free(bwt);
  free(llv);
  return 0;
}
