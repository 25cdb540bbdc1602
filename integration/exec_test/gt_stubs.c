/*
 * gt_stubs.c -- test doubles for the few libgenometools symbols the shim
 * (integration/esa_linsmax.c) calls, so the shim can be linked and RUN
 * against libgtsmax_hip.so without building the reference.  This is not a
 * reference build: the shim is compiled against the reference's own headers
 * (struct layouts of Suffixarray, Sequentialsuffixarrayreader, GtGenericEncseq,
 * the GtProcessmaxpairs type), and only these functions are replaced:
 *
 *   gt_newSequentialsuffixarrayreaderfromfile  src/match/esa-seqread.h:217-222
 *     reads INDEX.prj (totallength, specialcharacters, readmode, mirrored)
 *     and, for the mapped mode, INDEX.{lcp,llv,bwt,suf} into a Suffixarray
 *     as esa-map.c would map them (8-byte .suf, as ESASuffixptr on LP64);
 *     with scanfile the tables are left to the caller, as the reference's
 *     streams are (the shim reads them itself)
 *   gt_suffixarraySequentialsuffixarrayreader, gt_encseqSequentialsuffixarrayreader,
 *   gt_freeSequentialsuffixarrayreader
 *   gt_encseq_total_length, gt_encseq_specialcharacters  (from the .prj)
 *   gt_error_set / gt_error_is_set, gt_malloc_mem / gt_realloc_mem / gt_free_mem
 *   gt_esa_visitor_visit_leaf_edge / _branching_edge / _lcp_interval,
 *   gt_esa_visitor_info_new / _delete (src/match/esa_visitor.h:30-61): a
 *   recording visitor -- every call printed with the ids of its
 *   GtESAVisitorInfo objects (numbered in creation order), every deletion
 *   printed, for gt_esa_bottomup_gpu's execution test
 *
 * The expected output of the execution test comes from the repo's oracle
 * (tests/test_shim_exec_gpu.py), never from these stubs.
 */
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "core/encseq.h"
#include "core/error_api.h"
#include "core/ma_api.h"
#include "match/esa-seqread.h"
#include "match/sarr-def.h"
#include "match/esa_visitor.h"

struct GtEncseq {
  GtUword totallength, specialcharacters;
};

struct GtError {
  char msg[4096];
  bool isset;
};

void gt_error_set(GtError *err, const char *format, ...)
{
  va_list ap;
  if (err == NULL) return;
  va_start(ap, format);
  (void) vsnprintf(err->msg, sizeof err->msg, format, ap);
  va_end(ap);
  err->isset = true;
}

bool gt_error_is_set(const GtError *err)
{
  return err != NULL && err->isset;
}

void *gt_malloc_mem(size_t size, const char *src_file, int src_line)
{
  void *p = malloc(size ? size : 1);
  (void) src_file; (void) src_line;
  if (p == NULL) { perror("malloc"); exit(2); }
  return p;
}

void *gt_realloc_mem(void *ptr, size_t size, const char *src_file, int src_line)
{
  void *p = realloc(ptr, size ? size : 1);
  (void) src_file; (void) src_line;
  if (p == NULL) { perror("realloc"); exit(2); }
  return p;
}

void gt_free_mem(void *ptr, const char *src_file, int src_line)
{
  (void) src_file; (void) src_line;
  free(ptr);
}

GtUword gt_encseq_total_length(const GtEncseq *encseq)
{
  return encseq->totallength;
}

GtUword gt_encseq_specialcharacters(const GtEncseq *encseq)
{
  return encseq->specialcharacters;
}

static void *stub_read(const char *indexname, const char *suffix, GtUword *bytes)
{
  char path[4096];
  FILE *fp;
  long size;
  void *buf;
  (void) snprintf(path, sizeof path, "%s%s", indexname, suffix);
  *bytes = 0;
  if ((fp = fopen(path, "rb")) == NULL) return NULL;
  (void) fseek(fp, 0, SEEK_END);
  size = ftell(fp);
  (void) fseek(fp, 0, SEEK_SET);
  buf = malloc((size_t) size + 1);
  if (size > 0 && fread(buf, 1, (size_t) size, fp) != (size_t) size) { free(buf); buf = NULL; }
  (void) fclose(fp);
  *bytes = (GtUword) size;
  return buf;
}

Sequentialsuffixarrayreader *gt_newSequentialsuffixarrayreaderfromfile(
                                        const char *indexname,
                                        unsigned int demand,
                                        bool scanfile,
                                        GtLogger *logger,
                                        GtError *err)
{
  char path[4096], line[512];
  FILE *fp;
  Sequentialsuffixarrayreader *ssar;
  Suffixarray *sa;
  GtEncseq *es;
  GtUword bytes, readmode = 0, mirrored = 0;
  (void) logger;
  (void) snprintf(path, sizeof path, "%s.prj", indexname);
  if ((fp = fopen(path, "r")) == NULL) {
    gt_error_set(err, "cannot open file \"%s\"", path);
    return NULL;
  }
  ssar = calloc(1, sizeof *ssar);
  sa = calloc(1, sizeof *sa);
  es = calloc(1, sizeof *es);
  while (fgets(line, sizeof line, fp) != NULL) {
    unsigned long v;
    if (sscanf(line, "totallength=%lu", &v) == 1) es->totallength = v;
    else if (sscanf(line, "specialcharacters=%lu", &v) == 1) es->specialcharacters = v;
    else if (sscanf(line, "readmode=%lu", &v) == 1) readmode = v;
    else if (sscanf(line, "mirrored=%lu", &v) == 1) mirrored = v;
    else if (sscanf(line, "largelcpvalues=%lu", &v) == 1) {
      sa->numoflargelcpvalues.defined = true;
      sa->numoflargelcpvalues.valueunsignedlong = v;
    }
  }
  (void) fclose(fp);
  sa->encseq = es;
  sa->readmode = (GtReadmode) readmode;
  sa->mirroredencseq = mirrored != 0;
  if (!scanfile) {
    if (demand & SARR_LCPTAB) sa->lcptab = stub_read(indexname, ".lcp", &bytes);
    if (demand & SARR_LCPTAB) sa->llvtab = stub_read(indexname, ".llv", &bytes);
    if (demand & SARR_BWTTAB) sa->bwttab = stub_read(indexname, ".bwt", &bytes);
    if (demand & SARR_SUFTAB) {
      sa->suftab = stub_read(indexname, ".suf", &bytes);
      if (bytes != sizeof (ESASuffixptr) * (es->totallength + 1)) {
        gt_error_set(err, "stub reader: mapped .suf must hold %u-byte entries",
                     (unsigned) sizeof (ESASuffixptr));
        return NULL;
      }
    }
    if (sa->lcptab == NULL || ((demand & SARR_BWTTAB) && sa->bwttab == NULL)) {
      gt_error_set(err, "stub reader: missing .lcp/.bwt of %s", indexname);
      return NULL;
    }
  }
  ssar->suffixarray = sa;
  ssar->encseq = es;
  ssar->scanfile = scanfile;
  ssar->readmode = sa->readmode;
  return ssar;
}

const Suffixarray *gt_suffixarraySequentialsuffixarrayreader(
              const Sequentialsuffixarrayreader *ssar)
{
  return ssar->suffixarray;
}

const GtEncseq *gt_encseqSequentialsuffixarrayreader(
                          const Sequentialsuffixarrayreader *ssar)
{
  return ssar->encseq;
}

void gt_freeSequentialsuffixarrayreader(Sequentialsuffixarrayreader **ssar)
{
  Suffixarray *sa;
  if (ssar == NULL || *ssar == NULL) return;
  sa = (*ssar)->suffixarray;
  free((void *) sa->lcptab);
  free((void *) sa->llvtab);
  free((void *) sa->bwttab);
  free((void *) sa->suftab);
  free(sa->encseq);
  free(sa);
  free(*ssar);
  *ssar = NULL;
}

/* ---------------------------------------------- recording GtESAVisitor */

struct GtESAVisitor {
  FILE *out;
  GtUword next_id;
};

struct GtESAVisitorInfo {
  GtUword id;
};

GtESAVisitor *stub_visitor_new(FILE *out)
{
  GtESAVisitor *ev = calloc(1, sizeof *ev);
  ev->out = out;
  return ev;
}

GtESAVisitorInfo *gt_esa_visitor_info_new(GtESAVisitor *ev)
{
  GtESAVisitorInfo *info = malloc(sizeof *info);
  info->id = ++ev->next_id;
  return info;
}

void gt_esa_visitor_info_delete(GtESAVisitorInfo *info, GtESAVisitor *ev)
{
  if (info == NULL) return;
  fprintf(ev->out, "D %lu\n", (unsigned long) info->id);
  free(info);
}

int gt_esa_visitor_visit_leaf_edge(GtESAVisitor *ev, bool firstsucc, GtUword fd,
                                   GtUword flb, GtESAVisitorInfo *finfo,
                                   GtUword leafnumber, GtError *err)
{
  (void) err;
  fprintf(ev->out, "0 %d %lu %lu %lu 0 0 %lu 0\n", firstsucc ? 1 : 0,
          (unsigned long) fd, (unsigned long) flb, (unsigned long) leafnumber,
          (unsigned long) (finfo ? finfo->id : 0));
  return 0;
}

int gt_esa_visitor_visit_branching_edge(GtESAVisitor *ev, bool firstsucc,
                                        GtUword fd, GtUword flb,
                                        GtESAVisitorInfo *finfo, GtUword sd,
                                        GtUword slb, GtUword srb,
                                        GtESAVisitorInfo *sinfo, GtError *err)
{
  (void) err;
  fprintf(ev->out, "1 %d %lu %lu %lu %lu %lu %lu %lu\n", firstsucc ? 1 : 0,
          (unsigned long) fd, (unsigned long) flb, (unsigned long) sd,
          (unsigned long) slb, (unsigned long) srb,
          (unsigned long) (finfo ? finfo->id : 0),
          (unsigned long) (sinfo ? sinfo->id : 0));
  return 0;
}

int gt_esa_visitor_visit_lcp_interval(GtESAVisitor *ev, GtUword lcp, GtUword lb,
                                      GtUword rb, GtESAVisitorInfo *info,
                                      GtError *err)
{
  (void) err;
  fprintf(ev->out, "2 0 %lu %lu %lu 0 0 %lu 0\n", (unsigned long) lcp,
          (unsigned long) lb, (unsigned long) rb,
          (unsigned long) (info ? info->id : 0));
  return 0;
}
