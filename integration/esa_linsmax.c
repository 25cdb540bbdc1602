/*
 * esa_linsmax.c -- GenomeTools-side shim of the MI355X smax layer.
 *
 * Belongs in the reference tree as src/match/esa_linsmax.c.  It opens the
 * index with the reference's own sequential reader
 * (gt_newSequentialsuffixarrayreaderfromfile, src/match/esa-seqread.h:217-222)
 * asking for the BWT table in addition to what gt_callenummaxpairs maps
 * (src/match/esa-maxpairs.c:488-495), hands the mapped tables of the
 * Suffixarray (src/match/sarr-def.h:101-126, through
 * gt_suffixarraySequentialsuffixarrayreader, esa-seqread.h:238-239) to
 * libgtsmax_hip.so as plain pointers, and forwards the results to the
 * caller's GtProcessmaxpairs function with a GtGenericEncseq built as
 * gt_enumeratemaxpairs_generic does (src/match/esa-maxpairs.c:407-410).
 *
 * With -scan the reference streams the tables through FILE buffers instead
 * of mapping them (Suffixarray's *stream members, sarr-def.h:117-123); the
 * GPU needs whole tables, so the shim reads .lcp/.llv/.bwt/.suf itself
 * (4-byte .suf from -suftabuint is accepted there, esa-map.c:362-381).
 *
 * Errors: the library's errbuf is copied into GtError; return 0 / -1 as
 * gt_callenummaxpairs does (haserr ? -1 : 0, esa-maxpairs.c:519).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "core/encseq.h"
#include "core/error_api.h"
#include "core/logger_api.h"
#include "core/ma_api.h"
#include "match/esa-maxpairs.h"
#include "match/esa-seqread.h"
#include "match/sarr-def.h"
#include "match/esa_linsmax.h"
#include "match/esa_visitor.h"
#include "gt_lcpitv_hip.h"
#include "gt_maxpairs_hip.h"
#include "gt_smax_hip.h"

typedef struct
{
  GtProcessmaxpairs processmaxpairs;
  void *processmaxpairsinfo;
  GtGenericEncseq genericencseq;
  const void *suftab;
  int suftab_bytes;
  GtUword *occ;
  GtUword occcap;
  GtError *err;
} GtSmaxShimState;

/* tables the shim read itself (-scan) */
typedef struct
{
  void *lcptab, *llvtab, *bwttab, *suftab;
} GtSmaxScanTables;

static GtUword smax_shim_suffix(const GtSmaxShimState *st, GtUword row)
{
  return st->suftab_bytes == 4 ? (GtUword) ((const uint32_t *) st->suftab)[row]
                               : (GtUword) ((const uint64_t *) st->suftab)[row];
}

/* GtSmaxIntervalFunc: every occurrence pair of [lb..rb], in occurrence-row
   order, to the repfind output function (the pairs gt_repfind -smax prints) */
static int smax_shim_interval(void *data, uint64_t lcp, uint64_t lb,
                              uint64_t rb)
{
  GtSmaxShimState *st = data;
  GtUword w = (GtUword) (rb - lb + 1), a, b;

  if (w > st->occcap)
  {
    st->occ = gt_realloc(st->occ, sizeof (*st->occ) * w);
    st->occcap = w;
  }
  for (a = 0; a < w; a++)
  {
    st->occ[a] = smax_shim_suffix(st, (GtUword) lb + a);
  }
  for (a = 0; a < w; a++)
  {
    for (b = a + 1; b < w; b++)
    {
      if (st->processmaxpairs(st->processmaxpairsinfo, &st->genericencseq,
                              (GtUword) lcp, st->occ[a], st->occ[b],
                              st->err) != 0)
      {
        return -1;
      }
    }
  }
  return 0;
}

/* GtMaxpairsFunc: one maximal pair */
static int smax_shim_maxpair(void *data, uint64_t len, uint64_t pos1,
                             uint64_t pos2)
{
  GtSmaxShimState *st = data;
  return st->processmaxpairs(st->processmaxpairsinfo, &st->genericencseq,
                             (GtUword) len, (GtUword) pos1, (GtUword) pos2,
                             st->err);
}

static void *smax_shim_readfile(const char *indexname, const char *suffix,
                                GtUword *bytes, bool mustexist, GtError *err)
{
  char path[4096];
  FILE *fp;
  void *buf = NULL;
  long size;

  (void) snprintf(path, sizeof path, "%s%s", indexname, suffix);
  *bytes = 0;
  fp = fopen(path, "rb");
  if (fp == NULL)
  {
    if (mustexist)
    {
      gt_error_set(err, "cannot open file \"%s\"", path);
    }
    return NULL;
  }
  if (fseek(fp, 0, SEEK_END) != 0 || (size = ftell(fp)) < 0 ||
      fseek(fp, 0, SEEK_SET) != 0)
  {
    gt_error_set(err, "cannot determine the size of \"%s\"", path);
    (void) fclose(fp);
    return NULL;
  }
  buf = gt_malloc((size_t) size + 1);
  if (size > 0 && fread(buf, 1, (size_t) size, fp) != (size_t) size)
  {
    gt_error_set(err, "cannot read \"%s\"", path);
    gt_free(buf);
    buf = NULL;
  } else
  {
    *bytes = (GtUword) size;
  }
  (void) fclose(fp);
  return buf;
}

/* fills in from the reader's Suffixarray (mapped) or reads the tables (scan) */
static int smax_shim_input(const char *indexname, bool scanfile,
                           const Suffixarray *sa, GtSmaxInput *in,
                           GtSmaxScanTables *own, GtError *err)
{
  const GtUword totallength = gt_encseq_total_length(sa->encseq);

  memset(in, 0, sizeof *in);
  memset(own, 0, sizeof *own);
  in->totallength = (uint64_t) totallength;
  in->nonspecials = (uint64_t) (totallength -
                                gt_encseq_specialcharacters(sa->encseq));
  if (sa->readmode != GT_READMODE_FORWARD || sa->mirroredencseq)
  {
    gt_error_set(err, "smax supports forward, non-mirrored indexes only");
    return -1;
  }
  if (!scanfile)
  {
    in->lcptab = sa->lcptab;
    in->llvtab = (const GtSmaxLlv *) sa->llvtab;
    in->numllv = (uint64_t) sa->numoflargelcpvalues.valueunsignedlong;
    in->bwttab = sa->bwttab;
    in->suftab = sa->suftab;
    in->suftab_bytes = (int) sizeof (ESASuffixptr);
  } else
  {
    GtUword bytes;

    own->lcptab = smax_shim_readfile(indexname, ".lcp", &bytes, true, err);
    if (own->lcptab == NULL || bytes != totallength + 1)
    {
      if (own->lcptab != NULL)
      {
        gt_error_set(err, "%s.lcp: unexpected size " GT_WU, indexname, bytes);
      }
      return -1;
    }
    own->bwttab = smax_shim_readfile(indexname, ".bwt", &bytes, true, err);
    if (own->bwttab == NULL || bytes != totallength + 1)
    {
      if (own->bwttab != NULL)
      {
        gt_error_set(err, "%s.bwt: unexpected size " GT_WU, indexname, bytes);
      }
      return -1;
    }
    own->llvtab = smax_shim_readfile(indexname, ".llv", &bytes, false, err);
    if (bytes % sizeof (Largelcpvalue) != 0)
    {
      gt_error_set(err, "%s.llv: size not a multiple of " GT_WU, indexname,
                   (GtUword) sizeof (Largelcpvalue));
      return -1;
    }
    in->numllv = (uint64_t) (bytes / sizeof (Largelcpvalue));
    own->suftab = smax_shim_readfile(indexname, ".suf", &bytes, true, err);
    if (own->suftab == NULL)
    {
      return -1;
    }
    if (bytes == sizeof (uint32_t) * (totallength + 1))
    {
      in->suftab_bytes = 4;
    } else if (bytes == sizeof (uint64_t) * (totallength + 1))
    {
      in->suftab_bytes = 8;
    } else
    {
      gt_error_set(err, "%s.suf: number of mapped units does not match",
                   indexname);
      return -1;
    }
    in->lcptab = own->lcptab;
    in->llvtab = own->llvtab;
    in->bwttab = own->bwttab;
    in->suftab = own->suftab;
  }
  return 0;
}

static void smax_shim_free(GtSmaxScanTables *own)
{
  gt_free(own->lcptab);
  gt_free(own->llvtab);
  gt_free(own->bwttab);
  gt_free(own->suftab);
}

static int smax_shim_run(const char *indexname, unsigned int minlen,
                         bool scanfile, int num_gpus, bool supermax,
                         GtProcessmaxpairs processmaxpairs,
                         void *processmaxpairsinfo, GtLogger *logger,
                         GtError *err)
{
  bool haserr = false;
  Sequentialsuffixarrayreader *ssar;
  GtSmaxScanTables own;
  GtSmaxInput in;
  GtSmaxShimState st;
  char msg[1024];

  gt_error_check(err);
  memset(&own, 0, sizeof own);
  /* the tables gt_callenummaxpairs asks for, plus the BWT */
  ssar = gt_newSequentialsuffixarrayreaderfromfile(indexname,
                                                   SARR_LCPTAB |
                                                   SARR_SUFTAB |
                                                   SARR_ESQTAB |
                                                   SARR_SSPTAB |
                                                   SARR_BWTTAB,
                                                   scanfile,
                                                   logger,
                                                   err);
  if (ssar == NULL)
  {
    return -1;
  }
  if (smax_shim_input(indexname, scanfile,
                      gt_suffixarraySequentialsuffixarrayreader(ssar), &in,
                      &own, err) != 0)
  {
    haserr = true;
  }
  if (!haserr)
  {
    memset(&st, 0, sizeof st);
    st.processmaxpairs = processmaxpairs;
    st.processmaxpairsinfo = processmaxpairsinfo;
    st.genericencseq.hasencseq = true;            /* esa-maxpairs.c:409-410 */
    st.genericencseq.seqptr.encseq = gt_encseqSequentialsuffixarrayreader(ssar);
    st.suftab = in.suftab;
    st.suftab_bytes = in.suftab_bytes;
    st.err = err;
    msg[0] = '\0';
    if ((supermax
         ? gt_smax_hip_enumerate(&in, minlen, num_gpus, smax_shim_interval,
                                 &st, msg, sizeof msg)
         : gt_maxpairs_hip_enumerate(&in, minlen, smax_shim_maxpair, &st,
                                     msg, sizeof msg)) != 0)
    {
      if (!gt_error_is_set(err))
      {
        gt_error_set(err, "%s", msg);
      }
      haserr = true;
    }
    gt_free(st.occ);
  }
  smax_shim_free(&own);
  gt_freeSequentialsuffixarrayreader(&ssar);
  return haserr ? -1 : 0;
}

int gt_callenumsupermaxrepeats(const char *indexname,
                               unsigned int userdefinedleastlength,
                               bool scanfile,
                               int num_gpus,
                               GtProcessmaxpairs processmaxpairs,
                               void *processmaxpairsinfo,
                               GtLogger *logger,
                               GtError *err)
{
  return smax_shim_run(indexname, userdefinedleastlength, scanfile, num_gpus,
                       true, processmaxpairs, processmaxpairsinfo, logger,
                       err);
}

int gt_callenummaxpairs_hip(const char *indexname,
                            unsigned int userdefinedleastlength,
                            bool scanfile,
                            GtProcessmaxpairs processmaxpairs,
                            void *processmaxpairsinfo,
                            GtLogger *logger,
                            GtError *err)
{
  return smax_shim_run(indexname, userdefinedleastlength, scanfile, 1, false,
                       processmaxpairs, processmaxpairsinfo, logger, err);
}

/* ------------------------------------------- gt_esa_bottomup on the GPU */

typedef struct
{
  GtESAVisitor *ev;
  GtError *err;
} GtEsaBottomupGpu;

static int gpu_bu_leaf(void *data, int firstsucc, uint64_t fd, uint64_t flb,
                       void *finfo, uint64_t leafnumber)
{
  GtEsaBottomupGpu *st = data;
  return gt_esa_visitor_visit_leaf_edge(st->ev, firstsucc != 0, (GtUword) fd,
                                        (GtUword) flb, finfo,
                                        (GtUword) leafnumber, st->err);
}

static int gpu_bu_branch(void *data, int firstsucc, uint64_t fd, uint64_t flb,
                         void *finfo, uint64_t sd, uint64_t slb, uint64_t srb,
                         void *sinfo)
{
  GtEsaBottomupGpu *st = data;
  return gt_esa_visitor_visit_branching_edge(st->ev, firstsucc != 0,
                                             (GtUword) fd, (GtUword) flb,
                                             finfo, (GtUword) sd,
                                             (GtUword) slb, (GtUword) srb,
                                             sinfo, st->err);
}

static int gpu_bu_interval(void *data, uint64_t lcp, uint64_t lb, uint64_t rb,
                           void *info)
{
  GtEsaBottomupGpu *st = data;
  return gt_esa_visitor_visit_lcp_interval(st->ev, (GtUword) lcp,
                                           (GtUword) lb, (GtUword) rb, info,
                                           st->err);
}

static void *gpu_bu_info_new(void *data)
{
  GtEsaBottomupGpu *st = data;
  return gt_esa_visitor_info_new(st->ev);
}

static void gpu_bu_info_delete(void *info, void *data)
{
  GtEsaBottomupGpu *st = data;
  gt_esa_visitor_info_delete(info, st->ev);
}

int gt_esa_bottomup_gpu(Sequentialsuffixarrayreader *ssar, GtESAVisitor *ev,
                        GtError *err)
{
  const Suffixarray *sa = gt_suffixarraySequentialsuffixarrayreader(ssar);
  GtLcpitvInfoVisitor v;
  GtEsaBottomupGpu st;
  GtSmaxInput in;
  char msg[1024];
  GtUword totallength;

  gt_error_check(err);
  if (sa == NULL || sa->lcptab == NULL || sa->suftab == NULL)
  {
    gt_error_set(err, "gt_esa_bottomup_gpu needs the mapped lcp and suffix "
                      "tables (a reader opened without scanfile)");
    return -1;
  }
  totallength = gt_encseq_total_length(sa->encseq);
  memset(&in, 0, sizeof in);
  in.lcptab = sa->lcptab;
  in.llvtab = (const GtSmaxLlv *) sa->llvtab;
  in.numllv = (uint64_t) sa->numoflargelcpvalues.valueunsignedlong;
  in.bwttab = sa->bwttab;
  in.suftab = sa->suftab;
  in.suftab_bytes = (int) sizeof (ESASuffixptr);
  in.totallength = (uint64_t) totallength;
  in.nonspecials = (uint64_t) (totallength -
                               gt_encseq_specialcharacters(sa->encseq));
  st.ev = ev;
  st.err = err;
  v.leaf_edge = gpu_bu_leaf;
  v.branching_edge = gpu_bu_branch;
  v.lcp_interval = gpu_bu_interval;
  v.info_new = gpu_bu_info_new;
  v.info_delete = gpu_bu_info_delete;
  msg[0] = '\0';
  if (gt_esa_bottomup_info_hip(&in, &v, &st, msg, sizeof msg) != 0)
  {
    if (!gt_error_is_set(err))
    {
      gt_error_set(err, "%s", msg);
    }
    return -1;
  }
  return 0;
}
