/*
 * gt_smax_esa.h -- GPU construction of the smax inputs:
 * the `gt suffixerator -dna -suf -lcp -bwt` tables, built in HBM.
 *
 * Replaces, for the smax path, suffixeratorwithoutput
 * (src/match/sfx-run.c:213-300): bwttab2file (:174-212), outlcpvalues
 * (src/match/sfx-lcpvalues.c:371-470) and the suffix sort.  Output tables are
 * byte-identical to suffixerator's (.suf values, .lcp bytes, .llv entries,
 * .bwt bytes), plus the packed bit-plane BWT the smax scan streams
 * (GT_SMAX_PK_GROUPS in gt_smax_hip.h), emitted with the BWT bytes.  Limited
 * to n+1 < 2^32 suffixes (32-bit suffix array).
 */
#ifndef GT_SMAX_ESA_H
#define GT_SMAX_ESA_H

#include <stddef.h>
#include <stdint.h>

#include "gt_smax_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int device;
  uint64_t totallength, nonspecials, numllv, maxbranchdepth;
  double averagelcp;
  int sort_rounds;            /* prefix-doubling rounds after the 21-mer sort */
  uint8_t *lcptab_dev;        /* totallength+1 bytes, GT_SMAX_PAD layout     */
  uint8_t *bwttab_dev;        /* totallength+1 bytes, GT_SMAX_PAD layout     */
  GtSmaxLlv *llvtab_dev;      /* numllv entries                              */
  uint32_t *suftab_dev;       /* totallength+1 entries, or NULL              */
  uint64_t *bwtpk_dev;        /* packed BWT, GT_SMAX_PK_GROUPS(totallength+1) */
} GtSmaxEsaDev;

/* text: n encoded symbols on the host (0..3, 254 wildcard, 255 separator). */
int gt_smax_esa_build(int device, const uint8_t *text, uint64_t n,
                      int keep_suftab, GtSmaxEsaDev *out, char *errbuf,
                      size_t errlen);

/* Copies tables to host buffers (any may be NULL); suftab widened to 8 B. */
int gt_smax_esa_download(const GtSmaxEsaDev *esa, uint8_t *lcptab,
                         uint8_t *bwttab, GtSmaxLlv *llvtab, uint64_t *suftab,
                         char *errbuf, size_t errlen);

/* Copies the packed BWT (GT_SMAX_PK_GROUPS(totallength+1) u64) to pk. */
int gt_smax_esa_download_packed(const GtSmaxEsaDev *esa, uint64_t *pk,
                                char *errbuf, size_t errlen);

void gt_smax_esa_release(GtSmaxEsaDev *esa);

/*
 * 64-bit, range-restricted builder (esa_build64.hip): the rows
 * [row_lo, row_hi) of the suffix array of text[0 .. n) (n+1 suffixes,
 * row_hi == 0 means n+1), for texts of any length -- BASELINE config C5
 * (12 Gbp, > 2^32 suffixes, 8-byte suftab as the reference mandates there,
 * src/match/sfx-suffixgetset.c:48-51) and the per-rank builds of a
 * suffix-array range.  Tables are local: lcptab_dev[i] is
 * LCP[row_lo + i] (GT_SMAX_PAD layout), likewise bwttab_dev/suftab_dev, the
 * packed BWT covers the local rows (GT_SMAX_PK_GROUPS(row_hi - row_lo)),
 * .llv positions are global rows in [row_lo, row_hi).  Byte-identical to
 * gt_smax_esa_build on the rows both build.  batch_max caps the suffixes
 * sorted together (0: as the free HBM allows).
 */
typedef struct {
  int device;
  uint64_t totallength, nonspecials;   /* of the whole text                  */
  uint64_t row_lo, row_hi;             /* rows held                          */
  uint64_t numllv, maxbranchdepth;     /* maxbranchdepth: max LCP of the rows */
  double averagelcp;                   /* over the rows held                 */
  int sort_rounds, batches;
  uint8_t *lcptab_dev;
  uint8_t *bwttab_dev;
  uint64_t *bwtpk_dev;
  GtSmaxLlv *llvtab_dev;
  uint64_t *suftab_dev;                /* 8-byte suffixes, or NULL           */
} GtSmaxEsa64Dev;

int gt_smax_esa64_build(int device, const uint8_t *text, uint64_t n,
                        uint64_t row_lo, uint64_t row_hi, int keep_suftab,
                        uint64_t batch_max, GtSmaxEsa64Dev *out,
                        char *errbuf, size_t errlen);

/* Copies the held rows' tables to host buffers (any may be NULL). */
int gt_smax_esa64_download(const GtSmaxEsa64Dev *esa, uint8_t *lcptab,
                           uint8_t *bwttab, GtSmaxLlv *llvtab,
                           uint64_t *suftab, uint64_t *bwtpk, char *errbuf,
                           size_t errlen);

void gt_smax_esa64_release(GtSmaxEsa64Dev *esa);

/*
 * The file side of the GPU suffixerator.
 *
 * gt_smax_encode_fasta: (multi-)FASTA bytes -> encoded DNA text (a/c/g/t/u
 * -> 0..3, IUPAC wildcards -> 254, one SEPARATOR 255 between sequences), as
 * GenomeTools' DNA alphabet and encseq produce it (src/core/alphabet.c:63,
 * 440-465; src/core/chardef.h:34-40).  out holds >= len bytes.
 *
 * gt_smax_esa64_write: a whole-array build (rows [0, n+1), keep_suftab) ->
 * indexname.{suf,lcp,llv,bwt,prj} as `gt suffixerator -dna -suf -lcp -bwt`
 * writes them (src/match/sfx-run.c:174-300, src/match/sfx-outprj.c:39-120);
 * suftab_bytes 8, or 4 (-suftabuint) when n+1 < 2^32.  dbfile / dbfile_bytes
 * name the FASTA in the .prj's dbfile line.
 */
int gt_smax_encode_fasta(const char *buf, uint64_t len, uint8_t *out,
                         uint64_t *n, uint64_t *numseq, char *errbuf,
                         size_t errlen);
int gt_smax_esa64_write(const GtSmaxEsa64Dev *esa, const uint8_t *text,
                        uint64_t n, uint64_t numseq, const char *dbfile,
                        uint64_t dbfile_bytes, const char *indexname,
                        int suftab_bytes, char *errbuf, size_t errlen);

#ifdef __cplusplus
}
#endif

#endif
