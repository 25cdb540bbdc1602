/*
 * esa_reader.h -- C host reader of a GenomeTools enhanced suffix array.
 *
 * Restates the parts of Suffixarray / gt_mapsuffixarray / streamsuffixarray
 * the smax path needs (src/match/sarr-def.h:101-126,
 * src/match/esa-map.c:55-214 (.prj checks), :296-515 (table mapping)), without
 * linking libgenometools: tables are mmap'd (or read with -scan), sizes are
 * checked against totallength+1, nonspecials = totallength -
 * specialcharacters (src/match/esa-seqread.c:56-57), and sequence boundaries
 * come from the separator rows of .bwt instead of the encseq's .ssp.
 */
#ifndef SMAX_ESA_READER_H
#define SMAX_ESA_READER_H

#include <stddef.h>
#include <stdint.h>

#include "gt_smax_hip.h"

typedef struct {
  uint64_t totallength, specialcharacters, nonspecials, numofsequences,
           largelcpvalues;
  int integersize, littleendian, readmode, mirrored;
  int has_largelcpvalues, has_numofsequences;
  const uint8_t *lcptab, *bwttab;
  const GtSmaxLlv *llvtab;
  uint64_t numllv;
  const void *suftab;
  int suftab_bytes;
  /* mappings to release */
  void *maps[4];
  size_t mapsizes[4];
  int scanned;
} SmaxEsa;

/* The .prj's totallength and nonspecials (totallength - specialcharacters)
 * alone, before any table is mapped: 0, or -1 with a message. */
int smax_esa_sizes(const char *indexname, uint64_t *totallength, uint64_t *nonspecials,
                   char *errbuf, size_t errlen);
/* 0 on success, -1 with a gt-style message in errbuf. */
int smax_esa_open(SmaxEsa *esa, const char *indexname, int need_suftab,
                  int scanfile, char *errbuf, size_t errlen);
/* Same, with the .bwt table optional (need_bwt == 0: esa->bwttab NULL). */
int smax_esa_open_tables(SmaxEsa *esa, const char *indexname, int need_suftab,
                         int need_bwt, int scanfile, char *errbuf, size_t errlen);
void smax_esa_close(SmaxEsa *esa);
uint64_t smax_esa_suffix(const SmaxEsa *esa, uint64_t idx);
void smax_esa_input(const SmaxEsa *esa, GtSmaxInput *in);

/* Sorted separator positions {suftab[k]-1 : bwt[k] == 255}. */
int smax_esa_separators(const SmaxEsa *esa, uint64_t **sep, uint64_t *nsep);

#endif
