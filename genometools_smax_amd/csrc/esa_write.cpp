// esa_write.cpp -- the file side of the GPU suffixerator:
// FASTA -> GenomeTools' encoded DNA text, and a GPU-built ESA -> the
// .suf/.lcp/.llv/.bwt/.prj files `gt suffixerator -dna -suf -lcp -bwt`
// writes (src/match/sfx-run.c:174-300 tables, src/match/sfx-outprj.c:39-120
// project file, including `longest=`, the row of suffix 0, that esa-map.c:384-387
// requires with SARR_SUFTAB).  No encoded-sequence files (.esq/.ssp/.des/.sds)
// are written, so such an index is read by this repo's bin/gt-repfind (and
// anything else that maps only .suf/.lcp/.llv/.bwt/.prj), not by the
// reference's readers, which also ask for SARR_ESQTAB.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "gt_smax_esa.h"

namespace {

void seterr(char *errbuf, size_t errlen, const char *fmt, ...) {
  if (errbuf == NULL || errlen == 0) return;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(errbuf, errlen, fmt, ap);
  va_end(ap);
}

// DNA alphabet of src/core/alphabet.c:63,440-465: a/A c/C g/G t/T/u/U ->
// 0..3, the IUPAC wildcards nsywrkvbdhm (either case) -> WILDCARD (254)
int dna_code(unsigned char c) {
  switch (c) {
    case 'a': case 'A': return 0;
    case 'c': case 'C': return 1;
    case 'g': case 'G': return 2;
    case 't': case 'T': case 'u': case 'U': return 3;
    case 'n': case 'N': case 's': case 'S': case 'y': case 'Y': case 'w': case 'W':
    case 'r': case 'R': case 'k': case 'K': case 'v': case 'V': case 'b': case 'B':
    case 'd': case 'D': case 'h': case 'H': case 'm': case 'M':
      return 254;
    default:
      return -1;
  }
}

// special-range statistics of the .prj (count, ranges, prefix, suffix run)
void range_stats(const uint8_t *t, uint64_t n, bool wildonly, uint64_t out[4]) {
  uint64_t c = 0, r = 0, pre = 0, suf = 0;
  bool prev = false;
  auto sp = [&](uint64_t i) { return wildonly ? t[i] == 254 : t[i] >= 254; };
  for (uint64_t i = 0; i < n; i++) {
    const bool s = sp(i);
    if (s) { c++; if (!prev) r++; }
    prev = s;
  }
  while (pre < n && sp(pre)) pre++;
  while (suf < n && sp(n - 1 - suf)) suf++;
  out[0] = c; out[1] = r; out[2] = pre; out[3] = suf;
}

// device bytes -> file, through a bounce buffer
bool dev_to_file(FILE *fp, const void *dev, uint64_t bytes, std::vector<char> &buf) {
  const uint64_t CH = buf.size();
  for (uint64_t off = 0; off < bytes; off += CH) {
    const uint64_t n = std::min(CH, bytes - off);
    if (hipMemcpy(buf.data(), (const char *) dev + off, n, hipMemcpyDeviceToHost) != hipSuccess)
      return false;
    if (fwrite(buf.data(), 1, n, fp) != n) return false;
  }
  return true;
}

}  // namespace

extern "C" int gt_smax_encode_fasta(const char *buf, uint64_t len, uint8_t *out, uint64_t *n_out,
                                    uint64_t *numseq_out, char *errbuf, size_t errlen) {
  uint64_t n = 0, numseq = 0;
  bool inheader = false, atlinestart = true;
  for (uint64_t i = 0; i < len; i++) {
    const unsigned char c = (unsigned char) buf[i];
    if (c == '\n') { inheader = false; atlinestart = true; continue; }
    if (inheader) continue;
    if (atlinestart && c == '>') {
      if (numseq > 0) out[n++] = 255;   // SEPARATOR between sequences
      numseq++;
      inheader = true;
      atlinestart = false;
      continue;
    }
    atlinestart = false;
    if (c == ' ' || c == '\t' || c == '\r') continue;
    const int code = dna_code(c);
    if (code < 0) {
      seterr(errbuf, errlen, "illegal character '%c' (0x%02x) at offset %lu", c >= 32 && c < 127 ? c : '?',
             c, (unsigned long) i);
      return -1;
    }
    if (numseq == 0) numseq = 1;
    out[n++] = (uint8_t) code;
  }
  *n_out = n;
  *numseq_out = numseq;
  return 0;
}

extern "C" int gt_smax_esa64_write(const GtSmaxEsa64Dev *e, const uint8_t *text, uint64_t n,
                                   uint64_t numseq, const char *dbfile, uint64_t dbfile_bytes,
                                   const char *indexname, int suftab_bytes, char *errbuf,
                                   size_t errlen) {
  const uint64_t m = n + 1;
  std::vector<char> buf(64u << 20);
  std::string base(indexname);
  FILE *fp = NULL;
  uint64_t sp[4], wc[4], longest = UINT64_MAX;
  if (errbuf && errlen) errbuf[0] = 0;
  if (e->row_lo != 0 || e->row_hi != m || e->totallength != n) {
    seterr(errbuf, errlen, "index files need the whole suffix array (rows [0, %lu))",
           (unsigned long) m);
    return -1;
  }
  if (e->suftab_dev == NULL) {
    seterr(errbuf, errlen, ".suf needs the suffix array: build with keep_suftab");
    return -1;
  }
  if (suftab_bytes != 8 && !(suftab_bytes == 4 && m <= 0xffffffffull)) {
    seterr(errbuf, errlen, "suffix width %d unsupported for %lu suffixes", suftab_bytes,
           (unsigned long) m);
    return -1;
  }
  if (hipSetDevice(e->device) != hipSuccess) {
    seterr(errbuf, errlen, "hipSetDevice failed");
    return -1;
  }
  auto open = [&](const char *suffix, const char *mode) {
    fp = fopen((base + suffix).c_str(), mode);
    if (fp == NULL) seterr(errbuf, errlen, "cannot open %s%s for writing", indexname, suffix);
    return fp != NULL;
  };
  // .suf: 8-byte suffixes (GtUword), or 4 with -suftabuint
  // (src/match/sfx-suffixgetset.c:467-481)
  // longest: the row holding suffix 0 (gt_suffixsortspace_setdirect,
  // src/match/sfx-suffixgetset.c:246-250), found while the rows stream out
  if (!open(".suf", "wb")) return -1;
  {
    std::vector<uint64_t> s(8u << 20);
    std::vector<uint32_t> s32(s.size());
    for (uint64_t off = 0; off < m; off += s.size()) {
      const uint64_t k = std::min<uint64_t>(s.size(), m - off);
      if (hipMemcpy(s.data(), e->suftab_dev + off, sizeof (uint64_t) * k, hipMemcpyDeviceToHost) !=
          hipSuccess)
        goto ioerr;
      for (uint64_t i = 0; i < k; i++)
        if (s[i] == 0) longest = off + i;
      if (suftab_bytes == 8) {
        if (fwrite(s.data(), sizeof (uint64_t), k, fp) != k) goto ioerr;
      } else {
        for (uint64_t i = 0; i < k; i++) s32[i] = (uint32_t) s[i];
        if (fwrite(s32.data(), sizeof (uint32_t), k, fp) != k) goto ioerr;
      }
    }
  }
  if (fclose(fp) != 0) { fp = NULL; goto ioerr; }
  // .lcp bytes, .llv {position, value} pairs, .bwt bytes
  if (!open(".lcp", "wb") || !dev_to_file(fp, e->lcptab_dev, m, buf)) goto ioerr;
  if (fclose(fp) != 0) { fp = NULL; goto ioerr; }
  if (!open(".llv", "wb") || !dev_to_file(fp, e->llvtab_dev, sizeof (GtSmaxLlv) * e->numllv, buf))
    goto ioerr;
  if (fclose(fp) != 0) { fp = NULL; goto ioerr; }
  if (!open(".bwt", "wb") || !dev_to_file(fp, e->bwttab_dev, m, buf)) goto ioerr;
  if (fclose(fp) != 0) { fp = NULL; goto ioerr; }
  // .prj (src/match/sfx-outprj.c:39-120): the keys this path's readers check
  range_stats(text, n, false, sp);
  range_stats(text, n, true, wc);
  if (!open(".prj", "w")) return -1;
  fprintf(fp, "dbfile=%s %lu %lu\n", dbfile, (unsigned long) dbfile_bytes, (unsigned long) n);
  fprintf(fp, "totallength=%lu\n", (unsigned long) n);
  fprintf(fp, "specialcharacters=%lu\n", (unsigned long) sp[0]);
  fprintf(fp, "specialranges=%lu\n", (unsigned long) sp[1]);
  fprintf(fp, "realspecialranges=%lu\n", (unsigned long) sp[1]);
  fprintf(fp, "lengthofspecialprefix=%lu\n", (unsigned long) sp[2]);
  fprintf(fp, "lengthofspecialsuffix=%lu\n", (unsigned long) sp[3]);
  fprintf(fp, "wildcards=%lu\n", (unsigned long) wc[0]);
  fprintf(fp, "wildcardranges=%lu\n", (unsigned long) wc[1]);
  fprintf(fp, "realwildcardranges=%lu\n", (unsigned long) wc[1]);
  fprintf(fp, "lengthofwildcardprefix=%lu\n", (unsigned long) wc[2]);
  fprintf(fp, "lengthofwildcardsuffix=%lu\n", (unsigned long) wc[3]);
  fprintf(fp, "numofsequences=%lu\n", (unsigned long) numseq);
  fprintf(fp, "numofdbsequences=%lu\n", (unsigned long) numseq);
  fprintf(fp, "numofquerysequences=0\n");
  fprintf(fp, "numberofallsortedsuffixes=%lu\n", (unsigned long) m);
  if (longest != UINT64_MAX) fprintf(fp, "longest=%lu\n", (unsigned long) longest);
  fprintf(fp, "prefixlength=0\n");
  fprintf(fp, "largelcpvalues=%lu\n", (unsigned long) e->numllv);
  fprintf(fp, "averagelcp=%.2f\n", e->averagelcp);
  fprintf(fp, "maxbranchdepth=%lu\n", (unsigned long) e->maxbranchdepth);
  fprintf(fp, "integersize=64\n");
  fprintf(fp, "littleendian=1\n");
  fprintf(fp, "readmode=0\n");
  fprintf(fp, "mirrored=0\n");
  if (fclose(fp) != 0) { fp = NULL; goto ioerr; }
  return 0;
ioerr:
  if (fp) fclose(fp);
  if (errbuf && errlen && !errbuf[0]) seterr(errbuf, errlen, "writing index %s failed", indexname);
  return -1;
}
