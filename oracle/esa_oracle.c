/*
 * oracle/esa_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of how GenomeTools' `gt suffixerator -dna -suf -lcp -bwt`
 * lays out an enhanced suffix array, used as the CHECKER for the product's
 * GPU ESA builder and as the input producer for parity tests.  Nothing under
 * genometools_smax_amd/ links, imports or executes this file; only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may.
 *
 * Reference behaviour restated (paths relative to the GenomeTools tree):
 *   - DNA symbol map: a/A->0 c/C->1 g/G->2 t/T/u/U->3, the IUPAC wildcards
 *     "nsywrkvbdhmNSYWRKVBDHM" -> WILDCARD (254)   src/core/alphabet.c:63,440-465
 *   - sequences joined by SEPARATOR (255)          src/core/chardef.h:34-40
 *   - suffix order: special characters (WILDCARD, SEPARATOR, end of text)
 *     compare as unique symbols ranked by position, above every base;
 *     suffixes starting at special positions therefore come last, in
 *     position order, and suftab[n] = n                  
 *   - .suf: GtUword (8 B) per suffix, 4 B with -suftabuint
 *                                                 src/match/sfx-suffixgetset.c:467-481
 *   - .lcp: one byte per suffix, lcp >= 255 stored as 255 plus a
 *     {position,value} GtUword pair in .llv           src/match/sfx-lcpvalues.c:371-433
 *     the tail of special suffixes has lcp 0          src/match/sfx-lcpvalues.c:435-470
 *   - .bwt: 254 (UNDEFBWTCHAR) for suftab[k]==0, else the encoded char at
 *     suftab[k]-1                                      src/match/sfx-run.c:174-212
 *   - .prj keys                                        src/match/sfx-outprj.c:39-80
 *
 * The sort is a plain comparison sort over the restated order (qsort): it is
 * meant to be obviously right, not fast; the tests only feed it inputs up to
 * a few Mbp.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define ORC_WILDCARD 254
#define ORC_SEPARATOR 255

typedef struct { uint64_t position, value; } OrcLlv;

/* ------------------------------------------------------------------ FASTA */

static int dna_code(unsigned char c)
{
  switch (c) {
    case 'a': case 'A': return 0;
    case 'c': case 'C': return 1;
    case 'g': case 'G': return 2;
    case 't': case 'T': case 'u': case 'U': return 3;
    default: break;
  }
  if (strchr("nsywrkvbdhmNSYWRKVBDHM", c) != NULL && c != '\0')
    return ORC_WILDCARD;
  return -1;
}

/* Encodes a (multi-)FASTA buffer.  out must hold >= len bytes.  Returns 0 or
 * -1 on an illegal symbol.  Sequence k>0 is preceded by one SEPARATOR. */
int orc_encode_fasta(const char *buf, uint64_t len, uint8_t *out,
                     uint64_t *n_out, uint64_t *numseq_out)
{
  uint64_t i = 0, n = 0, numseq = 0;
  int inheader = 0, atlinestart = 1;
  for (i = 0; i < len; i++) {
    unsigned char c = (unsigned char) buf[i];
    if (c == '\n') { inheader = 0; atlinestart = 1; continue; }
    if (inheader) continue;
    if (atlinestart && c == '>') {
      if (numseq > 0) out[n++] = ORC_SEPARATOR;
      numseq++;
      inheader = 1;
      atlinestart = 0;
      continue;
    }
    atlinestart = 0;
    if (c == ' ' || c == '\t' || c == '\r') continue;
    {
      int code = dna_code(c);
      if (code < 0) return -1;
      if (numseq == 0) numseq = 1;
      out[n++] = (uint8_t) code;
    }
  }
  *n_out = n;
  *numseq_out = numseq;
  return 0;
}

/* ------------------------------------------------------------- suffix sort */

static const uint8_t *g_text;
static uint64_t g_n;

static int is_special_at(uint64_t p)
{
  return p >= g_n || g_text[p] >= ORC_WILDCARD;
}

static int cmp_suffix(const void *va, const void *vb)
{
  uint64_t a = *(const uint64_t *) va, b = *(const uint64_t *) vb;
  for (;;) {
    int sa = is_special_at(a), sb = is_special_at(b);
    if (sa || sb) {
      if (sa && sb) return (a < b) ? -1 : (a > b);
      return sa ? 1 : -1;
    }
    if (g_text[a] != g_text[b]) return g_text[a] < g_text[b] ? -1 : 1;
    a++; b++;
  }
}

/* suftab[0..n] (n+1 suffixes incl. the virtual end suffix n). */
void orc_suffix_sort(const uint8_t *text, uint64_t n, uint64_t *suftab)
{
  uint64_t i;
  for (i = 0; i <= n; i++) suftab[i] = i;
  g_text = text;
  g_n = n;
  qsort(suftab, n + 1, sizeof (uint64_t), cmp_suffix);
}

/* Kasai et al. over the restated order: specials never match. lcp[0]=0. */
void orc_lcp_kasai(const uint8_t *text, uint64_t n, const uint64_t *suftab,
                   uint64_t *lcp)
{
  uint64_t *rank = malloc(sizeof (uint64_t) * (n + 1));
  uint64_t i, h = 0;
  for (i = 0; i <= n; i++) rank[suftab[i]] = i;
  lcp[0] = 0;
  for (i = 0; i <= n; i++) {
    uint64_t r = rank[i];
    if (r == 0) { h = 0; continue; }
    {
      uint64_t j = suftab[r - 1];
      while (i + h < n && j + h < n && text[i + h] < ORC_WILDCARD &&
             text[i + h] == text[j + h])
        h++;
      lcp[r] = h;
      if (h > 0) h--;
    }
  }
  free(rank);
}

void orc_bwt(const uint8_t *text, uint64_t n, const uint64_t *suftab,
             uint8_t *bwt)
{
  uint64_t k;
  for (k = 0; k <= n; k++)
    bwt[k] = suftab[k] == 0 ? (uint8_t) ORC_WILDCARD : text[suftab[k] - 1];
}

/* ------------------------------------------------------------ statistics */

typedef struct {
  uint64_t totallength, specialcharacters, specialranges,
           lengthofspecialprefix, lengthofspecialsuffix, wildcards,
           wildcardranges, lengthofwildcardprefix, lengthofwildcardsuffix,
           numofsequences, largelcpvalues, maxbranchdepth;
  double averagelcp;
} OrcPrj;

static void range_stats(const uint8_t *text, uint64_t n, int wildonly,
                        uint64_t *count, uint64_t *ranges, uint64_t *prefix,
                        uint64_t *suffix)
{
  uint64_t i, c = 0, r = 0, pre = 0, suf = 0;
  int prev = 0;
  for (i = 0; i < n; i++) {
    int s = wildonly ? text[i] == ORC_WILDCARD : text[i] >= ORC_WILDCARD;
    if (s) { c++; if (!prev) r++; }
    prev = s;
  }
  for (i = 0; i < n; i++) {
    int s = wildonly ? text[i] == ORC_WILDCARD : text[i] >= ORC_WILDCARD;
    if (!s) break;
    pre++;
  }
  for (i = n; i > 0; i--) {
    int s = wildonly ? text[i - 1] == ORC_WILDCARD
                     : text[i - 1] >= ORC_WILDCARD;
    if (!s) break;
    suf++;
  }
  *count = c; *ranges = r; *prefix = pre; *suffix = suf;
}

void orc_prj_stats(const uint8_t *text, uint64_t n, uint64_t numseq,
                   const uint64_t *lcp, OrcPrj *prj)
{
  uint64_t k, large = 0, maxd = 0;
  double sum = 0.0;
  memset(prj, 0, sizeof *prj);
  prj->totallength = n;
  prj->numofsequences = numseq;
  range_stats(text, n, 0, &prj->specialcharacters, &prj->specialranges,
              &prj->lengthofspecialprefix, &prj->lengthofspecialsuffix);
  range_stats(text, n, 1, &prj->wildcards, &prj->wildcardranges,
              &prj->lengthofwildcardprefix, &prj->lengthofwildcardsuffix);
  if (lcp != NULL) {
    for (k = 0; k <= n; k++) {
      if (lcp[k] >= 255) large++;
      if (lcp[k] > maxd) maxd = lcp[k];
      sum += (double) lcp[k];
    }
    prj->largelcpvalues = large;
    prj->maxbranchdepth = maxd;
    prj->averagelcp = sum / (double) (n + 1);
  }
}

/* ------------------------------------------------------------ whole index */

/* Builds the full index in memory.  Caller frees with free(). */
int orc_build_esa(const uint8_t *text, uint64_t n, uint64_t **suftab_out,
                  uint64_t **lcp_out, uint8_t **lcpbytes_out,
                  OrcLlv **llv_out, uint64_t *numllv_out, uint8_t **bwt_out)
{
  uint64_t *suftab = malloc(sizeof (uint64_t) * (n + 1));
  uint64_t *lcp = malloc(sizeof (uint64_t) * (n + 1));
  uint8_t *lcpbytes = malloc(n + 1);
  uint8_t *bwt = malloc(n + 1);
  OrcLlv *llv;
  uint64_t k, numllv = 0;
  if (!suftab || !lcp || !lcpbytes || !bwt) return -1;
  orc_suffix_sort(text, n, suftab);
  orc_lcp_kasai(text, n, suftab, lcp);
  orc_bwt(text, n, suftab, bwt);
  for (k = 0; k <= n; k++) if (lcp[k] >= 255) numllv++;
  llv = malloc(sizeof (OrcLlv) * (numllv ? numllv : 1));
  numllv = 0;
  for (k = 0; k <= n; k++) {
    if (lcp[k] >= 255) {
      lcpbytes[k] = 255;
      llv[numllv].position = k;
      llv[numllv].value = lcp[k];
      numllv++;
    } else {
      lcpbytes[k] = (uint8_t) lcp[k];
    }
  }
  *suftab_out = suftab; *lcp_out = lcp; *lcpbytes_out = lcpbytes;
  *llv_out = llv; *numllv_out = numllv; *bwt_out = bwt;
  return 0;
}

void orc_free(void *p) { free(p); }

static int write_file(const char *base, const char *suffix, const void *data,
                      size_t bytes)
{
  char path[4096];
  FILE *fp;
  snprintf(path, sizeof path, "%s%s", base, suffix);
  fp = fopen(path, "wb");
  if (fp == NULL) return -1;
  if (bytes > 0 && fwrite(data, 1, bytes, fp) != bytes) { fclose(fp); return -1; }
  return fclose(fp) == 0 ? 0 : -1;
}

/* Indexes a FASTA file and writes indexname.{suf,lcp,llv,bwt,prj}.
 * suftab_bytes: 8 (default) or 4 (-suftabuint). */
int orc_index_fasta(const char *fastapath, const char *indexname,
                    int suftab_bytes)
{
  FILE *fp = fopen(fastapath, "rb");
  char *buf;
  long len;
  uint8_t *text, *lcpbytes, *bwt;
  uint64_t n, numseq, *suftab, *lcp, numllv, k;
  OrcLlv *llv;
  OrcPrj prj;
  int rc = 0;
  if (fp == NULL) return -1;
  fseek(fp, 0, SEEK_END);
  len = ftell(fp);
  fseek(fp, 0, SEEK_SET);
  buf = malloc((size_t) len + 1);
  if (fread(buf, 1, (size_t) len, fp) != (size_t) len) { fclose(fp); return -1; }
  fclose(fp);
  text = malloc((size_t) len + 1);
  if (orc_encode_fasta(buf, (uint64_t) len, text, &n, &numseq) != 0) return -2;
  free(buf);
  if (orc_build_esa(text, n, &suftab, &lcp, &lcpbytes, &llv, &numllv, &bwt))
    return -3;
  if (suftab_bytes == 4) {
    uint32_t *s32 = malloc(sizeof (uint32_t) * (n + 1));
    for (k = 0; k <= n; k++) s32[k] = (uint32_t) suftab[k];
    rc |= write_file(indexname, ".suf", s32, sizeof (uint32_t) * (n + 1));
    free(s32);
  } else {
    rc |= write_file(indexname, ".suf", suftab, sizeof (uint64_t) * (n + 1));
  }
  rc |= write_file(indexname, ".lcp", lcpbytes, n + 1);
  rc |= write_file(indexname, ".llv", llv, sizeof (OrcLlv) * numllv);
  rc |= write_file(indexname, ".bwt", bwt, n + 1);
  orc_prj_stats(text, n, numseq, lcp, &prj);
  {
    char path[4096];
    snprintf(path, sizeof path, "%s.prj", indexname);
    fp = fopen(path, "w");
    if (fp == NULL) return -4;
    fprintf(fp, "dbfile=%s %ld %lu\n", fastapath, len, (unsigned long) n);
    fprintf(fp, "totallength=%lu\n", (unsigned long) n);
    fprintf(fp, "specialcharacters=%lu\n", (unsigned long) prj.specialcharacters);
    fprintf(fp, "specialranges=%lu\n", (unsigned long) prj.specialranges);
    fprintf(fp, "realspecialranges=%lu\n", (unsigned long) prj.specialranges);
    fprintf(fp, "lengthofspecialprefix=%lu\n", (unsigned long) prj.lengthofspecialprefix);
    fprintf(fp, "lengthofspecialsuffix=%lu\n", (unsigned long) prj.lengthofspecialsuffix);
    fprintf(fp, "wildcards=%lu\n", (unsigned long) prj.wildcards);
    fprintf(fp, "wildcardranges=%lu\n", (unsigned long) prj.wildcardranges);
    fprintf(fp, "realwildcardranges=%lu\n", (unsigned long) prj.wildcardranges);
    fprintf(fp, "lengthofwildcardprefix=%lu\n", (unsigned long) prj.lengthofwildcardprefix);
    fprintf(fp, "lengthofwildcardsuffix=%lu\n", (unsigned long) prj.lengthofwildcardsuffix);
    fprintf(fp, "numofsequences=%lu\n", (unsigned long) numseq);
    fprintf(fp, "numofdbsequences=%lu\n", (unsigned long) numseq);
    fprintf(fp, "numofquerysequences=0\n");
    fprintf(fp, "numberofallsortedsuffixes=%lu\n", (unsigned long) (n + 1));
    /* longest: the row of suffix 0 (src/match/sfx-outprj.c:70-73 writes it
     * whenever .suf is written; src/match/sfx-suffixgetset.c:246-250) */
    for (k = 0; k <= n; k++)
      if (suftab[k] == 0) {
        fprintf(fp, "longest=%lu\n", (unsigned long) k);
        break;
      }
    fprintf(fp, "prefixlength=0\n");
    fprintf(fp, "largelcpvalues=%lu\n", (unsigned long) numllv);
    fprintf(fp, "averagelcp=%.2f\n", prj.averagelcp);
    fprintf(fp, "maxbranchdepth=%lu\n", (unsigned long) prj.maxbranchdepth);
    fprintf(fp, "integersize=64\n");
    fprintf(fp, "littleendian=1\n");
    fprintf(fp, "readmode=0\n");
    fprintf(fp, "mirrored=0\n");
    fclose(fp);
  }
  free(text); free(suftab); free(lcp); free(lcpbytes); free(llv); free(bwt);
  return rc;
}
