/* esa_reader.c -- see esa_reader.h. */
#include "esa_reader.h"

#include <errno.h>
#include <fcntl.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

static void seterr(char *errbuf, size_t errlen, const char *fmt, ...)
{
  va_list ap;
  if (errbuf == NULL || errlen == 0) return;
  va_start(ap, fmt);
  vsnprintf(errbuf, errlen, fmt, ap);
  va_end(ap);
}

static int parse_prj(SmaxEsa *esa, const char *indexname, char *errbuf,
                     size_t errlen)
{
  char path[4096], line[4096];
  FILE *fp;
  int have_total = 0, have_spec = 0, have_int = 0, have_le = 0, have_rm = 0,
      have_mir = 0;
  snprintf(path, sizeof path, "%s.prj", indexname);
  fp = fopen(path, "r");
  if (fp == NULL) {
    seterr(errbuf, errlen, "cannot open file \"%s\": %s", path, strerror(errno));
    return -1;
  }
  while (fgets(line, sizeof line, fp) != NULL) {
    char *eq = strchr(line, '=');
    unsigned long long v;
    if (strncmp(line, "dbfile=", 7) == 0 || eq == NULL) continue;
    *eq = '\0';
    v = strtoull(eq + 1, NULL, 10);
    if (strcmp(line, "totallength") == 0) { esa->totallength = v; have_total = 1; }
    else if (strcmp(line, "specialcharacters") == 0) { esa->specialcharacters = v; have_spec = 1; }
    else if (strcmp(line, "numofsequences") == 0) { esa->numofsequences = v; esa->has_numofsequences = 1; }
    else if (strcmp(line, "largelcpvalues") == 0) { esa->largelcpvalues = v; esa->has_largelcpvalues = 1; }
    else if (strcmp(line, "integersize") == 0) { esa->integersize = (int) v; have_int = 1; }
    else if (strcmp(line, "littleendian") == 0) { esa->littleendian = (int) v; have_le = 1; }
    else if (strcmp(line, "readmode") == 0) { esa->readmode = (int) v; have_rm = 1; }
    else if (strcmp(line, "mirrored") == 0) { esa->mirrored = (int) v; have_mir = 1; }
  }
  fclose(fp);
  if (!have_total || !have_spec || !have_int || !have_le || !have_rm) {
    seterr(errbuf, errlen, "file %s: missing key in project file", path);
    return -1;
  }
  if (!have_mir) esa->mirrored = 0;
  /* checks of scanprjfileuintkeysviafileptr (src/match/esa-map.c:146-208) */
  if (esa->integersize != 32 && esa->integersize != 64) {
    seterr(errbuf, errlen, "%s contains illegal line defining the integer size", path);
    return -1;
  }
  if (esa->integersize != 64) {
    seterr(errbuf, errlen, "index was generated for %d-bit integers while this "
           "program uses 64-bit integers", esa->integersize);
    return -1;
  }
  if (esa->littleendian != 1) {
    seterr(errbuf, errlen, "computer has little endian byte order, while index "
           "was built on computer with big endian byte order");
    return -1;
  }
  if (esa->readmode > 3) {
    seterr(errbuf, errlen, "illegal readmode %d", esa->readmode);
    return -1;
  }
  if (esa->mirrored > 1) {
    seterr(errbuf, errlen, "illegal mirroring flag: only 0(=no mirroring) and 1 "
           "(=mirroring) is supported, but read %d", esa->mirrored);
    return -1;
  }
  /* smax-specific restriction (SURVEY.md §8(b) Errors) */
  if (esa->readmode != 0 || esa->mirrored != 0) {
    seterr(errbuf, errlen, "-smax requires a forward, non-mirrored index "
           "(readmode=%d, mirrored=%d)", esa->readmode, esa->mirrored);
    return -1;
  }
  if (esa->specialcharacters > esa->totallength) {
    seterr(errbuf, errlen, "%s: specialcharacters > totallength", path);
    return -1;
  }
  esa->nonspecials = esa->totallength - esa->specialcharacters;
  return 0;
}

/* maps (or reads, with scan) a table; expected size in units of `unit`;
 * unit==0 means "any multiple of 16". */
static int map_table(SmaxEsa *esa, int slot, const char *indexname,
                     const char *suffix, uint64_t expect, size_t unit,
                     int optional, const void **out, uint64_t *bytes_out,
                     char *errbuf, size_t errlen)
{
  char path[4096];
  struct stat st;
  int fd;
  void *p;
  snprintf(path, sizeof path, "%s%s", indexname, suffix);
  fd = open(path, O_RDONLY);
  if (fd < 0) {
    if (optional) { *out = NULL; *bytes_out = 0; return 0; }
    seterr(errbuf, errlen, "cannot open file \"%s\": %s", path, strerror(errno));
    return -1;
  }
  if (fstat(fd, &st) != 0) {
    close(fd);
    seterr(errbuf, errlen, "cannot stat \"%s\"", path);
    return -1;
  }
  if (unit > 0 && (uint64_t) st.st_size != expect * unit) {
    close(fd);
    seterr(errbuf, errlen, "number of mapped units (of size %zu) = %llu != %llu",
           unit, (unsigned long long) st.st_size / unit,
           (unsigned long long) expect);
    return -1;
  }
  if (st.st_size == 0) {
    close(fd);
    *out = NULL;
    *bytes_out = 0;
    return 0;
  }
  if (esa->scanned) {
    FILE *fp = fdopen(fd, "rb");
    p = malloc((size_t) st.st_size);
    if (p == NULL || fread(p, 1, (size_t) st.st_size, fp) != (size_t) st.st_size) {
      fclose(fp);
      free(p);
      seterr(errbuf, errlen, "cannot read \"%s\"", path);
      return -1;
    }
    fclose(fp);
  } else {
    p = mmap(NULL, (size_t) st.st_size, PROT_READ, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) {
      seterr(errbuf, errlen, "cannot map \"%s\": %s", path, strerror(errno));
      return -1;
    }
  }
  esa->maps[slot] = p;
  esa->mapsizes[slot] = (size_t) st.st_size;
  *out = p;
  *bytes_out = (uint64_t) st.st_size;
  return 0;
}

int smax_esa_sizes(const char *indexname, uint64_t *totallength, uint64_t *nonspecials,
                   char *errbuf, size_t errlen)
{
  SmaxEsa esa;
  memset(&esa, 0, sizeof esa);
  if (parse_prj(&esa, indexname, errbuf, errlen) != 0) return -1;
  *totallength = esa.totallength;
  *nonspecials = esa.totallength - esa.specialcharacters;
  return 0;
}

int smax_esa_open(SmaxEsa *esa, const char *indexname, int need_suftab,
                  int scanfile, char *errbuf, size_t errlen)
{
  return smax_esa_open_tables(esa, indexname, need_suftab, 1, scanfile, errbuf, errlen);
}

int smax_esa_open_tables(SmaxEsa *esa, const char *indexname, int need_suftab,
                         int need_bwt, int scanfile, char *errbuf, size_t errlen)
{
  const void *p;
  uint64_t bytes, n;
  memset(esa, 0, sizeof *esa);
  esa->scanned = scanfile;
  if (parse_prj(esa, indexname, errbuf, errlen) != 0) return -1;
  n = esa->totallength;
  if (map_table(esa, 0, indexname, ".lcp", n + 1, 1, 0, &p, &bytes, errbuf, errlen))
    goto fail;
  esa->lcptab = p;
  if (need_bwt) {
    if (map_table(esa, 1, indexname, ".bwt", n + 1, 1, 0, &p, &bytes, errbuf, errlen))
      goto fail;
    esa->bwttab = p;
  }
  if (map_table(esa, 2, indexname, ".llv", 0, 0, 1, &p, &bytes, errbuf, errlen))
    goto fail;
  if (bytes % sizeof (GtSmaxLlv) != 0) {
    seterr(errbuf, errlen, "%s.llv: size %llu is not a multiple of %zu", indexname,
           (unsigned long long) bytes, sizeof (GtSmaxLlv));
    goto fail;
  }
  esa->llvtab = p;
  esa->numllv = bytes / sizeof (GtSmaxLlv);
  if (esa->has_largelcpvalues && esa->largelcpvalues != esa->numllv) {
    seterr(errbuf, errlen, "%s.llv holds %llu entries, project file says %llu",
           indexname, (unsigned long long) esa->numllv,
           (unsigned long long) esa->largelcpvalues);
    goto fail;
  }
  if (need_suftab) {
    char path[4096];
    struct stat st;
    size_t unit = 8;
    snprintf(path, sizeof path, "%s.suf", indexname);
    if (stat(path, &st) == 0 && (uint64_t) st.st_size == 4 * (n + 1)) {
      /* 4-byte suftab (-suftabuint) is only readable with -scan
       * (src/match/esa-map.c:346-381) */
      if (!scanfile) {
        seterr(errbuf, errlen, "number of mapped units (of size 8) = %llu != %llu",
               (unsigned long long) st.st_size / 8, (unsigned long long) (n + 1));
        goto fail;
      }
      unit = 4;
    }
    if (map_table(esa, 3, indexname, ".suf", n + 1, unit, 0, &p, &bytes, errbuf, errlen))
      goto fail;
    esa->suftab = p;
    esa->suftab_bytes = (int) unit;
  }
  return 0;
fail:
  smax_esa_close(esa);
  return -1;
}

void smax_esa_close(SmaxEsa *esa)
{
  int i;
  for (i = 0; i < 4; i++) {
    if (esa->maps[i] == NULL) continue;
    if (esa->scanned) free(esa->maps[i]);
    else munmap(esa->maps[i], esa->mapsizes[i]);
    esa->maps[i] = NULL;
  }
}

uint64_t smax_esa_suffix(const SmaxEsa *esa, uint64_t idx)
{
  if (esa->suftab_bytes == 4) return ((const uint32_t *) esa->suftab)[idx];
  return ((const uint64_t *) esa->suftab)[idx];
}

void smax_esa_input(const SmaxEsa *esa, GtSmaxInput *in)
{
  in->lcptab = esa->lcptab;
  in->llvtab = esa->llvtab;
  in->numllv = esa->numllv;
  in->bwttab = esa->bwttab;
  in->suftab = esa->suftab;
  in->suftab_bytes = esa->suftab_bytes;
  in->totallength = esa->totallength;
  in->nonspecials = esa->nonspecials;
}

static int cmp_u64(const void *a, const void *b)
{
  uint64_t x = *(const uint64_t *) a, y = *(const uint64_t *) b;
  return x < y ? -1 : x > y;
}

int smax_esa_separators(const SmaxEsa *esa, uint64_t **sep, uint64_t *nsep)
{
  uint64_t k, cnt = 0, n = esa->totallength;
  uint64_t *s;
  for (k = 0; k <= n; k++) if (esa->bwttab[k] == 255) cnt++;
  s = malloc(sizeof (uint64_t) * (cnt + 1));
  if (s == NULL) return -1;
  cnt = 0;
  for (k = 0; k <= n; k++)
    if (esa->bwttab[k] == 255) s[cnt++] = smax_esa_suffix(esa, k) - 1;
  qsort(s, cnt, sizeof (uint64_t), cmp_u64);
  *sep = s;
  *nsep = cnt;
  return 0;
}
