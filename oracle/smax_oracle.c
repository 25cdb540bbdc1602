/*
 * oracle/smax_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker; never part
 * of the product path, which fails loudly without its HIP library).
 *
 * Three independent CPU derivations of the supermaximal-repeat intervals of
 * an enhanced suffix array, plus a restatement of GenomeTools' maximal-pair
 * enumerator used to pin the ESA against the reference's golden
 * testdata/repfind-8-Atinsert.txt:
 *
 *  1. orc_linsmax        -- linear plateau scan over (.lcp/.llv, .bwt): the
 *                           A10 predicate of SURVEY.md §8(a).  This is also the
 *                           single-core CPU baseline ("port") timed by bench.py.
 *  2. orc_bottomup_smax  -- the stack-based bottom-up lcp-interval traversal of
 *                           src/match/esa-bottomup.c:116-273 driving a smax
 *                           visitor (leaf-only interval + pairwise distinct left
 *                           characters, ISLEFTDIVERSE semantics of
 *                           src/match/esa-maxpairs.c:24-31).
 *  3. orc_brute_smax     -- text-level definition, no ESA at all: a string w
 *                           (>= minlen, no special symbol) occurring >= 2 times
 *                           is supermaximal iff every one-symbol right extension
 *                           wc and every left extension cw occurs at most once
 *                           (specials and text ends are unique).  Small texts.
 *
 *  orc_maxpairs          -- restates gt_esa_bottomup_maxpairs
 *                           (src/match/esa-bottomup-maxpairs.inc:136-264) with
 *                           processleafedge/processbranchingedge
 *                           (src/match/esa-maxpairs.c:181-360), including the
 *                           stack-slot reuse that hands a popped child's lists
 *                           to its new father, so the pair ORDER matches
 *                           `gt repfind`.
 *  orc_format_pair       -- gt_simpleexactselfmatchoutput + gt_querymatch_output
 *                           (src/tools/gt_repfind.c:49-84,
 *                           src/match/querymatch.c:130-190).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct { uint64_t position, value; } OrcLlv;

/* ----------------------------------------------------------- LCP decoding */

/* Sequential decode as SSAR_NEXTSEQUENTIALLCPTABVALUE does
 * (src/match/esa-seqread.h:104-157): byte 255 consumes the next .llv entry. */
int orc_decode_lcp(const uint8_t *lcpbytes, uint64_t count, const OrcLlv *llv,
                   uint64_t numllv, uint64_t *out)
{
  uint64_t k, li = 0;
  for (k = 0; k < count; k++) {
    if (lcpbytes[k] < 255) {
      out[k] = lcpbytes[k];
    } else {
      if (li >= numllv || llv[li].position != k) return -1;
      out[k] = llv[li++].value;
    }
  }
  return 0;
}

/* ----------------------------------------------------- diversity helper */

typedef struct { uint64_t w[4]; } Seen;

/* returns 1 if c (<254) was already seen; B >= 254 counts as unique */
static int seen_add(Seen *s, uint8_t c)
{
  uint64_t bit;
  if (c >= 254) return 0;
  bit = (uint64_t) 1 << (c & 63);
  if (s->w[c >> 6] & bit) return 1;
  s->w[c >> 6] |= bit;
  return 0;
}

static int leftdiverse(const uint8_t *bwt, uint64_t lb, uint64_t rb)
{
  Seen s;
  uint64_t k;
  memset(&s, 0, sizeof s);
  for (k = lb; k <= rb; k++)
    if (seen_add(&s, bwt[k])) return 0;
  return 1;
}

/* --------------------------------------------------------- 1. linsmax */

/* L[k] = lcp(S[k-1],S[k]) for 1<=k<=N-1, L[0]=L[N]=0.
 * out: triples (lcp, lb, rb) in ascending lb, at most cap of them; returns the
 * total number found (may exceed cap). */
/* Scan of the plateaus whose first row k (= lb+1) lies in [kbeg, kend);
 * a plateau starting before kend is followed past it.  prev must be L[kbeg-1]
 * and li any .llv index not beyond the first entry at position >= kbeg. */
typedef struct { uint64_t *buf, n, cap; int grow; } OrcOut;

static void orc_out_put(OrcOut *o, uint64_t l, uint64_t lb, uint64_t rb)
{
  if (o->n >= o->cap) {
    if (!o->grow) { o->n++; return; }
    o->cap = o->cap ? 2 * o->cap : 4096;
    o->buf = realloc(o->buf, 3 * sizeof (uint64_t) * o->cap);
  }
  o->buf[3 * o->n] = l;
  o->buf[3 * o->n + 1] = lb;
  o->buf[3 * o->n + 2] = rb;
  o->n++;
}

static void orc_linsmax_range(const uint8_t *lcpbytes, const OrcLlv *llv,
                              uint64_t numllv, const uint8_t *bwt, uint64_t N,
                              uint64_t minlen, uint64_t kbeg, uint64_t kend,
                              uint64_t prev, uint64_t li, OrcOut *o)
{
  uint64_t k;
#define ORC_L(IDX, VAR)                                                       \
  do {                                                                        \
    uint64_t ix_ = (IDX);                                                     \
    if (ix_ == 0 || ix_ >= N) { VAR = 0; }                                    \
    else if (lcpbytes[ix_] < 255) { VAR = lcpbytes[ix_]; }                    \
    else { while (li < numllv && llv[li].position < ix_) li++;                \
           VAR = llv[li].value; }                                             \
  } while (0)
  k = kbeg;
  while (k < kend) {
    uint64_t l, j, next;
    ORC_L(k, l);
    if (l > prev && l >= minlen) {
      j = k;
      for (;;) {
        if (j + 1 > N - 1) { next = 0; break; }
        ORC_L(j + 1, next);
        if (next != l) break;
        j++;
      }
      if (next < l && leftdiverse(bwt, k - 1, j))
        orc_out_put(o, l, k - 1, j);
      /* position j+1 starts a new comparison against L[j] == l */
      prev = l;
      k = j + 1;
      continue;
    }
    prev = l;
    k++;
  }
#undef ORC_L
}

/* L[k] = lcp(S[k-1],S[k]) for 1<=k<=N-1, L[0]=L[N]=0.
 * out: triples (lcp, lb, rb) in ascending lb, at most cap of them; returns the
 * total number found (may exceed cap). */
uint64_t orc_linsmax(const uint8_t *lcpbytes, const OrcLlv *llv,
                     uint64_t numllv, const uint8_t *bwt, uint64_t nonspecials,
                     uint64_t minlen, uint64_t *out, uint64_t cap)
{
  OrcOut o = {out, 0, cap, 0};
  if (nonspecials < 2) return 0;
  orc_linsmax_range(lcpbytes, llv, numllv, bwt, nonspecials, minlen,
                    1, nonspecials, 0, 0, &o);
  return o.n;
}

/* All-core form of orc_linsmax (the CPU baseline's multi-thread figure,
 * SURVEY.md §8(d)): rows split in equal ranges, one pthread each; a plateau
 * belongs to the range holding its first row (the GPU's shard rule) and is
 * followed past the range end.  Output identical to orc_linsmax. */
typedef struct {
  const uint8_t *lcpbytes, *bwt; const OrcLlv *llv;
  uint64_t numllv, N, minlen, kbeg, kend;
  OrcOut o;
} OrcTask;

static uint64_t orc_llv_lower(const OrcLlv *llv, uint64_t numllv, uint64_t pos)
{
  uint64_t lo = 0, hi = numllv;
  while (lo < hi) {
    uint64_t mid = lo + (hi - lo) / 2;
    if (llv[mid].position < pos) lo = mid + 1; else hi = mid;
  }
  return lo;
}

static void *orc_linsmax_task(void *arg)
{
  OrcTask *t = arg;
  uint64_t prev = 0, li = orc_llv_lower(t->llv, t->numllv, t->kbeg - 1);
  if (t->kbeg > 1 && t->kbeg - 1 < t->N) {
    uint8_t b = t->lcpbytes[t->kbeg - 1];
    prev = b < 255 ? b : t->llv[li].value;
  }
  orc_linsmax_range(t->lcpbytes, t->llv, t->numllv, t->bwt, t->N, t->minlen,
                    t->kbeg, t->kend, prev, li, &t->o);
  return NULL;
}

uint64_t orc_linsmax_mt(const uint8_t *lcpbytes, const OrcLlv *llv,
                        uint64_t numllv, const uint8_t *bwt, uint64_t nonspecials,
                        uint64_t minlen, uint64_t *out, uint64_t cap, int threads)
{
  OrcTask *t;
  pthread_t *tid;
  uint64_t N = nonspecials, total = 0, w = 0;
  int i;
  if (N < 2) return 0;
  if (threads < 1) threads = 1;
  t = calloc((size_t) threads, sizeof *t);
  tid = calloc((size_t) threads, sizeof *tid);
  for (i = 0; i < threads; i++) {
    t[i].lcpbytes = lcpbytes; t[i].bwt = bwt; t[i].llv = llv;
    t[i].numllv = numllv; t[i].N = N; t[i].minlen = minlen;
    t[i].kbeg = 1 + (N - 1) * (uint64_t) i / (uint64_t) threads;
    t[i].kend = 1 + (N - 1) * (uint64_t) (i + 1) / (uint64_t) threads;
    t[i].o.grow = 1;
    pthread_create(&tid[i], NULL, orc_linsmax_task, &t[i]);
  }
  for (i = 0; i < threads; i++) {
    pthread_join(tid[i], NULL);
    total += t[i].o.n;
  }
  for (i = 0; i < threads; i++) {
    uint64_t m = t[i].o.n;
    if (w < cap) {
      uint64_t c = m < cap - w ? m : cap - w;
      memcpy(out + 3 * w, t[i].o.buf, 3 * sizeof (uint64_t) * c);
    }
    w += m;
    free(t[i].o.buf);
  }
  free(t);
  free(tid);
  return total;
}

/* --------------------------------------------- 2. bottom-up smax visitor */

typedef struct {
  uint64_t lcp, lb, rb;
  int has_branch;   /* a branching edge ends here: not a local maximum */
  int dup;          /* two leaves with the same left character < 254 */
  Seen seen;
} BUItv;

typedef struct {
  BUItv *space;
  uint64_t next, alloc;
} BUStack;

static void bu_push(BUStack *st, uint64_t lcp, uint64_t lb)
{
  if (st->next >= st->alloc) {
    uint64_t na = st->alloc + 32;
    st->space = realloc(st->space, sizeof (BUItv) * na);
    memset(st->space + st->alloc, 0, sizeof (BUItv) * 32);
    st->alloc = na;
  }
  st->space[st->next].lcp = lcp;
  st->space[st->next].lb = lb;
  st->space[st->next].rb = UINT64_MAX;
  st->next++;
}

#define BU_TOP(st) ((st)->space[(st)->next - 1])

static uint8_t leftchar_of(const uint8_t *text, uint64_t pos)
{
  return pos == 0 ? (uint8_t) 254 : text[pos - 1];
}

static void smax_leaf(BUItv *f, int firstsucc, uint8_t lc)
{
  if (firstsucc) {
    f->has_branch = 0; f->dup = 0; memset(&f->seen, 0, sizeof f->seen);
  }
  if (seen_add(&f->seen, lc)) f->dup = 1;
}

static void smax_branch(BUItv *f, int firstsucc)
{
  /* any interval child disqualifies the father as a local maximum; with
   * firstsucc the father reuses the child's slot, so reset it. */
  if (firstsucc) {
    f->dup = 0; memset(&f->seen, 0, sizeof f->seen);
  }
  f->has_branch = 1;
}

/* Traversal as in gt_esa_bottomup (src/match/esa-bottomup.c:116-273), over
 * either
 *  - lcp: decoded (lcp[idx+1] read at step idx), left characters from the
 *    text through the suffix array (suftab, text), or
 *  - the mapped tables as the sequential reader hands them out
 *    (SSAR_NEXTSEQUENTIALLCPTABVALUE, src/match/esa-seqread.h:104-157: a
 *    255 byte takes the next .llv value), left characters from the .bwt
 *    (text[suftab[idx]-1], 254 for suffix 0 -- the same symbols).
 * The steps run over rows [0, rows) (rows = N: the whole index); the value
 * after the last row is taken as 0 (LCP[N] == 0 on file-based indexes). */
static uint64_t bu_smax_core(const uint64_t *lcp, const uint64_t *suftab,
                             const uint8_t *text, const uint8_t *lcpbytes,
                             const OrcLlv *llv, uint64_t numllv,
                             const uint8_t *bwt, uint64_t rows,
                             uint64_t minlen, uint64_t *out, uint64_t cap)
{
  BUStack st = {NULL, 0, 0};
  BUItv *last = NULL;
  BUItv lastcopy;
  uint64_t idx, found = 0, li = 0;
  const uint64_t nonspecials = rows;
  int firstedgefromroot = 1;
  if (lcpbytes != NULL && rows > 0 && lcpbytes[0] == 255) li = 1;
#define EMIT(I)                                                              \
  do {                                                                       \
    if ((I)->lcp >= minlen && !(I)->has_branch && !(I)->dup) {               \
      if (found < cap) { out[3*found] = (I)->lcp; out[3*found+1] = (I)->lb;  \
                         out[3*found+2] = (I)->rb; }                         \
      found++;                                                               \
    }                                                                        \
  } while (0)
  bu_push(&st, 0, 0);
  for (idx = 0; idx < nonspecials; idx++) {
    uint64_t lcpvalue;
    uint8_t lc;
    int firstedge;
    if (lcp != NULL) {
      lcpvalue = lcp[idx + 1];
      lc = leftchar_of(text, suftab[idx]);
    } else {
      if (idx + 1 >= rows) lcpvalue = 0;
      else if (lcpbytes[idx + 1] < 255) lcpvalue = lcpbytes[idx + 1];
      else lcpvalue = li < numllv ? llv[li++].value : 0;
      lc = bwt[idx];
    }
    if (lcpvalue <= BU_TOP(&st).lcp) {
      if (BU_TOP(&st).lcp > 0 || !firstedgefromroot) firstedge = 0;
      else { firstedge = 1; firstedgefromroot = 0; }
      smax_leaf(&BU_TOP(&st), firstedge, lc);
    }
    last = NULL;
    while (lcpvalue < BU_TOP(&st).lcp) {
      st.next--;
      lastcopy = st.space[st.next];
      last = &lastcopy;
      last->rb = idx;
      EMIT(last);
      if (lcpvalue <= BU_TOP(&st).lcp) {
        if (BU_TOP(&st).lcp > 0 || !firstedgefromroot) firstedge = 0;
        else { firstedge = 1; firstedgefromroot = 0; }
        smax_branch(&BU_TOP(&st), firstedge);
        last = NULL;
      }
    }
    if (lcpvalue > BU_TOP(&st).lcp) {
      if (last != NULL) {
        bu_push(&st, lcpvalue, last->lb);
        smax_branch(&BU_TOP(&st), 1);
        last = NULL;
      } else {
        bu_push(&st, lcpvalue, idx);
        smax_leaf(&BU_TOP(&st), 1, lc);
      }
    }
  }
  if (BU_TOP(&st).lcp > 0) {
    /* never reached on file-based indexes: LCP[N] == 0 */
    BU_TOP(&st).rb = idx;
    EMIT(&BU_TOP(&st));
  }
  free(st.space);
#undef EMIT
  return found;
}

uint64_t orc_bottomup_smax(const uint64_t *lcp, const uint64_t *suftab,
                           const uint8_t *text, uint64_t nonspecials,
                           uint64_t minlen, uint64_t *out, uint64_t cap)
{
  return bu_smax_core(lcp, suftab, text, NULL, NULL, 0, NULL, nonspecials,
                      minlen, out, cap);
}

/* The same traversal over the mapped .lcp/.llv/.bwt tables, rows [0, rows):
 * bench.py's reference-algorithm CPU anchor (the stack walk the GPU path
 * replaces) and, with rows = N, a fourth derivation of the smax list. */
uint64_t orc_bottomup_smax_tables(const uint8_t *lcpbytes, const OrcLlv *llv,
                                  uint64_t numllv, const uint8_t *bwt,
                                  uint64_t rows, uint64_t minlen,
                                  uint64_t *out, uint64_t cap)
{
  return bu_smax_core(NULL, NULL, NULL, lcpbytes, llv, numllv, bwt, rows,
                      minlen, out, cap);
}

/* Full event stream of gt_esa_bottomup (src/match/esa-bottomup.c:116-273)
 * for a visitor with all three callbacks, as 7-word records:
 *   (0, firstsucc, fd, flb, leafnumber, 0, 0)       visit_leaf_edge
 *   (1, firstsucc, fd, flb, sd, slb, srb)           visit_branching_edge
 *   (2, 0, lcp, lb, rb, 0, 0)                       visit_lcp_interval
 * (F3 checker).  Returns the number of events; *ev is malloc'd. */
/* With slots != NULL also the stack slot of each event's interval(s) -- the
 * reference binds one GtESAVisitorInfo to each slot (esa-bottomup.c:20-110):
 * per event (father slot, son slot) for edges, (popped slot, -) for
 * lcp-intervals, NONE (UINT64_MAX) where there is no son info (a leaf, or a
 * father pushed into its first child's slot); *nslots = slots allocated
 * (32 at a time, as allocateBUstack). */
static uint64_t bu_events(const uint64_t *lcp, const uint64_t *suftab,
                          uint64_t nonspecials, uint64_t **ev, uint64_t **slots,
                          uint64_t *nslots)
{
  BUStack st = {NULL, 0, 0};
  BUItv *last = NULL;
  BUItv lastcopy;
  uint64_t idx, n = 0, alloc = 0, *e = NULL, *sl = NULL, lastslot = 0;
  const uint64_t NONE = UINT64_MAX;
  int firstedgefromroot = 1;
#define EVS(T, F, A, B, C, D, E, S0, S1)                                     \
  do {                                                                       \
    if (n + 1 > alloc) {                                                     \
      alloc = alloc * 2 + 1024;                                              \
      e = realloc(e, sizeof (uint64_t) * 7 * alloc);                         \
      if (slots) sl = realloc(sl, sizeof (uint64_t) * 2 * alloc);            \
    }                                                                        \
    if (slots) { sl[2 * n] = (S0); sl[2 * n + 1] = (S1); }                   \
    uint64_t *r_ = e + 7 * n++;                                              \
    r_[0] = (T); r_[1] = (F); r_[2] = (A); r_[3] = (B); r_[4] = (C);          \
    r_[5] = (D); r_[6] = (E);                                                \
  } while (0)
#define EV(T, F, A, B, C, D, E) EVS(T, F, A, B, C, D, E, NONE, NONE)
#define FIRSTEDGE(F)                                                         \
  do {                                                                       \
    if (BU_TOP(&st).lcp > 0 || !firstedgefromroot) (F) = 0;                  \
    else { (F) = 1; firstedgefromroot = 0; }                                 \
  } while (0)
  bu_push(&st, 0, 0);
  for (idx = 0; idx < nonspecials; idx++) {
    uint64_t lcpvalue = lcp[idx + 1];
    uint64_t prevsuffix = suftab[idx];
    int firstedge;
    if (lcpvalue <= BU_TOP(&st).lcp) {
      FIRSTEDGE(firstedge);
      EVS(0, firstedge, BU_TOP(&st).lcp, BU_TOP(&st).lb, prevsuffix, 0, 0, st.next - 1, NONE);
    }
    last = NULL;
    while (lcpvalue < BU_TOP(&st).lcp) {
      st.next--;
      lastcopy = st.space[st.next];
      last = &lastcopy;
      last->rb = idx;
      lastslot = st.next;
      EVS(2, 0, last->lcp, last->lb, last->rb, 0, 0, lastslot, NONE);
      if (lcpvalue <= BU_TOP(&st).lcp) {
        FIRSTEDGE(firstedge);
        EVS(1, firstedge, BU_TOP(&st).lcp, BU_TOP(&st).lb, last->lcp, last->lb, last->rb,
            st.next - 1, lastslot);
        last = NULL;
      }
    }
    if (lcpvalue > BU_TOP(&st).lcp) {
      if (last != NULL) {
        uint64_t l = last->lcp, b = last->lb, r = last->rb;
        bu_push(&st, lcpvalue, b);
        EVS(1, 1, BU_TOP(&st).lcp, BU_TOP(&st).lb, l, b, r, st.next - 1, NONE);
        last = NULL;
      } else {
        bu_push(&st, lcpvalue, idx);
        EVS(0, 1, BU_TOP(&st).lcp, BU_TOP(&st).lb, prevsuffix, 0, 0, st.next - 1, NONE);
      }
    }
  }
  if (nslots) *nslots = st.alloc;
  free(st.space);
#undef EV
#undef EVS
#undef FIRSTEDGE
  *ev = e;
  if (slots) *slots = sl;
  return n;
}

uint64_t orc_bottomup_events(const uint64_t *lcp, const uint64_t *suftab,
                             uint64_t nonspecials, uint64_t **ev)
{
  return bu_events(lcp, suftab, nonspecials, ev, NULL, NULL);
}

/* orc_bottomup_events plus the stack slot (GtESAVisitorInfo) of each event,
 * 2 words per event in *slots (malloc'd), and the number of slots allocated
 * (F3's info-visitor checker). */
uint64_t orc_bottomup_events_slots(const uint64_t *lcp, const uint64_t *suftab,
                                   uint64_t nonspecials, uint64_t **ev,
                                   uint64_t **slots, uint64_t *nslots)
{
  return bu_events(lcp, suftab, nonspecials, ev, slots, nslots);
}

/* The other traversal gt dev sfxmap has: -enumlcpitvtree, the depth-first
 * enumeration gt_depthfirstesa (src/match/esa-dfs.c:90-271) with the elcp
 * callbacks of src/match/esa-lcpintervals.c:44-130.  Its L/B lines must
 * equal those of -enumlcpitvtreeBU (gt_esa_bottomup + the lcpitvs visitor):
 * the reference's own test diffs the two (testsuite/gt_suffixerator_include.rb:
 * 597-603), which pins orc_bottomup_events, and through it the GPU event
 * stream, to a second reference algorithm.  Records as orc_bottomup_events
 * without the lcp-interval events and with srb = 0:
 *   (0, firstsucc, fd, flb, leafnumber, 0, 0), (1, firstsucc, fd, flb, sd, slb, 0)
 * Stack slots keep their node info when popped and are reused by the next
 * push, as the reference's preallocated Dfsinfo slots are: a node pushed
 * right after a pop starts with the popped child's leftmost leaf. */
typedef struct {
  uint64_t depth, left, offset;
  int lastisleafedge;
} DfsItv;

uint64_t orc_dfs_events(const uint64_t *lcp, const uint64_t *suftab, uint64_t nonspecials,
                        uint64_t **ev)
{
  DfsItv *stk = NULL;
  uint64_t next = 0, alloc = 0, idx, n = 0, evalloc = 0, *e = NULL;
  uint64_t lastoffset = 0, lastleft = 0;      /* Elcpstate.lastcompletenode */
  int firstrootedge = 1;
#define DFS_EV(T, F, A, B, C, D)                                             \
  do {                                                                       \
    if (n + 1 > evalloc) {                                                   \
      evalloc = evalloc * 2 + 1024;                                          \
      e = realloc(e, sizeof (uint64_t) * 7 * evalloc);                       \
    }                                                                        \
    uint64_t *r_ = e + 7 * n++;                                              \
    r_[0] = (T); r_[1] = (F); r_[2] = (A); r_[3] = (B); r_[4] = (C);          \
    r_[5] = (D); r_[6] = 0;                                                  \
  } while (0)
#define DFS_PUSH(D, B)                                                       \
  do {                                                                       \
    if (next >= alloc) {                                                     \
      stk = realloc(stk, sizeof (DfsItv) * (alloc + 32));                    \
      memset(stk + alloc, 0, sizeof (DfsItv) * 32);                          \
      alloc += 32;                                                           \
    }                                                                        \
    stk[next].depth = (D); stk[next].lastisleafedge = (B);                   \
    next++;                                                                  \
  } while (0)
#define TOPD (stk[next - 1])
#define ABOVE (stk[next])
#define BELOW (stk[next - 2])
  DFS_PUSH(0, 1);
  TOPD.left = 0;
  for (idx = 0; idx < nonspecials; idx++) {
    uint64_t cur = lcp[idx + 1], prev = suftab[idx];
    while (cur < TOPD.depth) {
      if (TOPD.lastisleafedge)
        DFS_EV(0, 0, TOPD.depth, TOPD.left, prev, 0);
      else
        DFS_EV(1, 0, TOPD.depth, TOPD.left, ABOVE.offset, ABOVE.left);
      /* assignrightmostleaf: right = idx (unused by the lines);
         processcompletenode: offset = depth, lastcompletenode */
      TOPD.offset = TOPD.depth;
      lastoffset = TOPD.offset;
      lastleft = TOPD.left;
      next--;
    }
    if (cur == TOPD.depth) {
      int firstedge = 0;
      if (firstrootedge && TOPD.depth == 0) { firstedge = 1; firstrootedge = 0; }
      if (TOPD.lastisleafedge) {
        DFS_EV(0, firstedge, TOPD.depth, TOPD.left, prev, 0);
      } else {
        DFS_EV(1, firstedge, TOPD.depth, TOPD.left, ABOVE.offset, ABOVE.left);
        TOPD.lastisleafedge = 1;
      }
    } else {
      DFS_PUSH(cur, 1);
      if (BELOW.lastisleafedge) {
        TOPD.left = idx;
        DFS_EV(0, 1, TOPD.depth, TOPD.left, prev, 0);
        BELOW.lastisleafedge = 0;
      } else {
        /* son == NULL: the last complete node's offset and left */
        DFS_EV(1, 1, TOPD.depth, TOPD.left, lastoffset, lastleft);
      }
    }
  }
  free(stk);
#undef DFS_EV
#undef DFS_PUSH
#undef TOPD
#undef ABOVE
#undef BELOW
  *ev = e;
  return n;
}

/* --------------------------------------------------------- 3. brute force */

static int is_spec(const uint8_t *t, uint64_t n, int64_t p)
{
  return p < 0 || (uint64_t) p >= n || t[p] >= 254;
}

/* All supermaximal repeats of text[0..n) with length >= minlen.
 * out: (length, first occurrence, number of occurrences) triples sorted by
 * (first occ); occs receives all occurrence positions, ascending per repeat.
 * O(n^3); meant for n <= ~400. */
uint64_t orc_brute_smax(const uint8_t *t, uint64_t n, uint64_t minlen,
                        uint64_t *out, uint64_t cap, uint64_t *occs,
                        uint64_t occcap)
{
  uint64_t found = 0, nocc = 0, i, len;
  uint64_t *pos = malloc(sizeof (uint64_t) * (n + 1));
  for (len = minlen > 0 ? minlen : 1; len <= n; len++) {
    for (i = 0; i + len <= n; i++) {
      uint64_t j, cnt = 0, q;
      int ok = 1, firstocc = 1;
      for (q = 0; q < len; q++) if (t[i + q] >= 254) { ok = 0; break; }
      if (!ok) continue;
      /* i must be the first occurrence */
      for (j = 0; j < i && firstocc; j++)
        if (memcmp(t + j, t + i, len) == 0) firstocc = 0;
      if (!firstocc) continue;
      for (j = i; j + len <= n; j++)
        if (memcmp(t + j, t + i, len) == 0) pos[cnt++] = j;
      if (cnt < 2) continue;
      /* right extensions: pairwise distinct or special */
      {
        uint64_t a, b;
        for (a = 0; a < cnt && ok; a++)
          for (b = a + 1; b < cnt && ok; b++) {
            int64_t ra = (int64_t) (pos[a] + len), rb = (int64_t) (pos[b] + len);
            int64_t la = (int64_t) pos[a] - 1, lb = (int64_t) pos[b] - 1;
            if (!is_spec(t, n, ra) && !is_spec(t, n, rb) && t[ra] == t[rb])
              ok = 0;
            if (!is_spec(t, n, la) && !is_spec(t, n, lb) && t[la] == t[lb])
              ok = 0;
          }
      }
      if (!ok) continue;
      if (found < cap) {
        out[3 * found] = len; out[3 * found + 1] = i; out[3 * found + 2] = cnt;
      }
      for (j = 0; j < cnt; j++) { if (nocc < occcap) occs[nocc] = pos[j]; nocc++; }
      found++;
    }
  }
  free(pos);
  return found;
}

/* ------------------------------------------------------------- maxpairs */

typedef struct { uint64_t start, length; } MPList;

typedef struct {
  uint8_t commonchar;
  uint64_t ucstart, uclen;
  MPList npl[4];
} MPInfo;

typedef struct {
  uint64_t lcp, lb, rb;
  MPInfo info;
} MPItv;

typedef struct { uint64_t *space, next, alloc; } U64Arr;

static void arr_add(U64Arr *a, uint64_t v)
{
  if (a->next >= a->alloc) {
    a->alloc = a->alloc * 2 + 64;
    a->space = realloc(a->space, sizeof (uint64_t) * a->alloc);
  }
  a->space[a->next++] = v;
}

typedef struct {
  unsigned sigma, searchlength;
  int initialized;
  U64Arr uniquechar, poslist[4];
  const uint8_t *text;
  U64Arr pairs; /* len, pos1, pos2 triples in emission order */
} MPState;

#define ISLD(s) ((uint8_t) (s)->sigma)
#define INITC(s) ((uint8_t) ((s)->sigma + 1))

static void mp_emit(MPState *s, uint64_t len, uint64_t p1, uint64_t p2)
{
  arr_add(&s->pairs, len); arr_add(&s->pairs, p1); arr_add(&s->pairs, p2);
}

static void mp_add2poslist(MPState *s, MPInfo *ni, unsigned base, uint64_t leaf)
{
  if (base >= s->sigma) { ni->uclen++; arr_add(&s->uniquechar, leaf); }
  else { arr_add(&s->poslist[base], leaf); ni->npl[base].length++; }
}

static void mp_cart1(MPState *s, uint64_t depth, const MPInfo *ni,
                     unsigned base, uint64_t leaf)
{
  uint64_t k;
  const MPList *pl = &ni->npl[base];
  for (k = 0; k < pl->length; k++)
    mp_emit(s, depth, leaf, s->poslist[base].space[pl->start + k]);
}

static void mp_cart2(MPState *s, uint64_t depth, const MPInfo *n1,
                     unsigned b1, const MPInfo *n2, unsigned b2)
{
  uint64_t a, b;
  const MPList *p1 = &n1->npl[b1], *p2 = &n2->npl[b2];
  for (a = 0; a < p1->length; a++)
    for (b = 0; b < p2->length; b++)
      mp_emit(s, depth, s->poslist[b1].space[p1->start + a],
              s->poslist[b2].space[p2->start + b]);
}

static void mp_setpostabto0(MPState *s)
{
  unsigned b;
  if (!s->initialized) {
    for (b = 0; b < s->sigma; b++) s->poslist[b].next = 0;
    s->uniquechar.next = 0;
    s->initialized = 1;
  }
}

static void mp_leaf(MPState *s, int firstsucc, uint64_t depth, MPInfo *f,
                    uint64_t leaf)
{
  unsigned base;
  uint8_t lc;
  if (depth < s->searchlength) { mp_setpostabto0(s); return; }
  lc = leaf == 0 ? INITC(s) : s->text[leaf - 1];
  s->initialized = 0;
  if (firstsucc) {
    f->commonchar = lc; f->uclen = 0; f->ucstart = s->uniquechar.next;
    for (base = 0; base < s->sigma; base++) {
      f->npl[base].start = s->poslist[base].next;
      f->npl[base].length = 0;
    }
    mp_add2poslist(s, f, lc, leaf);
    return;
  }
  if (f->commonchar != ISLD(s)) {
    if (f->commonchar != lc || lc >= ISLD(s)) f->commonchar = ISLD(s);
  }
  if (f->commonchar == ISLD(s)) {
    uint64_t k;
    for (base = 0; base < s->sigma; base++)
      if (lc != (uint8_t) base) mp_cart1(s, depth, f, base, leaf);
    for (k = 0; k < f->uclen; k++)
      mp_emit(s, depth, leaf, s->uniquechar.space[f->ucstart + k]);
  }
  mp_add2poslist(s, f, lc, leaf);
}

static void mp_branch(MPState *s, int firstsucc, uint64_t depth, MPInfo *f,
                      MPInfo *son)
{
  unsigned cf, cs, base;
  uint64_t k, m;
  if (depth < s->searchlength) { mp_setpostabto0(s); return; }
  s->initialized = 0;
  if (firstsucc) return;
  if (f->commonchar != ISLD(s)) {
    if (son->commonchar != ISLD(s)) {
      if (f->commonchar != son->commonchar || son->commonchar >= ISLD(s))
        f->commonchar = ISLD(s);
    } else {
      f->commonchar = ISLD(s);
    }
  }
  if (f->commonchar == ISLD(s)) {
    for (cf = 0; cf < s->sigma; cf++) {
      for (cs = 0; cs < s->sigma; cs++)
        if (cs != cf) mp_cart2(s, depth, f, cf, son, cs);
      for (k = 0; k < son->uclen; k++)
        mp_cart1(s, depth, f, cf, s->uniquechar.space[son->ucstart + k]);
    }
    for (m = 0; m < f->uclen; m++) {
      uint64_t fp = s->uniquechar.space[f->ucstart + m];
      for (cs = 0; cs < s->sigma; cs++) mp_cart1(s, depth, son, cs, fp);
      for (k = 0; k < son->uclen; k++)
        mp_emit(s, depth, fp, s->uniquechar.space[son->ucstart + k]);
    }
  }
  for (base = 0; base < s->sigma; base++)
    f->npl[base].length += son->npl[base].length;
  f->uclen += son->uclen;
}

/* Returns number of pairs; *pairs_out (malloc'd) holds (len,pos1,pos2). */
uint64_t orc_maxpairs(const uint64_t *lcp, const uint64_t *suftab,
                      const uint8_t *text, uint64_t nonspecials,
                      unsigned minlen, uint64_t **pairs_out)
{
  MPState s;
  MPItv *stk = NULL;
  uint64_t next = 0, alloc = 0, idx;
  MPItv *last = NULL;
  int firstedgefromroot = 1;
  memset(&s, 0, sizeof s);
  s.sigma = 4; s.searchlength = minlen; s.text = text;
#define MP_TOP (stk[next - 1])
#define MP_PUSH(L, B)                                                        \
  do {                                                                       \
    if (next >= alloc) {                                                     \
      stk = realloc(stk, sizeof (MPItv) * (alloc + 32));                     \
      memset(stk + alloc, 0, sizeof (MPItv) * 32);                           \
      alloc += 32;                                                           \
    }                                                                        \
    stk[next].lcp = (L); stk[next].lb = (B); stk[next].rb = UINT64_MAX;      \
    next++;                                                                  \
  } while (0)
  MP_PUSH(0, 0);
  for (idx = 0; idx < nonspecials; idx++) {
    uint64_t lcpvalue = lcp[idx + 1], prevsuffix = suftab[idx];
    int firstedge;
    if (lcpvalue <= MP_TOP.lcp) {
      if (MP_TOP.lcp > 0 || !firstedgefromroot) firstedge = 0;
      else { firstedge = 1; firstedgefromroot = 0; }
      mp_leaf(&s, firstedge, MP_TOP.lcp, &MP_TOP.info, prevsuffix);
    }
    last = NULL;
    while (lcpvalue < MP_TOP.lcp) {
      last = &stk[--next];     /* slot stays valid: reused by a later PUSH */
      last->rb = idx;
      if (lcpvalue <= MP_TOP.lcp) {
        if (MP_TOP.lcp > 0 || !firstedgefromroot) firstedge = 0;
        else { firstedge = 1; firstedgefromroot = 0; }
        mp_branch(&s, firstedge, MP_TOP.lcp, &MP_TOP.info, &last->info);
        last = NULL;
      }
    }
    if (lcpvalue > MP_TOP.lcp) {
      if (last != NULL) {
        uint64_t llb = last->lb;
        /* PUSH writes into the popped child's slot: father inherits info */
        MP_PUSH(lcpvalue, llb);
        mp_branch(&s, 1, MP_TOP.lcp, &MP_TOP.info, NULL);
        last = NULL;
      } else {
        MP_PUSH(lcpvalue, idx);
        mp_leaf(&s, 1, MP_TOP.lcp, &MP_TOP.info, prevsuffix);
      }
    }
  }
  free(stk);
  free(s.uniquechar.space);
  {
    unsigned b;
    for (b = 0; b < 4; b++) free(s.poslist[b].space);
  }
  *pairs_out = s.pairs.space;
#undef MP_TOP
#undef MP_PUSH
  return s.pairs.next / 3;
}

/* ------------------------------------------------------- pair formatting */

/* seqnum of absolute position p given sorted separator positions */
static uint64_t seqnum_of(const uint64_t *sep, uint64_t nsep, uint64_t p)
{
  uint64_t lo = 0, hi = nsep;
  while (lo < hi) {
    uint64_t mid = (lo + hi) / 2;
    if (sep[mid] < p) lo = mid + 1; else hi = mid;
  }
  return lo;
}

/* Formats one repfind line "len seq1 rel1 F len seq2 rel2\n" into buf.
 * Returns number of chars, or 0 if filtered. */
int orc_format_pair(uint64_t len, uint64_t pos1, uint64_t pos2,
                    const uint64_t *sep, uint64_t nsep, char *buf, int bufsz)
{
  uint64_t s1, s2, st1, st2;
  if (pos1 > pos2) { uint64_t t = pos1; pos1 = pos2; pos2 = t; }
  s1 = seqnum_of(sep, nsep, pos1);
  s2 = seqnum_of(sep, nsep, pos2);
  st1 = s1 == 0 ? 0 : sep[s1 - 1] + 1;
  st2 = s2 == 0 ? 0 : sep[s2 - 1] + 1;
  if (s1 == s2 && pos1 - st1 > pos2 - st2) return 0;
  return snprintf(buf, (size_t) bufsz, "%lu %lu %lu F %lu %lu %lu\n",
                  (unsigned long) len, (unsigned long) s1,
                  (unsigned long) (pos1 - st1), (unsigned long) len,
                  (unsigned long) s2, (unsigned long) (pos2 - st2));
}

/* ------------------------------------------- checkers past 2^32 rows */

/* exact L[k] of the mapped tables (255 -> .llv by binary search) */
static uint64_t orc_lcp_at(const uint8_t *lcpbytes, const OrcLlv *llv,
                           uint64_t numllv, uint64_t k)
{
  uint64_t i;
  if (lcpbytes[k] < 255) return lcpbytes[k];
  i = orc_llv_lower(llv, numllv, k);
  return i < numllv && llv[i].position == k ? llv[i].value : 0;
}

/* Every lcp-interval of depth > 0 with its father, in the pop order of
 * gt_esa_bottomup (src/match/esa-bottomup.c:116-273): at step
 * idx the intervals deeper than L[idx+1] are popped (rb = idx); a popped
 * interval's father is the stack top if L[idx+1] <= its depth, else the
 * interval (L[idx+1], popped lb) pushed right after.  5 words per interval
 * (lcp, lb, rb, father lcp, father lb); F3's gt_lcpitv list, for tables too
 * large for orc_bottomup_events.  L[N] is taken as 0. */
uint64_t orc_lcp_intervals(const uint8_t *lcpbytes, const OrcLlv *llv,
                           uint64_t numllv, uint64_t nonspecials,
                           uint64_t *out, uint64_t cap)
{
  uint64_t *sl = NULL, *sb = NULL, top = 0, alloc = 0, idx, found = 0, li = 0;
  const uint64_t N = nonspecials;
  if (N > 0 && lcpbytes[0] == 255) li = 1;
  alloc = 1024;
  sl = malloc(sizeof (uint64_t) * alloc);
  sb = malloc(sizeof (uint64_t) * alloc);
  sl[0] = 0; sb[0] = 0; top = 1;
  for (idx = 0; idx < N; idx++) {
    uint64_t v, lastlb = 0;
    int popped = 0;
    if (idx + 1 >= N) v = 0;
    else if (lcpbytes[idx + 1] < 255) v = lcpbytes[idx + 1];
    else v = li < numllv ? llv[li++].value : 0;
    while (v < sl[top - 1]) {
      uint64_t l = sl[top - 1], b = sb[top - 1], fl, fb;
      top--;
      if (v <= sl[top - 1]) { fl = sl[top - 1]; fb = sb[top - 1]; }
      else { fl = v; fb = b; }
      if (found < cap) {
        uint64_t *w = out + 5 * found;
        w[0] = l; w[1] = b; w[2] = idx; w[3] = fl; w[4] = fb;
      }
      found++;
      lastlb = b;
      popped = 1;
    }
    if (v > sl[top - 1]) {
      if (top >= alloc) {
        alloc *= 2;
        sl = realloc(sl, sizeof (uint64_t) * alloc);
        sb = realloc(sb, sizeof (uint64_t) * alloc);
      }
      sl[top] = v;
      sb[top] = popped ? lastlb : idx;
      top++;
    }
  }
  free(sl);
  free(sb);
  return found;
}

/* Maximal pairs by their definition, block by block: rows i < j of one
 * block (a maximal run of rows k with L[k] >= minlen, plus the row before
 * it) form a pair of length min L[i+1..j] when their left symbols differ
 * (symbols >= 254 unique, ISLEFTDIVERSE, src/match/esa-maxpairs.c:24-31);
 * triples (len, min pos, max pos) in no particular order; with suftab NULL
 * the rows (len, i, j) instead.  Quadratic in the block size: for sparse
 * synthetic tables past 2^32 rows (F2 checker). */
uint64_t orc_maxpairs_blocks(const uint8_t *lcpbytes, const OrcLlv *llv,
                             uint64_t numllv, const uint8_t *bwt,
                             const uint64_t *suftab, uint64_t nonspecials,
                             uint64_t minlen, uint64_t *out, uint64_t cap)
{
  const uint64_t N = nonspecials;
  const uint8_t mf = minlen < 255 ? (uint8_t) minlen : 255;
  uint64_t k = 1, found = 0;
  while (k < N) {
    uint64_t a, b, j;
    if (lcpbytes[k] < mf || orc_lcp_at(lcpbytes, llv, numllv, k) < minlen) { k++; continue; }
    a = k;
    b = k;
    while (b + 1 < N && lcpbytes[b + 1] >= mf &&
           orc_lcp_at(lcpbytes, llv, numllv, b + 1) >= minlen)
      b++;
    for (j = a; j <= b; j++) {
      uint64_t m = UINT64_MAX, i = j;
      while (i >= a) {
        uint64_t x = orc_lcp_at(lcpbytes, llv, numllv, i);
        m = x < m ? x : m;
        i--;
        if (bwt[i] >= 254 || bwt[j] >= 254 || bwt[i] != bwt[j]) {
          if (found < cap) {
            uint64_t p = suftab ? suftab[i] : i, q = suftab ? suftab[j] : j;
            out[3 * found] = m;
            out[3 * found + 1] = p < q ? p : q;
            out[3 * found + 2] = p < q ? q : p;
          }
          found++;
        }
      }
    }
    k = b + 1;
  }
  return found;
}

/* ---------------------------------------------------- spmitvs visitor (F3)
 *
 * orc_spmitv -- the GtESAVisitor of `gt dev sfxmap -spmitv`
 * (src/match/esa_spmitvs_visitor.c:59-152, driven by gt_esa_bottomup in
 * src/match/esa-spmitvs.c:25-69) restated over a gt_esa_bottomup event
 * stream in the 7-word form of orc_bottomup_events (which the GPU's
 * gt_lcpitv_plan_events writes too):
 *   leaf edge (:59-89): leaf number 0, or one right after a separator, is a
 *     "whole leaf" (:50-57) and becomes lastwholeleaf (its leaf index, the
 *     running count of leaf edges); any other leaf whose suffix continues
 *     past the father's depth without hitting a separator (leaf + fd <
 *     totallength, text[leaf + fd] != SEPARATOR) is an unnecessary leaf;
 *   branching edge (:91-125): for every depth fd < idx < sd the child
 *     interval [slb, srb] counts as a whole-leaf one at depth idx if
 *     lastwholeleaf lies in it (lastwholeleaf >= slb), else as a no-whole-leaf
 *     one, width srb - slb + 1 either way;
 *   lcp-interval (:127-152): the same count for the interval at its own lcp.
 * counts: 4 words per depth 0..maxlen (wholeleaf, wholeleafwidth,
 * nowholeleaf, nowholeleafwidth), zeroed here.  Returns -1 where the
 * reference asserts (a depth above maxlen, lastwholeleaf past rb, a whole
 * leaf at leaf index totallength), else 0.  text: the encoded sequence
 * (255 = separator). */
int orc_spmitv(const uint64_t *ev, uint64_t nev, const uint8_t *text, uint64_t totallength,
               uint64_t maxlen, uint64_t *counts, uint64_t *unnecessary)
{
  const uint64_t undef = totallength;            /* lastwholeleaf "undefined" (:193) */
  uint64_t current = 0, lastwhole = undef, unnec = 0;
  memset(counts, 0, sizeof (uint64_t) * 4 * (maxlen + 1));
  for (uint64_t k = 0; k < nev; k++) {
    const uint64_t *r = ev + 7 * k;
    if (r[0] == 0) {
      const uint64_t fd = r[2], leaf = r[4];
      if (leaf == 0 || text[leaf - 1] == 255) {
        if (current == totallength) return -1;
        lastwhole = current;
      } else if (leaf + fd < totallength && text[leaf + fd] != 255) {
        unnec++;
      }
      current++;
    } else if (r[0] == 1) {
      const uint64_t fd = r[2], sd = r[4], slb = r[5], srb = r[6];
      for (uint64_t idx = fd + 1; idx < sd; idx++) {
        uint64_t *c = counts + 4 * idx;
        if (idx > maxlen) return -1;
        if (lastwhole != undef && lastwhole >= slb) {
          if (lastwhole > srb) return -1;
          c[0]++;
          c[1] += srb - slb + 1;
        } else {
          c[2]++;
          c[3] += srb - slb + 1;
        }
      }
    } else {
      const uint64_t lcp = r[2], lb = r[3], rb = r[4];
      uint64_t *c;
      if (lcp > maxlen) return -1;
      c = counts + 4 * lcp;
      if (lastwhole != undef && lastwhole >= lb) {
        if (lastwhole > rb) return -1;
        c[0]++;
        c[1] += rb - lb + 1;
      } else {
        c[2]++;
        c[3] += rb - lb + 1;
      }
    }
  }
  *unnecessary = unnec;
  return 0;
}
