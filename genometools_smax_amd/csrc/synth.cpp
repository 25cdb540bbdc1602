// synth.cpp -- deterministic synthetic genomes for the benchmark configs
// (SURVEY.md §8(d)), written directly in GenomeTools' encoded alphabet:
// bases 0..3 (acgt), WILDCARD 254 for N, SEPARATOR 255 between sequences
// (src/core/chardef.h:34-65, src/core/alphabet.c:440-465).
//
//   GT_SMAX_SYNTH_UNIFORM  C2: i.i.d. uniform ACGT, one sequence, no N.
//   GT_SMAX_SYNTH_HUMAN    C3: 24 sequences; 40 % of bases from 200
//                          interspersed families (consensus 300-6,000 bp,
//                          fragments with 2-20 % substitution divergence,
//                          either strand), 2 % short tandem repeats (period
//                          1-6), 0.5 % segmental duplications (1-50 kb,
//                          <= 0.5 % divergence; force lcp >= 255 -> .llv),
//                          1 % N in 50 kb gaps.
//   GT_SMAX_SYNTH_PLANT    C5: 10 sequences; 80 % LTR-retrotransposon-like
//                          families (5-15 kb, 0.5-15 % divergence, nested
//                          insertions), 1 % N in 50 kb gaps.
//
// Random numbers: xoshiro256** seeded through splitmix64.  Every sequence has
// its own stream (seed, sequence number), so sequences are generated in
// parallel and the output does not depend on the thread count.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "gt_smax_synth.h"

namespace {

struct Rng {
  uint64_t s[4];
  static uint64_t splitmix(uint64_t &x) {
    uint64_t z = (x += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
  }
  Rng(uint64_t seed, uint64_t stream) {
    uint64_t x = seed * 0x632be59bd9b4e019ull + stream * 0x8cb92ba72f3d8dd7ull + 1;
    for (int i = 0; i < 4; i++) s[i] = splitmix(x);
  }
  static uint64_t rotl(uint64_t v, int k) { return (v << k) | (v >> (64 - k)); }
  uint64_t next() {
    const uint64_t r = rotl(s[1] * 5, 7) * 9;
    const uint64_t t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3];
    s[2] ^= t; s[3] = rotl(s[3], 45);
    return r;
  }
  // uniform integer in [lo, hi]
  uint64_t range(uint64_t lo, uint64_t hi) {
    return lo + (uint64_t) (((unsigned __int128) next() * (hi - lo + 1)) >> 64);
  }
  double unit() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
};

// fills dst[0..len) with uniform bases, 32 per random word
void fill_uniform(Rng &r, uint8_t *dst, uint64_t len) {
  uint64_t i = 0;
  while (i < len) {
    uint64_t w = r.next();
    for (int k = 0; k < 32 && i < len; k++, i++) { dst[i] = (uint8_t) (w & 3); w >>= 2; }
  }
}

// copy src (length len) into dst with substitution rate d, optionally
// reverse-complemented
void copy_mutated(Rng &r, uint8_t *dst, const uint8_t *src, uint64_t len, double d,
                  bool revcomp) {
  const uint64_t thr = (uint64_t) (d * 18446744073709551615.0);
  for (uint64_t i = 0; i < len; i++) {
    uint8_t b = revcomp ? (uint8_t) (3 - src[len - 1 - i]) : src[i];
    if (b < 4 && r.next() < thr) b = (uint8_t) ((b + 1 + r.range(0, 2)) & 3);
    dst[i] = b;
  }
}

struct Families {
  std::vector<std::vector<uint8_t>> cons;
};

Families make_families(uint64_t seed, int count, uint64_t minlen, uint64_t maxlen) {
  Families f;
  Rng r(seed, 0xfa11111e5ull);
  f.cons.resize(count);
  for (int i = 0; i < count; i++) {
    f.cons[i].resize(r.range(minlen, maxlen));
    fill_uniform(r, f.cons[i].data(), f.cons[i].size());
  }
  return f;
}

enum Seg { BG, FAM, STR, SEGDUP, NGAP, NSEG };

struct Profile {
  double frac[NSEG];        // target fraction of bases
  double meanlen[NSEG];     // mean segment length
  double div_lo, div_hi;    // family divergence range
  uint64_t fam_min, fam_max;
  int nfam;
  double nested;            // probability a family insert is nested
};

void gen_sequence(const Profile &p, const Families &fam, uint64_t seed, uint64_t seqno,
                  uint8_t *dst, uint64_t len) {
  Rng r(seed, seqno + 1);
  double w[NSEG], wsum = 0;
  for (int k = 0; k < NSEG; k++) { w[k] = p.frac[k] / p.meanlen[k]; wsum += w[k]; }
  uint64_t pos = 0;
  while (pos < len) {
    double u = r.unit() * wsum;
    int k = 0;
    while (k < NSEG - 1 && u >= w[k]) { u -= w[k]; k++; }
    uint64_t room = len - pos;
    switch (k) {
      case BG: {
        uint64_t L = std::min<uint64_t>(room, r.range(1, (uint64_t) (2 * p.meanlen[BG])));
        fill_uniform(r, dst + pos, L);
        pos += L;
        break;
      }
      case FAM: {
        const std::vector<uint8_t> &c = fam.cons[r.range(0, p.nfam - 1)];
        uint64_t cl = c.size();
        uint64_t flen = r.range(std::min<uint64_t>(100, cl), cl);
        uint64_t off = r.range(0, cl - flen);
        flen = std::min(flen, room);
        double d = p.div_lo + (p.div_hi - p.div_lo) * r.unit();
        bool rc = (r.next() & 1) != 0;
        if (p.nested > 0 && flen > 400 && r.unit() < p.nested) {
          // nested insertion: host fragment split by a second fragment
          uint64_t cut = r.range(100, flen - 100);
          copy_mutated(r, dst + pos, c.data() + off, cut, d, rc);
          pos += cut;
          const std::vector<uint8_t> &c2 = fam.cons[r.range(0, p.nfam - 1)];
          uint64_t l2 = std::min<uint64_t>(len - pos, r.range(std::min<uint64_t>(100, c2.size()), c2.size()));
          copy_mutated(r, dst + pos, c2.data(), l2, d * 0.5, !rc);
          pos += l2;
          uint64_t rest = std::min<uint64_t>(len - pos, flen - cut);
          copy_mutated(r, dst + pos, c.data() + off + cut, rest, d, rc);
          pos += rest;
        } else {
          copy_mutated(r, dst + pos, c.data() + off, flen, d, rc);
          pos += flen;
        }
        break;
      }
      case STR: {
        uint64_t period = r.range(1, 6);
        uint8_t unit[6];
        for (uint64_t i = 0; i < period; i++) unit[i] = (uint8_t) (r.next() & 3);
        uint64_t L = std::min<uint64_t>(room, r.range(20, 300));
        for (uint64_t i = 0; i < L; i++) dst[pos + i] = unit[i % period];
        pos += L;
        break;
      }
      case SEGDUP: {
        uint64_t L = std::min<uint64_t>(room, r.range(1000, 50000));
        if (pos < 2 * L) {   // nothing earlier to copy yet: background
          fill_uniform(r, dst + pos, L);
        } else {
          uint64_t from = r.range(0, pos - L);
          double d = 0.005 * r.unit();
          copy_mutated(r, dst + pos, dst + from, L, d, false);
        }
        pos += L;
        break;
      }
      default: {   // N gap of 50 kb
        uint64_t L = std::min<uint64_t>(room, 50000);
        memset(dst + pos, 254, L);
        pos += L;
        break;
      }
    }
  }
}

int profile_of(int kind, Profile *p, uint64_t *numseq) {
  memset(p, 0, sizeof *p);
  switch (kind) {
    case GT_SMAX_SYNTH_HUMAN:
      *numseq = 24;
      p->frac[BG] = 0.565; p->meanlen[BG] = 2000;
      p->frac[FAM] = 0.40; p->meanlen[FAM] = 1600;
      p->frac[STR] = 0.02; p->meanlen[STR] = 160;
      p->frac[SEGDUP] = 0.005; p->meanlen[SEGDUP] = 25500;
      p->frac[NGAP] = 0.01; p->meanlen[NGAP] = 50000;
      p->div_lo = 0.02; p->div_hi = 0.20;
      p->fam_min = 300; p->fam_max = 6000; p->nfam = 200; p->nested = 0;
      return 0;
    case GT_SMAX_SYNTH_PLANT:
      *numseq = 10;
      p->frac[BG] = 0.19; p->meanlen[BG] = 2000;
      p->frac[FAM] = 0.80; p->meanlen[FAM] = 5500;
      p->frac[STR] = 1e-9; p->meanlen[STR] = 160;
      p->frac[SEGDUP] = 1e-9; p->meanlen[SEGDUP] = 25500;
      p->frac[NGAP] = 0.01; p->meanlen[NGAP] = 50000;
      p->div_lo = 0.005; p->div_hi = 0.15;
      p->fam_min = 5000; p->fam_max = 15000; p->nfam = 400; p->nested = 0.3;
      return 0;
    case GT_SMAX_SYNTH_UNIFORM:
      *numseq = 1;
      return 0;
    default:
      return -1;
  }
}

}  // namespace

extern "C" int gt_smax_synth_total_length(int kind, uint64_t bases, uint64_t *n_out) {
  Profile p;
  uint64_t numseq;
  if (profile_of(kind, &p, &numseq) != 0 || bases < numseq) return -1;
  *n_out = bases + numseq - 1;
  return 0;
}

extern "C" int gt_smax_synth_generate(int kind, uint64_t bases, uint64_t seed, uint8_t *out,
                                      uint64_t cap, uint64_t *n_out, int threads) {
  Profile p;
  uint64_t numseq;
  if (profile_of(kind, &p, &numseq) != 0 || bases < numseq) return -1;
  const uint64_t n = bases + numseq - 1;
  if (cap < n) return -1;
  if (kind == GT_SMAX_SYNTH_UNIFORM) {
    // chunked so it parallelises; chunk streams are fixed, not per-thread
    const uint64_t chunk = 1ull << 24;
    const uint64_t nch = (bases + chunk - 1) / chunk;
    int nt = threads > 0 ? threads : 1;
    std::vector<std::thread> pool;
    for (int t = 0; t < nt; t++) {
      pool.emplace_back([&, t]() {
        for (uint64_t c = (uint64_t) t; c < nch; c += (uint64_t) nt) {
          Rng r(seed, 0x100000000ull + c);
          uint64_t lo = c * chunk, len = std::min(chunk, bases - lo);
          fill_uniform(r, out + lo, len);
        }
      });
    }
    for (auto &th : pool) th.join();
    *n_out = n;
    return 0;
  }
  Families fam = make_families(seed, p.nfam, p.fam_min, p.fam_max);
  std::vector<uint64_t> start(numseq), len(numseq);
  uint64_t pos = 0;
  for (uint64_t s = 0; s < numseq; s++) {
    // unequal sequence lengths (roughly like chromosomes), deterministic
    len[s] = bases / numseq;
    if (s < bases % numseq) len[s]++;
    start[s] = pos;
    pos += len[s] + 1;
    if (s + 1 < numseq) out[start[s] + len[s]] = 255;
  }
  int nt = threads > 0 ? threads : 1;
  std::vector<std::thread> pool;
  for (int t = 0; t < nt; t++) {
    pool.emplace_back([&, t]() {
      for (uint64_t s = (uint64_t) t; s < numseq; s += (uint64_t) nt)
        gen_sequence(p, fam, seed, s, out + start[s], len[s]);
    });
  }
  for (auto &th : pool) th.join();
  *n_out = n;
  return 0;
}
