/*
 * gt_smax_synth.h -- deterministic synthetic genomes for the benchmark
 * configurations of SURVEY.md §8(d), in GenomeTools' encoded alphabet
 * (0..3 bases, 254 wildcard, 255 separator).  No reference counterpart:
 * the reference's benchmarks use external genomes that are not available
 * offline.
 */
#ifndef GT_SMAX_SYNTH_H
#define GT_SMAX_SYNTH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GT_SMAX_SYNTH_UNIFORM 0   /* C2 */
#define GT_SMAX_SYNTH_HUMAN 1     /* C3/C4 */
#define GT_SMAX_SYNTH_PLANT 2     /* C5 */

/* totallength n for `bases` sequence symbols (separators added). */
int gt_smax_synth_total_length(int kind, uint64_t bases, uint64_t *n_out);

/* Writes n encoded symbols into out (cap >= n); threads >= 1. */
int gt_smax_synth_generate(int kind, uint64_t bases, uint64_t seed, uint8_t *out,
                           uint64_t cap, uint64_t *n_out, int threads);

#ifdef __cplusplus
}
#endif

#endif
