/*
 * mhmkc_synth.h — deterministic synthetic read generator (libmhmkc_synth.so, host only).
 *
 * Implements the generator of SURVEY.md §8(d) / BASELINE.md (the arctic FASTQ sets cannot be fetched
 * offline): splitmix64, an i.i.d. uniform ACGT genome of length G, reads of length L starting
 * uniformly in [0, G-L], reverse-complemented with p = 0.5, substitutions with p = sub_rate (uniform
 * over the other 3 bases), N with p = n_rate; quality Q40 ('I') by default, substituted bases get Q2
 * ('#') with p = 0.5, an independent lowq_rate of bases gets Q10 ('+').
 *
 * Output is in the PackedRead byte layout (src/packed_reads.cpp:73-109): code | min(Q, 31) << 3.
 * Read i of a run depends only on (seed, i), so ranks can generate disjoint shards of one global set
 * (first_read) and any thread split gives identical bytes.
 */
#ifndef MHMKC_SYNTH_H
#define MHMKC_SYNTH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  uint64_t genome_len;  /* G */
  uint32_t read_len;    /* L, <= 65535 */
  uint64_t seed;
  double sub_rate;      /* 0.005 */
  double n_rate;        /* 0.0002 */
  double lowq_rate;     /* 0.02 */
  double subq_prob;     /* 0.5 */
} mhmkc_synth_config;

int mhmkc_synth_config_init(mhmkc_synth_config *cfg, uint64_t genome_len, uint32_t read_len, uint64_t seed);

/* genome: genome_len bytes, codes 0..3 */
int mhmkc_synth_genome(const mhmkc_synth_config *cfg, uint8_t *genome);

/* reads first_read .. first_read + n_reads - 1 of the global read set:
 * bytes[n_reads * read_len], offsets[n_reads + 1] (offsets[0] = 0). n_threads <= 0: 1. */
int mhmkc_synth_reads(const mhmkc_synth_config *cfg, const uint8_t *genome, uint64_t first_read, uint64_t n_reads,
                      uint8_t *bytes, uint64_t *offsets, int n_threads);

#ifdef __cplusplus
}
#endif

#endif /* MHMKC_SYNTH_H */
