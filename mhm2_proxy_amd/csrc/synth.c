/* Deterministic synthetic read generator; see include/mhmkc_synth.h. */
#include "../../include/mhmkc_synth.h"

#include <pthread.h>
#include <stdlib.h>

static inline uint64_t splitmix64(uint64_t *s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

int mhmkc_synth_config_init(mhmkc_synth_config *cfg, uint64_t genome_len, uint32_t read_len, uint64_t seed) {
  if (!cfg) return -1;
  cfg->genome_len = genome_len;
  cfg->read_len = read_len;
  cfg->seed = seed;
  cfg->sub_rate = 0.005;
  cfg->n_rate = 0.0002;
  cfg->lowq_rate = 0.02;
  cfg->subq_prob = 0.5;
  return 0;
}

int mhmkc_synth_genome(const mhmkc_synth_config *cfg, uint8_t *genome) {
  if (!cfg || !genome) return -1;
  uint64_t s = cfg->seed ^ 0xA5A5A5A5A5A5A5A5ULL;
  for (uint64_t i = 0; i < cfg->genome_len; i += 32) {
    const uint64_t x = splitmix64(&s);
    for (uint64_t j = 0; j < 32 && i + j < cfg->genome_len; j++) genome[i + j] = (uint8_t)((x >> (2 * j)) & 3);
  }
  return 0;
}

typedef struct {
  const mhmkc_synth_config *cfg;
  const uint8_t *genome;
  uint64_t first, lo, hi;
  uint8_t *bytes;
} job_t;

static uint32_t thr32(double p) {
  double v = p * 4294967296.0;
  if (v <= 0) return 0;
  if (v >= 4294967295.0) return 0xFFFFFFFFu;
  return (uint32_t)v;
}

static void gen_range(const job_t *j) {
  const mhmkc_synth_config *c = j->cfg;
  const uint32_t L = c->read_len;
  const uint64_t span = c->genome_len - L + 1;
  const uint32_t t_sub = thr32(c->sub_rate), t_n = thr32(c->n_rate), t_lq = thr32(c->lowq_rate);
  const uint32_t t_sq = thr32(c->subq_prob);
  for (uint64_t r = j->lo; r < j->hi; r++) {
    const uint64_t gi = j->first + r;
    uint64_t s = c->seed * 0x9E3779B97F4A7C15ULL + (gi + 1) * 0xD1B54A32D192ED03ULL;
    (void)splitmix64(&s);
    const uint64_t start = splitmix64(&s) % span;
    const int rc = (int)(splitmix64(&s) & 1);
    uint8_t *out = j->bytes + r * L;
    for (uint32_t p = 0; p < L; p++) {
      uint32_t b = rc ? 3u - j->genome[start + L - 1 - p] : j->genome[start + p];
      uint32_t q = 40;
      const uint64_t u = splitmix64(&s), v = splitmix64(&s);
      if ((uint32_t)u < t_sub) {
        b = (b + 1 + (uint32_t)((u >> 32) % 3)) & 3;
        if ((uint32_t)(v >> 32) < t_sq) q = 2;
      }
      if ((uint32_t)v < t_n) b = 4;
      const uint64_t w = splitmix64(&s);
      if ((uint32_t)w < t_lq && q > 10) q = 10;
      out[p] = (uint8_t)(b | ((q > 31 ? 31 : q) << 3));
    }
  }
}

static void *worker(void *arg) {
  gen_range((const job_t *)arg);
  return NULL;
}

int mhmkc_synth_reads(const mhmkc_synth_config *cfg, const uint8_t *genome, uint64_t first_read, uint64_t n_reads,
                      uint8_t *bytes, uint64_t *offsets, int n_threads) {
  if (!cfg || !genome || (n_reads && (!bytes || !offsets)) || cfg->read_len == 0 || cfg->read_len > 65535 ||
      cfg->genome_len < cfg->read_len)
    return -1;
  for (uint64_t r = 0; r <= n_reads; r++) offsets[r] = r * cfg->read_len;
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 256) n_threads = 256;
  if ((uint64_t)n_threads > n_reads) n_threads = n_reads ? (int)n_reads : 1;
  job_t jobs[256];
  pthread_t th[256];
  for (int t = 0; t < n_threads; t++) {
    jobs[t].cfg = cfg;
    jobs[t].genome = genome;
    jobs[t].first = first_read;
    jobs[t].lo = n_reads * t / n_threads;
    jobs[t].hi = n_reads * (t + 1) / n_threads;
    jobs[t].bytes = bytes;
  }
  if (n_threads == 1) {
    gen_range(&jobs[0]);
    return 0;
  }
  int started = 0;
  for (int t = 0; t < n_threads; t++) {
    if (pthread_create(&th[t], NULL, worker, &jobs[t]) != 0) break;
    started++;
  }
  for (int t = started; t < n_threads; t++) gen_range(&jobs[t]);
  for (int t = 0; t < started; t++) pthread_join(th[t], NULL);
  return 0;
}
