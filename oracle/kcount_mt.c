/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. Not part of the product.
 *
 * Multi-threaded CPU restatement of the reference's kcount read pass (ajpowelsnl/mhm2_proxy
 * src/kcount/kcount_cpu.cpp with src/kmer.cpp and src/hash_funcs.c), for the two jobs a single-threaded
 * checker cannot do (BASELINE.md "CPU-baseline plan"):
 *   - the at-scale parity gate: C2-size (10M reads) tables compared row by row with the GPU on the GPU box;
 *   - bench.py's cpu_baseline: T threads on the GPU box's host cores, k-mers partitioned over the threads by
 *     their hash the way the reference partitions them over ranks (src/kcount/kmer_dht.cpp:193-196).
 * It is pinned to the single-threaded restatement (kcount_oracle.c) and to the golden fixtures by
 * tests/test_oracle.py; it shares no code with mhm2_proxy_amd/ or with kcount_oracle.c.
 *
 * Semantics: a read of length L >= k+2 contributes its interior windows
 * i in [1, L-k-1] (get_kmers_and_exts, kcount_cpu.cpp:316-334; one supermer per read at one rank,
 * kcount_cpu.cpp:84-101); bases code A0 C1 G2 T3 with N counted as G (Kmer::get_kmers, kmer.cpp:169,187-188);
 * an extension is the neighbour base when it is A/C/G/T with quality >= cutoff (count_kmers lowercasing,
 * kcount.cpp:80-85; ExtCounts::inc ignores the rest, kcount_cpu.cpp:152-164); canonical = min(kmer, revcomp)
 * with the extensions complemented and swapped (kcount_cpu.cpp:326-332); counts saturate at 65535
 * (:148-151: a saturating +1 is order independent, so a wide counter clamped at the end is the same);
 * finalize drops count < 2, picks get_ext with the exact double expression and drops X/X (:173-182,490-528).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define MT_MAXNL 4
#define MT_PARTS 256
#define MT_DIG 6 /* digest words per key range: rows, xor, sum, sum of fmix (of the row fingerprints), distinct, occurrences */

/* MurmurHash3_x64_128 h1 of the key words, seed 313 (src/hash_funcs.c:77-170,185-190; Kmer::hash,
 * src/kmer.cpp:465-468): the thread partition and the table slot. */
static inline uint64_t mt_rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t mt_fmix(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}
static uint64_t mt_hash(const uint64_t *w, int nl) {
  const uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
  uint64_t h1 = 313, h2 = 313;
  for (int b = 0; b < nl / 2; b++) {
    uint64_t k1 = w[2 * b] * c1, k2 = w[2 * b + 1] * c2;
    h1 ^= mt_rotl(k1, 31) * c2;
    h1 = mt_rotl(h1, 27) + h2;
    h1 = h1 * 5 + 0x52dce729;
    h2 ^= mt_rotl(k2, 33) * c1;
    h2 = mt_rotl(h2, 31) + h1;
    h2 = h2 * 5 + 0x38495ab5;
  }
  if (nl & 1) h1 ^= mt_rotl(w[nl - 1] * c1, 31) * c2;
  h1 ^= (uint64_t)(8 * nl);
  h2 ^= (uint64_t)(8 * nl);
  h1 += h2;
  h2 += h1;
  h1 = mt_fmix(h1);
  h2 = mt_fmix(h2);
  return h1 + h2;
}

/* records of one (thread, partition): key words + ext code (left << 3 | right, 4 = none) */
typedef struct {
  uint64_t *keys;
  uint8_t *ext;
  uint64_t n, cap;
} mt_bin;

static int bin_push(mt_bin *b, const uint64_t *key, int nl, uint8_t e) {
  if (b->n == b->cap) {
    /* (doubling: a 1.25x growth made a pass holding four key ranges' records 2.5x slower, reallocs copying) */
    uint64_t nc = b->cap ? 2 * b->cap : 4096;
    uint64_t *nk = (uint64_t *)realloc(b->keys, nc * 8 * (size_t)nl);
    if (!nk) return 0;
    b->keys = nk;
    uint8_t *ne = (uint8_t *)realloc(b->ext, nc);
    if (!ne) return 0;
    b->ext = ne;
    b->cap = nc;
  }
  memcpy(b->keys + b->n * nl, key, 8 * (size_t)nl);
  b->ext[b->n++] = e;
  return 1;
}

/* Key range of a canonical k-mer for a table built one part at a time (orc_kcount_mt_range): a one-multiply mix of
 * the first and last key words, cheap next to mt_hash, so that a pass over all windows spends the hash and the
 * binning only on the windows of its range. Any function of the key partitions the table; this one is the checker's
 * own (not the product's owner function). */
static inline uint32_t mt_range(const uint64_t *key, int nl, uint32_t n_ranges) {
  const uint64_t x = (key[0] * 0x9E3779B97F4A7C15ULL ^ key[nl - 1]) * 0xD6E8FEB86659FD93ULL;
  return (uint32_t)(((x >> 32) * (uint64_t)n_ranges) >> 32);
}

/* contig records of one partition, in contig order (the contig pass is order dependent): key words, ext codes
 * (left << 3 | right; A0 C1 G2 T3, 4 = none: 'N', or a base below the quality cutoff) and the contig's depth */
typedef struct {
  uint64_t *keys;
  uint8_t *ext;
  uint16_t *depth;
  uint64_t n, cap;
} mt_cbin;

static int cbin_push(mt_cbin *b, const uint64_t *key, int nl, uint8_t e, uint16_t d) {
  if (b->n == b->cap) {
    uint64_t nc = b->cap ? 2 * b->cap : 1024;
    uint64_t *nk = (uint64_t *)realloc(b->keys, nc * 8 * (size_t)nl);
    if (!nk) return 0;
    b->keys = nk;
    uint8_t *ne = (uint8_t *)realloc(b->ext, nc);
    if (!ne) return 0;
    b->ext = ne;
    uint16_t *nd = (uint16_t *)realloc(b->depth, nc * 2);
    if (!nd) return 0;
    b->depth = nd;
    b->cap = nc;
  }
  memcpy(b->keys + b->n * nl, key, 8 * (size_t)nl);
  b->ext[b->n] = e;
  b->depth[b->n++] = d;
  return 1;
}

typedef struct {
  /* input */
  const uint8_t *bytes;
  const uint64_t *offs;
  uint64_t r0, r1;
  uint32_t range, n_ranges; /* keep only the k-mers with mt_range in [range, range + n_sel) */
  uint32_t n_sel;           /* key ranges binned by one extraction pass (bins [n_sel][MT_PARTS]) */
  uint64_t *dig;            /* orc_kcount_mt_digests: per selected range rows, xor, sum of row fingerprints */
  int k, nl, qcut, dmin;
  double dyn_mult; /* 1.0 - DYN_MIN_DEPTH, in double as the reference computes it */
  int nthreads;
  mt_bin *bins; /* [MT_PARTS] of this thread */
  /* output of phase 2 */
  uint64_t *out_keys;
  uint16_t *out_counts;
  char *out_l, *out_r;
  uint64_t n_out, cap_out;
  uint64_t occ, distinct, purged;
  int fail;
} mt_work;

typedef struct {
  mt_work *w;
  int nthreads;
  int next_part, n_part_bins; /* partitions to count: n_sel x MT_PARTS */
  pthread_mutex_t lock;
  const mt_cbin *cbins; /* [MT_PARTS]: the contig pass's records, or NULL */
} mt_shared;

typedef struct {
  mt_shared *sh;
  int me;
} mt_arg;

/* phase 1: windows of this thread's reads -> records binned by partition */
static void *mt_extract(void *arg) {
  mt_work *w = (mt_work *)arg;
  const int k = w->k, nl = w->nl, klast = k - 32 * (nl - 1);
  const uint64_t lastmask = klast >= 32 ? ~0ULL : ~(~0ULL >> (2 * klast));
  for (uint64_t r = w->r0; r < w->r1; r++) {
    const uint64_t a = w->offs[r], L = w->offs[r + 1] - a;
    if (L < (uint64_t)k + 2) continue; /* kcount.cpp:78; process_seq emits a supermer of >= k+2 bases */
    const uint8_t *s = w->bytes + a;
    uint64_t fw[MT_MAXNL] = {0}, rc[MT_MAXNL] = {0};
    /* the first window (i = 0) built base by base, then rolled; window i is [i, i+k) */
    for (int j = 0; j < k; j++) {
      const uint32_t c = s[j] & 7u;
      if (c > 4) {
        w->fail = 1;
        return NULL;
      }
      const uint64_t t = c == 4 ? 2 : c; /* N -> G */
      fw[j >> 5] |= t << (62 - 2 * (j & 31));
      /* revcomp: base j of the k-mer is base k-1-j of the reverse complement, complemented */
      const int q = k - 1 - j;
      rc[q >> 5] |= (3 - t) << (62 - 2 * (q & 31));
    }
    for (uint64_t i = 0; i + k < L; i++) {
      if (i >= 1) {
        /* roll: base i-1 leaves, base i+k-1 enters */
        const uint32_t c = s[i + k - 1] & 7u;
        if (c > 4) {
          w->fail = 1;
          return NULL;
        }
        const uint64_t t = c == 4 ? 2 : c;
        for (int m = 0; m < nl - 1; m++) fw[m] = (fw[m] << 2) | (fw[m + 1] >> 62);
        fw[nl - 1] = ((fw[nl - 1] << 2) | (t << (64 - 2 * klast))) & lastmask;
        for (int m = nl - 1; m > 0; m--) rc[m] = (rc[m] >> 2) | (rc[m - 1] << 62);
        rc[0] = (rc[0] >> 2) | ((3 - t) << 62);
        rc[nl - 1] &= lastmask;
      }
      if (i == 0) continue; /* interior windows only: i in [1, L-k-1] */
      const uint8_t lb = s[i - 1], rb = s[i + k];
      if ((rb & 7u) > 4) {
        w->fail = 1;
        return NULL;
      }
      int l = ((lb & 7u) < 4 && (int)(lb >> 3) >= w->qcut) ? (lb & 7) : 4;
      int rr = ((rb & 7u) < 4 && (int)(rb >> 3) >= w->qcut) ? (rb & 7) : 4;
      int use_rc = 0;
      for (int m = 0; m < nl; m++)
        if (rc[m] != fw[m]) {
          use_rc = rc[m] < fw[m];
          break;
        }
      const uint64_t *key = use_rc ? rc : fw;
      uint32_t sel = 0;
      if (w->n_ranges > 1) {
        sel = mt_range(key, nl, w->n_ranges) - w->range;
        if (sel >= w->n_sel) continue;
      }
      if (use_rc) { /* complement and swap (comp_nucleotide, src/utils.cpp:121-143) */
        const int nl_ = rr < 4 ? 3 - rr : 4, nr_ = l < 4 ? 3 - l : 4;
        l = nl_;
        rr = nr_;
      }
      const uint64_t h = mt_hash(key, nl);
      if (!bin_push(&w->bins[sel * MT_PARTS + (h >> 56)], key, nl, (uint8_t)((l << 3) | rr))) {
        w->fail = 1;
        return NULL;
      }
    }
  }
  return NULL;
}

/* The contig pass's records (add_ctg_kmers, src/kcount/kcount.cpp:100-138 -> process_seq with count = depth, depth 0
 * -> 1, kcount_cpu.cpp:73-103 -> get_kmers_and_exts, :307-335): the interior windows of every contig of >= k + 2
 * bases, in contig order, binned by partition like the reads' records. Case is quality (upper = good); 'N' keys as G
 * and is no extension. Returns 0 on a character the reference DIEs on (:453-458) or allocation failure. */
static int mt_ctg_records(const char *chars, const uint64_t *offs, const uint16_t *depths, uint64_t n_ctgs, int k,
                          int nl, uint32_t range, uint32_t n_ranges, mt_cbin *cbins) {
  const int klast = k - 32 * (nl - 1);
  const uint64_t lastmask = klast >= 32 ? ~0ULL : ~(~0ULL >> (2 * klast));
  uint8_t *code = NULL, *ext = NULL;
  uint64_t cap = 0;
  int ok = 1;
  for (uint64_t c = 0; c < n_ctgs && ok; c++) {
    const uint64_t L = offs[c + 1] - offs[c];
    if (L < (uint64_t)k + 2) continue; /* kcount.cpp:128 */
    if (L > cap) {
      free(code);
      free(ext);
      cap = L;
      code = (uint8_t *)malloc(cap);
      ext = (uint8_t *)malloc(cap);
      if (!code || !ext) return 0;
    }
    const char *s = chars + offs[c];
    for (uint64_t j = 0; j < L; j++) {
      const char b = s[j], u = (b >= 'a' && b <= 'z') ? (char)(b - 32) : b;
      int t;
      switch (u) {
        case 'A': t = 0; break;
        case 'C': t = 1; break;
        case 'G': t = 2; break;
        case 'T': t = 3; break;
        case 'N': t = 4; break;
        default: ok = 0; t = 4;
      }
      code[j] = (uint8_t)(t == 4 ? 2 : t);
      ext[j] = (uint8_t)((b >= 'A' && b <= 'Z' && t < 4) ? t : 4);
    }
    if (!ok) break;
    const uint16_t depth = depths[c] ? depths[c] : 1;
    uint64_t fw[MT_MAXNL] = {0}, rc[MT_MAXNL] = {0};
    for (int j = 0; j < k; j++) {
      const uint64_t t = code[j];
      fw[j >> 5] |= t << (62 - 2 * (j & 31));
      const int q = k - 1 - j;
      rc[q >> 5] |= (3 - t) << (62 - 2 * (q & 31));
    }
    for (uint64_t i = 0; i + k < L && ok; i++) {
      if (i >= 1) {
        const uint64_t t = code[i + k - 1];
        for (int m = 0; m < nl - 1; m++) fw[m] = (fw[m] << 2) | (fw[m + 1] >> 62);
        fw[nl - 1] = ((fw[nl - 1] << 2) | (t << (64 - 2 * klast))) & lastmask;
        for (int m = nl - 1; m > 0; m--) rc[m] = (rc[m] >> 2) | (rc[m - 1] << 62);
        rc[0] = (rc[0] >> 2) | ((3 - t) << 62);
        rc[nl - 1] &= lastmask;
      }
      if (i == 0) continue;
      int l = ext[i - 1], r = ext[i + k];
      int use_rc = 0;
      for (int m = 0; m < nl; m++)
        if (rc[m] != fw[m]) {
          use_rc = rc[m] < fw[m];
          break;
        }
      const uint64_t *key = use_rc ? rc : fw;
      if (n_ranges > 1 && mt_range(key, nl, n_ranges) != range) continue;
      if (use_rc) {
        const int nl_ = r < 4 ? 3 - r : 4, nr_ = l < 4 ? 3 - l : 4;
        l = nl_;
        r = nr_;
      }
      ok = cbin_push(&cbins[mt_hash(key, nl) >> 56], key, nl, (uint8_t)((l << 3) | r), depth);
    }
  }
  free(code);
  free(ext);
  return ok;
}

/* get_ext (kcount_cpu.cpp:173-182, get_sorted :133-145: descending count, ties to the higher char) */
static char mt_get_ext(const uint32_t *e, uint32_t count, int dmin, double dyn_mult) {
  static const char ch[4] = {'A', 'C', 'G', 'T'};
  int top = -1, second = -1, arg = 0;
  for (int i = 3; i >= 0; i--) { /* from T down: the first maximum is the higher char */
    const int v = (int)(e[i] > 65535 ? 65535 : e[i]);
    if (v > top) {
      second = top;
      top = v;
      arg = i;
    } else if (v > second) {
      second = v;
    }
  }
  int thr = (int)(dyn_mult * (double)count);
  if (thr < dmin) thr = dmin;
  if (top < thr) return 'X';
  if (second >= thr) return 'F';
  return ch[arg];
}

typedef struct {
  uint32_t count;
  uint32_t l[4], r[4];
  uint32_t from_ctg; /* KmerExtsCounts::from_ctg (kcount_cpu.cpp:191-196) */
} mt_val;

static char mt_ext_char(int code) { return code < 4 ? "ACGT"[code] : 'N'; }

/* phase 2: count and finalize whole partitions (every record of a partition, from every thread) */
static void *mt_count(void *arg) {
  mt_shared *sh = ((mt_arg *)arg)->sh;
  mt_work *w = &sh->w[((mt_arg *)arg)->me];
  const int nl = w->nl;
  uint64_t tcap = 0;
  uint64_t *tk = NULL;
  mt_val *tv = NULL;
  uint8_t *used = NULL;
  for (;;) {
    pthread_mutex_lock(&sh->lock);
    const int p = sh->next_part < sh->n_part_bins ? sh->next_part++ : -1;
    pthread_mutex_unlock(&sh->lock);
    if (p < 0) break;
    uint64_t n = 0;
    for (int t = 0; t < sh->nthreads; t++) n += sh->w[t].bins[p].n;
    if (sh->cbins) n += sh->cbins[p].n;
    if (!n) continue;
    uint64_t cap = 1024;
    while (cap < n + n / 2) cap <<= 1; /* distinct <= records: load <= 2/3 */
    if (cap > tcap) {
      free(tk);
      free(tv);
      free(used);
      tk = (uint64_t *)malloc(cap * 8 * (size_t)nl);
      tv = (mt_val *)malloc(cap * sizeof(mt_val));
      used = (uint8_t *)malloc(cap);
      tcap = cap;
      if (!tk || !tv || !used) {
        w->fail = 1;
        break;
      }
    }
    memset(used, 0, cap);
    const uint64_t distinct0 = w->distinct, occ0 = w->occ;
    for (int t = 0; t < sh->nthreads; t++) {
      const mt_bin *b = &sh->w[t].bins[p];
      for (uint64_t i = 0; i < b->n; i++) {
        const uint64_t *key = b->keys + i * nl;
        uint64_t s = (mt_hash(key, nl) * 0x9E3779B97F4A7C15ULL) >> 8 & (cap - 1);
        for (;;) {
          if (!used[s]) {
            used[s] = 1;
            memcpy(tk + s * nl, key, 8 * (size_t)nl);
            memset(&tv[s], 0, sizeof(mt_val));
            w->distinct++;
            break;
          }
          if (memcmp(tk + s * nl, key, 8 * (size_t)nl) == 0) break;
          s = (s + 1) & (cap - 1);
        }
        mt_val *v = &tv[s];
        const uint8_t e = b->ext[i];
        v->count++;
        if ((e >> 3) < 4) v->l[e >> 3]++;
        if ((e & 7) < 4) v->r[e & 7]++;
        w->occ++;
      }
    }
    /* the contig pass over this partition, in contig order, after every read (insert_supermer_from_ctg,
     * kcount_cpu.cpp:356-406) */
    const mt_cbin *cb = sh->cbins ? &sh->cbins[p] : NULL;
    for (uint64_t i = 0; cb && i < cb->n; i++) {
      const uint64_t *key = cb->keys + i * nl;
      uint64_t s = (mt_hash(key, nl) * 0x9E3779B97F4A7C15ULL) >> 8 & (cap - 1);
      int is_new = 0;
      for (;;) {
        if (!used[s]) {
          used[s] = 1;
          memcpy(tk + s * nl, key, 8 * (size_t)nl);
          memset(&tv[s], 0, sizeof(mt_val));
          w->distinct++;
          is_new = 1;
          break;
        }
        if (memcmp(tk + s * nl, key, 8 * (size_t)nl) == 0) break;
        s = (s + 1) & (cap - 1);
      }
      mt_val *v = &tv[s];
      const int l = cb->ext[i] >> 3, r = cb->ext[i] & 7;
      uint32_t c = cb->depth[i];
      int insert_it = 0;
      if (is_new) {
        insert_it = 1;
      } else if (!v->from_ctg) { /* a read k-mer: replaced when it is a singleton or not UU */
        const uint32_t vc = v->count > 65535 ? 65535 : v->count;
        if (vc == 1) {
          insert_it = 1;
        } else {
          const char L = mt_get_ext(v->l, vc, w->dmin, w->dyn_mult), R = mt_get_ext(v->r, vc, w->dmin, w->dyn_mult);
          insert_it = L == 'X' || L == 'F' || R == 'X' || R == 'F';
        }
      } else if (v->count) { /* an earlier contig's k-mer: the lower depth, or 0 (purged) when they disagree */
        insert_it = 1;
        const char L = mt_get_ext(v->l, v->count, w->dmin, w->dyn_mult);
        const char R = mt_get_ext(v->r, v->count, w->dmin, w->dyn_mult);
        if (L != mt_ext_char(l) || R != mt_ext_char(r))
          c = 0;
        else if (v->count < c)
          c = v->count;
      }
      if (insert_it) {
        memset(v, 0, sizeof *v);
        v->count = c;
        v->from_ctg = 1;
        if (l < 4) v->l[l] = c;
        if (r < 4) v->r[r] = c;
      }
    }
    for (uint64_t s = 0; s < cap; s++) {
      if (!used[s]) continue;
      const mt_val *v = &tv[s];
      const uint32_t c = v->count > 65535 ? 65535 : v->count;
      if (c < 2) {
        w->purged++;
        continue;
      }
      const char L = mt_get_ext(v->l, c, w->dmin, w->dyn_mult), R = mt_get_ext(v->r, c, w->dmin, w->dyn_mult);
      if (L == 'X' && R == 'X') {
        w->purged++;
        continue;
      }
      if (w->dig) { /* digest only: the row's fingerprint (orc_row_fingerprints) into its range's sums */
        uint64_t h = 0x243F6A8885A308D3ULL;
        for (int q = 0; q < nl; q++) h = mt_fmix(h ^ tk[s * nl + q]) + 0x9E3779B97F4A7C15ULL;
        h = mt_fmix(h ^ ((uint64_t)c | (uint64_t)(uint8_t)L << 16 | (uint64_t)(uint8_t)R << 24));
        uint64_t *d = w->dig + MT_DIG * (size_t)(p / MT_PARTS);
        d[0]++;
        d[1] ^= h;
        d[2] += h;
        d[3] += mt_fmix(h);
        continue;
      }
      if (w->n_out == w->cap_out) {
        const uint64_t nc = w->cap_out ? 2 * w->cap_out : 1 << 16;
        uint64_t *ok = (uint64_t *)realloc(w->out_keys, nc * 8 * (size_t)nl);
        uint16_t *oc = ok ? (uint16_t *)realloc(w->out_counts, nc * 2) : NULL;
        char *ol = oc ? (char *)realloc(w->out_l, nc) : NULL;
        char *orr = ol ? (char *)realloc(w->out_r, nc) : NULL;
        if (ok) w->out_keys = ok;
        if (oc) w->out_counts = oc;
        if (ol) w->out_l = ol;
        if (!orr) {
          w->fail = 1;
          break;
        }
        w->out_r = orr;
        w->cap_out = nc;
      }
      memcpy(w->out_keys + w->n_out * nl, tk + s * nl, 8 * (size_t)nl);
      w->out_counts[w->n_out] = (uint16_t)c;
      w->out_l[w->n_out] = L;
      w->out_r[w->n_out] = R;
      w->n_out++;
    }
    if (w->dig) {
      w->dig[MT_DIG * (size_t)(p / MT_PARTS) + 4] += w->distinct - distinct0;
      w->dig[MT_DIG * (size_t)(p / MT_PARTS) + 5] += w->occ - occ0;
    }
    for (int t = 0; t < sh->nthreads; t++) { /* this partition's records are done */
      mt_bin *b = &sh->w[t].bins[p];
      free(b->keys);
      free(b->ext);
      b->keys = NULL;
      b->ext = NULL;
      b->n = b->cap = 0;
    }
  }
  free(tk);
  free(tv);
  free(used);
  return NULL;
}

/* The finished table, as kcount_oracle.c's accessors read it (orc_table_size / fetch / stats / free):
 * the layout below mirrors its struct orc_table field for field. */
typedef struct {
  int n_longs;
  uint64_t cap, n;
  uint64_t *keys;
  void *vals;
  uint8_t *used;
  uint64_t n_out;
  uint64_t *out_keys;
  uint16_t *out_counts;
  char *out_left, *out_right;
  uint64_t occurrences, purged, reads;
} mt_table;

/* The part `range` of n_ranges of the table (the k-mers with mt_range(key) == range): a table too large for host
 * memory at once (C3: 1.28e10 occurrences) is built and compared one part at a time. Returns NULL on bad input (a
 * base code > 4: the reference DIEs) or allocation failure. */
/* The core of both: n_sel consecutive ranges from `range` in one extraction pass; dig != NULL: no table, the rows'
 * fingerprint digests per range (MT_DIG words each) into dig, and a non-NULL return on success (an empty table). */
static mt_table *mt_run(const uint8_t *bytes, const uint64_t *offs, uint64_t n_reads, const char *ctg_chars,
                        const uint64_t *ctg_offs, const uint16_t *ctg_depths, uint64_t n_ctgs, int k, int n_longs,
                        int qual_cutoff, int dmin_thres, double dyn_min_depth, int threads, int range, int n_ranges,
                        int n_sel, uint64_t *dig) {
  const int nl = k / 32 + 1;
  if (k < 1 || k > 127 || k % 32 == 0 || n_longs < nl || n_longs > 8) return NULL;
  if (n_sel < 1 || (n_sel > 1 && n_ctgs) || range + n_sel > (n_ranges < 1 ? 1 : n_ranges)) return NULL;
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  mt_work *w = (mt_work *)calloc((size_t)threads, sizeof(mt_work));
  pthread_t *tid = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
  if (!w || !tid) return NULL;
  for (int t = 0; t < threads; t++) {
    w[t].bytes = bytes;
    w[t].offs = offs;
    w[t].r0 = n_reads * (uint64_t)t / (uint64_t)threads;
    w[t].r1 = n_reads * (uint64_t)(t + 1) / (uint64_t)threads;
    w[t].k = k;
    w[t].nl = nl;
    w[t].qcut = qual_cutoff;
    w[t].dmin = dmin_thres;
    w[t].dyn_mult = 1.0 - dyn_min_depth;
    w[t].nthreads = threads;
    w[t].range = (uint32_t)range;
    w[t].n_ranges = n_ranges < 1 ? 1u : (uint32_t)n_ranges;
    w[t].n_sel = (uint32_t)n_sel;
    w[t].bins = (mt_bin *)calloc((size_t)n_sel * MT_PARTS, sizeof(mt_bin));
    w[t].dig = dig ? (uint64_t *)calloc(MT_DIG * (size_t)n_sel, 8) : NULL;
    if (!w[t].bins || (dig && !w[t].dig)) return NULL;
  }
  for (uint64_t r = 0; r < n_reads; r++)
    if (offs[r + 1] < offs[r] || offs[r + 1] - offs[r] > 65535) return NULL;
  for (int t = 0; t < threads; t++) pthread_create(&tid[t], NULL, mt_extract, &w[t]);
  int fail = 0;
  mt_cbin *cbins = n_ctgs ? (mt_cbin *)calloc(MT_PARTS, sizeof(mt_cbin)) : NULL;
  if (n_ctgs && (!cbins || !mt_ctg_records(ctg_chars, ctg_offs, ctg_depths, n_ctgs, k, nl, (uint32_t)range,
                                           n_ranges < 1 ? 1u : (uint32_t)n_ranges, cbins)))
    fail = 1;
  for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
  for (int t = 0; t < threads; t++) fail |= w[t].fail;
  mt_shared sh;
  sh.w = w;
  sh.nthreads = threads;
  sh.next_part = 0;
  sh.n_part_bins = n_sel * MT_PARTS;
  sh.cbins = cbins;
  pthread_mutex_init(&sh.lock, NULL);
  mt_arg *args = (mt_arg *)calloc((size_t)threads, sizeof(mt_arg));
  if (!args) fail = 1;
  if (!fail) {
    for (int t = 0; t < threads; t++) {
      args[t].sh = &sh;
      args[t].me = t;
      pthread_create(&tid[t], NULL, mt_count, &args[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    for (int t = 0; t < threads; t++) fail |= w[t].fail;
  }
  pthread_mutex_destroy(&sh.lock);
  free(args);
  mt_table *out = fail ? NULL : (mt_table *)calloc(1, sizeof(mt_table));
  if (out) {
    uint64_t n = 0;
    for (int t = 0; t < threads; t++) n += w[t].n_out;
    out->n_longs = n_longs;
    out->n_out = n;
    out->out_keys = (uint64_t *)calloc(n + 1, 8 * (size_t)n_longs);
    out->out_counts = (uint16_t *)malloc((n + 1) * 2);
    out->out_left = (char *)malloc(n + 1);
    out->out_right = (char *)malloc(n + 1);
    if (!out->out_keys || !out->out_counts || !out->out_left || !out->out_right) {
      free(out->out_keys);
      free(out->out_counts);
      free(out->out_left);
      free(out->out_right);
      free(out);
      out = NULL;
    } else {
      uint64_t o = 0;
      for (int t = 0; t < threads; t++) {
        for (uint64_t i = 0; i < w[t].n_out; i++)
          memcpy(out->out_keys + (o + i) * n_longs, w[t].out_keys + i * nl, 8 * (size_t)nl);
        memcpy(out->out_counts + o, w[t].out_counts, 2 * w[t].n_out);
        memcpy(out->out_left + o, w[t].out_l, w[t].n_out);
        memcpy(out->out_right + o, w[t].out_r, w[t].n_out);
        o += w[t].n_out;
        out->occurrences += w[t].occ;
        out->n += w[t].distinct;
        out->purged += w[t].purged;
      }
      out->reads = n_reads;
    }
    if (out && dig) {
      memset(dig, 0, MT_DIG * 8 * (size_t)n_sel);
      for (int t = 0; t < threads; t++)
        for (int q = 0; q < MT_DIG * n_sel; q++) dig[q] = (q % MT_DIG == 1) ? dig[q] ^ w[t].dig[q] : dig[q] + w[t].dig[q];
    }
  }
  for (int t = 0; t < threads; t++) {
    for (int p = 0; p < n_sel * MT_PARTS; p++) {
      free(w[t].bins[p].keys);
      free(w[t].bins[p].ext);
    }
    free(w[t].bins);
    free(w[t].dig);
    free(w[t].out_keys);
    free(w[t].out_counts);
    free(w[t].out_l);
    free(w[t].out_r);
  }
  if (cbins) {
    for (int p = 0; p < MT_PARTS; p++) {
      free(cbins[p].keys);
      free(cbins[p].ext);
      free(cbins[p].depth);
    }
    free(cbins);
  }
  free(w);
  free(tid);
  return out;
}

mt_table *orc_kcount_mt_ctgs_range(const uint8_t *bytes, const uint64_t *offs, uint64_t n_reads, const char *ctg_chars,
                                   const uint64_t *ctg_offs, const uint16_t *ctg_depths, uint64_t n_ctgs, int k,
                                   int n_longs, int qual_cutoff, int dmin_thres, double dyn_min_depth, int threads,
                                   int range, int n_ranges) {
  return mt_run(bytes, offs, n_reads, ctg_chars, ctg_offs, ctg_depths, n_ctgs, k, n_longs, qual_cutoff, dmin_thres,
                dyn_min_depth, threads, range, n_ranges, 1, NULL);
}

/* Row-fingerprint digests (orc_row_fingerprints: MT_DIG words per range, see mt_run) of the key ranges [range, range +
 * n_sel) of n_ranges, from one extraction pass over the reads (the extraction is half of a range's time): the at-scale
 * gates compare them with the GPU's rows of the same ranges (orc_fp_digests) without building the tables. Returns 0,
 * or -1 on bad input or allocation failure. */
int orc_kcount_mt_digests(const uint8_t *bytes, const uint64_t *offs, uint64_t n_reads, int k, int qual_cutoff,
                          int dmin_thres, double dyn_min_depth, int threads, int range, int n_sel, int n_ranges,
                          uint64_t *dig) {
  mt_table *t = mt_run(bytes, offs, n_reads, NULL, NULL, NULL, 0, k, k / 32 + 1, qual_cutoff, dmin_thres,
                       dyn_min_depth, threads, range, n_ranges, n_sel, dig);
  if (!t) return -1;
  free(t->out_keys);
  free(t->out_counts);
  free(t->out_left);
  free(t->out_right);
  free(t);
  return 0;
}

/* The same digests of a GPU table's row fingerprints fps[n] by their key range parts[n] (orc_mt_ranges), ranges
 * [0, n_ranges): MT_DIG words each (distinct and occurrences left 0). */
void orc_fp_digests(const uint64_t *fps, const uint8_t *parts, uint64_t n, int n_ranges, uint64_t *dig) {
  memset(dig, 0, MT_DIG * 8 * (size_t)n_ranges);
  for (uint64_t i = 0; i < n; i++) {
    if (parts[i] >= n_ranges) continue;
    uint64_t *d = dig + MT_DIG * (size_t)parts[i];
    d[0]++;
    d[1] ^= fps[i];
    d[2] += fps[i];
    d[3] += mt_fmix(fps[i]);
  }
}

mt_table *orc_kcount_mt_range(const uint8_t *bytes, const uint64_t *offs, uint64_t n_reads, int k, int n_longs,
                              int qual_cutoff, int dmin_thres, double dyn_min_depth, int threads, int range,
                              int n_ranges) {
  return orc_kcount_mt_ctgs_range(bytes, offs, n_reads, NULL, NULL, NULL, 0, k, n_longs, qual_cutoff, dmin_thres,
                                  dyn_min_depth, threads, range, n_ranges);
}

/* The whole table (one range). */
mt_table *orc_kcount_mt(const uint8_t *bytes, const uint64_t *offs, uint64_t n_reads, int k, int n_longs,
                        int qual_cutoff, int dmin_thres, double dyn_min_depth, int threads) {
  return orc_kcount_mt_range(bytes, offs, n_reads, k, n_longs, qual_cutoff, dmin_thres, dyn_min_depth, threads, 0, 1);
}

/* mt_range of n keys (stride words per row, the first nl used) into out[n]: the part of each row of a GPU table. */
void orc_mt_ranges(const uint64_t *keys, uint64_t n, int stride, int nl, int n_ranges, uint8_t *out) {
  for (uint64_t i = 0; i < n; i++) out[i] = (uint8_t)mt_range(keys + i * (uint64_t)stride, nl, (uint32_t)n_ranges);
}

/* A 64-bit fingerprint of every row (key words, count, left, right) into out[n]: sorted, two tables' fingerprint
 * lists are compared element by element (equal tables give equal lists; a differing row changes its fingerprint). */
void orc_row_fingerprints(const uint64_t *keys, const uint16_t *counts, const char *left, const char *right, uint64_t n,
                          int stride, int nl, uint64_t *out) {
  for (uint64_t i = 0; i < n; i++) {
    uint64_t h = 0x243F6A8885A308D3ULL;
    for (int w = 0; w < nl; w++) h = mt_fmix(h ^ keys[i * (uint64_t)stride + w]) + 0x9E3779B97F4A7C15ULL;
    h = mt_fmix(h ^ ((uint64_t)counts[i] | (uint64_t)(uint8_t)left[i] << 16 | (uint64_t)(uint8_t)right[i] << 24));
    out[i] = h;
  }
}
