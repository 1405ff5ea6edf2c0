/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. Not part of the product.
 *
 * Plain-C restatement of the reference's CPU kcount read pass at one rank (ajpowelsnl/mhm2_proxy,
 * src/kcount/kcount_cpu.cpp with src/kmer.cpp, src/hash_funcs.c, src/packed_reads.cpp), used as the
 * checker for the HIP path. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it. It deliberately shares no code with mhm2_proxy_amd/.
 *
 * Pinning: MurmurHash3/quick_hash are checked bit-for-bit against the reference's own
 * hash_funcs.c compiled into oracle/_ref/ (the only reference source on this path that builds without
 * stand-ins); the Kmer layer against SURVEY.md Appendix A known answers and the invariants of the
 * reference's test/kmer-test.cpp; the count/extension rules against a literal string-level Python
 * restatement (tests/ref_literal.py). The reference kcount itself needs UPC++ headers that the image
 * lacks, so count tables are not pinned by reference-generated vectors ("parity partially pinned").
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------------------------------------
 * MurmurHash3_x64_128 (src/hash_funcs.c:65-170), seed 313 for the 64-bit variant (:185-190). */

static uint64_t rotl64(uint64_t x, int8_t r) { return (x << r) | (x >> (64 - r)); }

static uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}

void orc_murmur3_x64_128(const void *key, uint32_t len, uint32_t seed, void *out) {
  const uint8_t *data = (const uint8_t *)key;
  const uint32_t nblocks = len / 16;
  uint64_t h1 = seed, h2 = seed;
  const uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
  for (uint32_t i = 0; i < nblocks; i++) {
    uint64_t k1, k2;
    memcpy(&k1, data + 16 * i, 8);
    memcpy(&k2, data + 16 * i + 8, 8);
    k1 *= c1;
    k1 = rotl64(k1, 31);
    k1 *= c2;
    h1 ^= k1;
    h1 = rotl64(h1, 27);
    h1 += h2;
    h1 = h1 * 5 + 0x52dce729;
    k2 *= c2;
    k2 = rotl64(k2, 33);
    k2 *= c1;
    h2 ^= k2;
    h2 = rotl64(h2, 31);
    h2 += h1;
    h2 = h2 * 5 + 0x38495ab5;
  }
  const uint8_t *tail = data + nblocks * 16;
  uint64_t k1 = 0, k2 = 0;
  switch (len & 15) {
    case 15: k2 ^= (uint64_t)tail[14] << 48; /* fall through */
    case 14: k2 ^= (uint64_t)tail[13] << 40; /* fall through */
    case 13: k2 ^= (uint64_t)tail[12] << 32; /* fall through */
    case 12: k2 ^= (uint64_t)tail[11] << 24; /* fall through */
    case 11: k2 ^= (uint64_t)tail[10] << 16; /* fall through */
    case 10: k2 ^= (uint64_t)tail[9] << 8; /* fall through */
    case 9:
      k2 ^= (uint64_t)tail[8];
      k2 *= c2;
      k2 = rotl64(k2, 33);
      k2 *= c1;
      h2 ^= k2;
      /* fall through */
    case 8: k1 ^= (uint64_t)tail[7] << 56; /* fall through */
    case 7: k1 ^= (uint64_t)tail[6] << 48; /* fall through */
    case 6: k1 ^= (uint64_t)tail[5] << 40; /* fall through */
    case 5: k1 ^= (uint64_t)tail[4] << 32; /* fall through */
    case 4: k1 ^= (uint64_t)tail[3] << 24; /* fall through */
    case 3: k1 ^= (uint64_t)tail[2] << 16; /* fall through */
    case 2: k1 ^= (uint64_t)tail[1] << 8; /* fall through */
    case 1:
      k1 ^= (uint64_t)tail[0];
      k1 *= c1;
      k1 = rotl64(k1, 31);
      k1 *= c2;
      h1 ^= k1;
  }
  h1 ^= len;
  h2 ^= len;
  h1 += h2;
  h2 += h1;
  h1 = fmix64(h1);
  h2 = fmix64(h2);
  h1 += h2;
  h2 += h1;
  ((uint64_t *)out)[0] = h1;
  ((uint64_t *)out)[1] = h2;
}

uint64_t orc_murmur3_x64_64(const void *key, uint32_t len) {
  uint64_t t[2];
  orc_murmur3_x64_128(key, len, 313, t);
  return t[0];
}

/* quick_hash (src/hash_funcs.c:332-342) */
uint64_t orc_quick_hash(uint64_t v) {
  v = v * 3935559000370003845ULL + 2691343689449507681ULL;
  v ^= v >> 21;
  v ^= v << 37;
  v ^= v >> 4;
  v *= 4768777513237032717ULL;
  v ^= v << 20;
  v ^= v >> 41;
  v ^= v << 5;
  return v;
}

/* ---------------------------------------------------------------------------------------------
 * Kmer<MAX_K> with runtime n_longs (src/kmer.hpp:61-160, src/kmer.cpp). */

static uint64_t twin_table[256];
static uint64_t zero_mask[32];
static int tables_ready = 0;

static void init_tables(void) {
  if (tables_ready) return;
  /* TWIN_TABLE (src/kmer.cpp:66-79): reverse complement of the 4 bases packed in a byte */
  for (int b = 0; b < 256; b++) {
    int out = 0;
    for (int j = 0; j < 4; j++) {
      int base = (b >> (6 - 2 * j)) & 3;
      out |= (3 - base) << (2 * j);
    }
    twin_table[b] = (uint64_t)out;
  }
  /* ZERO_MASK (src/kmer.cpp:81-87): top 2*m bits */
  for (int m = 0; m < 32; m++) zero_mask[m] = m ? ~(~0ULL >> (2 * m)) : 0;
  tables_ready = 1;
}

/* The encoding bit trick of get_kmers/set_kmer (src/kmer.cpp:187-188,284-285): A0 C1 G2 T3, N->G. */
static uint64_t base_code(char c) {
  uint64_t x = ((uint64_t)c & 4) >> 1;
  return x + ((x ^ ((uint64_t)c & 2)) >> 1);
}

/* set_kmer (src/kmer.cpp:274-296) */
void orc_kmer_from_string(const char *s, int k, int n_longs, uint64_t *longs) {
  memset(longs, 0, 8 * (size_t)n_longs);
  for (int i = 0; i < k; i++) longs[i / 32] |= base_code(s[i]) << (2 * (31 - i % 32));
}

/* to_string / mer_to_string (src/kmer.cpp:595-634) */
void orc_kmer_to_string(const uint64_t *longs, int k, char *out) {
  static const char m[4] = {'A', 'C', 'G', 'T'};
  for (int i = 0; i < k; i++) out[i] = m[(longs[i / 32] >> (2 * (31 - i % 32))) & 3];
  out[k] = 0;
}

/* revcomp (src/kmer.cpp:485-505) */
void orc_kmer_revcomp(const uint64_t *longs, int k, int n_longs, uint64_t *out) {
  init_tables();
  uint64_t km[8] = {0};
  const int last_long = (k + 31) / 32;
  for (int i = 0; i < last_long; i++) {
    uint64_t v = longs[i];
    km[last_long - 1 - i] = (twin_table[v & 0xFF] << 56) | (twin_table[(v >> 8) & 0xFF] << 48) |
                            (twin_table[(v >> 16) & 0xFF] << 40) | (twin_table[(v >> 24) & 0xFF] << 32) |
                            (twin_table[(v >> 32) & 0xFF] << 24) | (twin_table[(v >> 40) & 0xFF] << 16) |
                            (twin_table[(v >> 48) & 0xFF] << 8) | (twin_table[(v >> 56)]);
  }
  const uint64_t shift = (k % 32) ? 2 * (32 - (k % 32)) : 0;
  const uint64_t shiftmask = (k % 32) ? (((((uint64_t)1) << shift) - 1) << (64 - shift)) : 0;
  if (shift) { /* (the reference shifts by 64 - 0 when k % 32 == 0, which is a no-op on its zero mask) */
    km[0] = km[0] << shift;
    for (int i = 1; i < last_long; i++) {
      km[i - 1] |= (km[i] & shiftmask) >> (64 - shift);
      km[i] = km[i] << shift;
    }
  }
  memcpy(out, km, 8 * (size_t)n_longs);
}

/* operator< (src/kmer.cpp:265-272) */
static int kmer_less(const uint64_t *a, const uint64_t *b, int n) {
  for (int i = 0; i < n; i++) {
    if (a[i] < b[i]) return 1;
    if (a[i] > b[i]) return 0;
  }
  return 0;
}

/* hash (src/kmer.cpp:465-468) */
uint64_t orc_kmer_hash(const uint64_t *longs, int n_longs) { return orc_murmur3_x64_64(longs, 8 * (uint32_t)n_longs); }

/* get_minimizer_fast with revcomp candidates (src/kmer.cpp:344-393, 395-403) */
uint64_t orc_get_minimizer_fast(const uint64_t *longs, int k, int n_longs, int m, int least_complement) {
  init_tables();
  uint64_t rcl[8] = {0};
  if (least_complement) orc_kmer_revcomp(longs, k, n_longs, rcl);
  const int chunk_step = 32 - ((m + 3) / 4) * 4;
  const int num_candidates = least_complement ? k - m + 1 : 1;
  uint64_t rc_cand[128];
  if (least_complement) {
    for (int base = 0; base <= k - m; base += chunk_step) {
      int shift = base % 32, l = base / 32;
      uint64_t tmp = rcl[l];
      if (shift) {
        tmp = tmp << (shift * 2);
        if (l < n_longs - 1) tmp |= rcl[l + 1] >> (64 - shift * 2);
      }
      for (int j = 0; j < chunk_step; j++) {
        if (base + j + m > k) break;
        rc_cand[base + j] = (tmp << (j * 2)) & zero_mask[m];
      }
    }
  }
  uint64_t minimizer = 0;
  for (int base = 0; base <= k - m; base += chunk_step) {
    int shift = base % 32, l = base / 32;
    uint64_t tmp = longs[l];
    if (shift) {
      tmp = tmp << (shift * 2);
      if (l < n_longs - 1) tmp |= longs[l + 1] >> (64 - shift * 2);
    }
    for (int j = 0; j < chunk_step; j++) {
      if (base + j + m > k) break;
      uint64_t fwd = (tmp << (j * 2)) & zero_mask[m];
      uint64_t rcc = least_complement ? rc_cand[num_candidates - base - j - 1] : fwd;
      uint64_t least = fwd < rcc ? fwd : rcc;
      if (least > minimizer) minimizer = least;
    }
  }
  return minimizer;
}

/* minimizer_hash_fast (src/kmer.cpp:454-463) */
uint64_t orc_minimizer_hash_fast(const uint64_t *longs, int k, int n_longs, int m) {
  return orc_quick_hash(orc_get_minimizer_fast(longs, k, n_longs, m, 1));
}

/* KmerDHT minimizer length (src/kcount/kmer_dht.cpp:114-116) and owner rank (:193-196) */
int orc_minimizer_len(int k) {
  int m = k * 2 / 3 + 1;
  if (m < 15) m = 15;
  if (m > 27) m = 27;
  return m;
}
int orc_kmer_target_rank(const uint64_t *longs, int k, int n_longs, int rank_n) {
  return (int)(orc_minimizer_hash_fast(longs, k, n_longs, orc_minimizer_len(k)) % (uint64_t)rank_n);
}

/* orc_kmer_target_rank of n keys (stride words per row) into out[n]. */
void orc_kmer_target_ranks(const uint64_t *keys, uint64_t n, int stride, int k, int n_longs, int rank_n, uint8_t *out) {
  for (uint64_t i = 0; i < n; i++) out[i] = (uint8_t)orc_kmer_target_rank(keys + i * (uint64_t)stride, k, n_longs, rank_n);
}

/* ---------------------------------------------------------------------------------------------
 * ExtCounts / KmerExtsCounts (src/kcount/kcount_cpu.cpp:115-200) */

typedef struct {
  uint16_t count;
  uint16_t left[4];  /* A C G T */
  uint16_t right[4];
  uint8_t from_ctg; /* KmerExtsCounts::from_ctg (kcount_cpu.cpp:191-196) */
} ext_counts;

static uint16_t inc_with_limit(int c1, int c2) { /* :148-151 */
  int c = c1 + c2;
  return (uint16_t)(c < 65535 ? c : 65535);
}

static void ext_inc(uint16_t *e, char ext, int count) { /* :152-164 */
  switch (ext) {
    case 'A': e[0] = inc_with_limit(e[0], count); break;
    case 'C': e[1] = inc_with_limit(e[1], count); break;
    case 'G': e[2] = inc_with_limit(e[2], count); break;
    case 'T': e[3] = inc_with_limit(e[3], count); break;
  }
}

/* get_ext (:173-182) with get_sorted (:133-145): descending count, ties -> higher char first */
static char get_ext(const uint16_t *e, uint16_t count, int dmin_thres, double dyn_min_depth) {
  char ch[4] = {'A', 'C', 'G', 'T'};
  int cnt[4] = {e[0], e[1], e[2], e[3]};
  for (int i = 1; i < 4; i++) { /* insertion sort with the reference comparator */
    char c = ch[i];
    int v = cnt[i];
    int j = i - 1;
    while (j >= 0 && (cnt[j] < v || (cnt[j] == v && ch[j] < c))) {
      ch[j + 1] = ch[j];
      cnt[j + 1] = cnt[j];
      j--;
    }
    ch[j + 1] = c;
    cnt[j + 1] = v;
  }
  int dmin_dyn = (int)((1.0 - dyn_min_depth) * count);
  if (dmin_dyn < dmin_thres) dmin_dyn = dmin_thres;
  if (cnt[0] < dmin_dyn) return 'X';
  if (cnt[1] >= dmin_dyn) return 'F';
  return ch[0];
}

/* comp_nucleotide (src/utils.cpp:121-143) restricted to the characters that reach it */
static char comp_nucleotide(char c) {
  switch (c) {
    case 'A': return 'T';
    case 'C': return 'G';
    case 'G': return 'C';
    case 'T': return 'A';
    case 'N': return 'N';
    case '0': return '0';
  }
  return 'N';
}

/* ---------------------------------------------------------------------------------------------
 * Open-addressing table keyed by the canonical k-mer (stand-in for KmerMapExts, kcount_cpu.cpp:205-294;
 * its slot order does not affect the result, and it never drops: it grows instead). */

typedef struct orc_table {
  int n_longs;
  uint64_t cap, n;
  uint64_t *keys;   /* [cap * n_longs] */
  ext_counts *vals; /* [cap] */
  uint8_t *used;
  /* finalized output (sorted by key) */
  uint64_t n_out;
  uint64_t *out_keys;
  uint16_t *out_counts;
  char *out_left, *out_right;
  uint64_t occurrences, purged, reads;
} orc_table;

static int tbl_init(orc_table *t, int n_longs, uint64_t cap) {
  memset(t, 0, sizeof *t);
  t->n_longs = n_longs;
  t->cap = cap;
  t->keys = (uint64_t *)malloc(cap * 8 * n_longs);
  t->vals = (ext_counts *)calloc(cap, sizeof(ext_counts));
  t->used = (uint8_t *)calloc(cap, 1);
  return t->keys && t->vals && t->used;
}

static ext_counts *tbl_get2(orc_table *t, const uint64_t *key, int *is_new);
static ext_counts *tbl_get(orc_table *t, const uint64_t *key) { return tbl_get2(t, key, NULL); }

static int tbl_grow(orc_table *t) {
  orc_table nt;
  if (!tbl_init(&nt, t->n_longs, t->cap * 2)) return 0;
  for (uint64_t i = 0; i < t->cap; i++) {
    if (!t->used[i]) continue;
    ext_counts *v = tbl_get(&nt, t->keys + i * t->n_longs);
    *v = t->vals[i];
  }
  free(t->keys);
  free(t->vals);
  free(t->used);
  t->keys = nt.keys;
  t->vals = nt.vals;
  t->used = nt.used;
  t->cap = nt.cap;
  return 1;
}

static ext_counts *tbl_get2(orc_table *t, const uint64_t *key, int *is_new) {
  if (is_new) *is_new = 0;
  if ((t->n + 1) * 10 > t->cap * 7) {
    if (!tbl_grow(t)) return NULL;
  }
  const int nl = t->n_longs;
  uint64_t s = orc_kmer_hash(key, nl) & (t->cap - 1);
  while (t->used[s]) {
    if (memcmp(t->keys + s * nl, key, 8 * (size_t)nl) == 0) return &t->vals[s];
    s = (s + 1) & (t->cap - 1);
  }
  t->used[s] = 1;
  memcpy(t->keys + s * nl, key, 8 * (size_t)nl);
  t->n++;
  if (is_new) *is_new = 1;
  return &t->vals[s];
}

static int g_sort_nl;
static const uint64_t *g_sort_keys;
static int cmp_idx(const void *a, const void *b) {
  const uint64_t ia = *(const uint64_t *)a, ib = *(const uint64_t *)b;
  const uint64_t *ka = g_sort_keys + ia * g_sort_nl, *kb = g_sort_keys + ib * g_sort_nl;
  for (int i = 0; i < g_sort_nl; i++) {
    if (ka[i] < kb[i]) return -1;
    if (ka[i] > kb[i]) return 1;
  }
  return 0;
}

/* insert_into_local_hashtable (src/kcount/kcount_cpu.cpp:490-528): purge count < 2 and X/X */
static int tbl_finalize(orc_table *t, int dmin_thres, double dyn_min_depth) {
  const int nl = t->n_longs;
  uint64_t *idx = (uint64_t *)malloc((t->n + 1) * 8);
  if (!idx) return 0;
  uint64_t m = 0;
  for (uint64_t i = 0; i < t->cap; i++) {
    if (!t->used[i]) continue;
    const ext_counts *v = &t->vals[i];
    if (v->count < 2) {
      t->purged++;
      continue;
    }
    char l = get_ext(v->left, v->count, dmin_thres, dyn_min_depth);
    char r = get_ext(v->right, v->count, dmin_thres, dyn_min_depth);
    if (l == 'X' && r == 'X') {
      t->purged++;
      continue;
    }
    idx[m++] = i;
  }
  g_sort_nl = nl;
  g_sort_keys = t->keys;
  qsort(idx, m, 8, cmp_idx);
  t->n_out = m;
  t->out_keys = (uint64_t *)malloc((m + 1) * 8 * nl);
  t->out_counts = (uint16_t *)malloc((m + 1) * 2);
  t->out_left = (char *)malloc(m + 1);
  t->out_right = (char *)malloc(m + 1);
  for (uint64_t j = 0; j < m; j++) {
    const uint64_t i = idx[j];
    const ext_counts *v = &t->vals[i];
    memcpy(t->out_keys + j * nl, t->keys + i * nl, 8 * (size_t)nl);
    t->out_counts[j] = v->count;
    t->out_left[j] = get_ext(v->left, v->count, dmin_thres, dyn_min_depth);
    t->out_right[j] = get_ext(v->right, v->count, dmin_thres, dyn_min_depth);
  }
  free(idx);
  return 1;
}

/* ---------------------------------------------------------------------------------------------
 * The read pass. */

/* Kmer::get_kmers of one string (src/kmer.cpp:155-257) for window i, via set_kmer semantics. */
static void window_kmer(const char *seq, int i, int k, int n_longs, uint64_t *out) {
  orc_kmer_from_string(seq + i, k, n_longs, out);
}

/* get_kmers_and_exts + insert_supermer_from_read (src/kcount/kcount_cpu.cpp:307-354) for one
 * supermer whose case encodes quality; count = supermer count (1 for reads). */
static int insert_supermer(orc_table *t, char *sm, int len, int k, int count) {
  const int nl = t->n_longs;
  char quals[65536];
  for (int i = 0; i < len; i++) {
    char b = sm[i];
    char u = (b >= 'a' && b <= 'z') ? (char)(b - 32) : b;
    if (u != 'A' && u != 'C' && u != 'G' && u != 'T' && u != 'N') return 0; /* DIE, :453-458 */
    quals[i] = (b >= 'A' && b <= 'Z');
    sm[i] = u;
  }
  uint64_t kmer[8], rc[8];
  for (int i = 1; i < len - k; i++) {
    window_kmer(sm, i, k, nl, kmer);
    char left = quals[i - 1] ? sm[i - 1] : '0';
    char right = quals[i + k] ? sm[i + k] : '0';
    orc_kmer_revcomp(kmer, k, nl, rc);
    if (kmer_less(rc, kmer, nl)) {
      memcpy(kmer, rc, 8 * (size_t)nl);
      char tmp = left;
      left = comp_nucleotide(right);
      right = comp_nucleotide(tmp);
    }
    ext_counts *v = tbl_get(t, kmer);
    if (!v) return 0;
    int c = v->count + count;
    v->count = (uint16_t)(c > 65535 ? 65535 : c);
    ext_inc(v->left, left, count);
    ext_inc(v->right, right, count);
    t->occurrences++;
  }
  return 1;
}

/* analyze_kmers read pass at rank_n()==1 (src/kcount/kcount.cpp:54-98,140-157 ->
 * SeqBlockInserter::process_seq, kcount_cpu.cpp:73-103, whose single supermer is the whole read when
 * L >= k+2). bytes/offs use the PackedRead byte layout (src/packed_reads.cpp:73-109,147-159).
 * Returns NULL on bad input (the reference DIEs). */
orc_table *orc_kcount(const uint8_t *bytes, const uint64_t *offs, uint64_t n_reads, int k, int n_longs,
                      int qual_cutoff, int dmin_thres, double dyn_min_depth) {
  static const char nucleotide_map[5] = {'A', 'C', 'G', 'T', 'N'};
  init_tables();
  if (k < 1 || n_longs < (k + 31) / 32 || n_longs > 8) return NULL;
  orc_table *t = (orc_table *)malloc(sizeof(orc_table));
  if (!t || !tbl_init(t, n_longs, 1 << 16)) return NULL;
  char seq[65536];
  for (uint64_t r = 0; r < n_reads; r++) {
    const uint64_t L64 = offs[r + 1] - offs[r];
    if (L64 > 65535) return NULL;
    const int L = (int)L64;
    t->reads++;
    for (int i = 0; i < L; i++) {
      const uint8_t b = bytes[offs[r] + i];
      if ((b & 7) > 4) return NULL;
      seq[i] = nucleotide_map[b & 7];          /* PackedRead::unpack */
      if ((b >> 3) < qual_cutoff) seq[i] += 32; /* count_kmers lowercasing (tolower), kcount.cpp:80-85 */
    }
    if (L < k) continue;         /* kcount.cpp:78 */
    if (L < k + 2) continue;     /* process_seq emits the supermer only when length >= k+2 */
    if (!insert_supermer(t, seq, L, k, 1)) return NULL;
  }
  if (!tbl_finalize(t, dmin_thres, dyn_min_depth)) return NULL;
  return t;
}

/* ---------------------------------------------------------------------------------------------
 * The contig pass: add_ctg_kmers (src/kcount/kcount.cpp:100-138) -> SeqBlockInserter::process_seq with
 * count = depth (kcount_cpu.cpp:73-103: depth 0 -> 1; one supermer per contig at one rank) ->
 * insert_supermer_from_ctg (kcount_cpu.cpp:356-406), applied in contig order after the read pass.
 * Literal restatement, order-dependent exactly as the reference is. */
static int insert_ctg_supermer(orc_table *t, char *sm, int len, int k, int count, int dmin_thres,
                               double dyn_min_depth) {
  const int nl = t->n_longs;
  char quals[65536];
  for (int i = 0; i < len; i++) { /* get_kmers_and_exts, kcount_cpu.cpp:307-335 */
    char b = sm[i];
    char u = (b >= 'a' && b <= 'z') ? (char)(b - 32) : b;
    if (u != 'A' && u != 'C' && u != 'G' && u != 'T' && u != 'N') return 0; /* DIE, :453-458 */
    quals[i] = (b >= 'A' && b <= 'Z');
    sm[i] = u;
  }
  uint64_t kmer[8], rc[8];
  for (int i = 1; i < len - k; i++) {
    window_kmer(sm, i, k, nl, kmer);
    char left = quals[i - 1] ? sm[i - 1] : '0';
    char right = quals[i + k] ? sm[i + k] : '0';
    orc_kmer_revcomp(kmer, k, nl, rc);
    if (kmer_less(rc, kmer, nl)) {
      memcpy(kmer, rc, 8 * (size_t)nl);
      char tmp = left;
      left = comp_nucleotide(right);
      right = comp_nucleotide(tmp);
    }
    int is_new = 0;
    ext_counts *v = tbl_get2(t, kmer, &is_new); /* KmerMapExts::insert(kmer, true): never full here */
    if (!v) return 0;
    int insert_it = 0;
    int c = count;
    if (is_new) {
      insert_it = 1;
    } else if (!v->from_ctg) { /* existing entry is from a read */
      if (v->count == 1) {
        insert_it = 1;
      } else {
        const char l = get_ext(v->left, v->count, dmin_thres, dyn_min_depth);
        const char r = get_ext(v->right, v->count, dmin_thres, dyn_min_depth);
        if (l == 'X' || l == 'F' || r == 'X' || r == 'F') insert_it = 1; /* non-UU */
      }
    } else if (v->count) { /* existing entry from a contig */
      insert_it = 1;
      const char l = get_ext(v->left, v->count, dmin_thres, dyn_min_depth);
      const char r = get_ext(v->right, v->count, dmin_thres, dyn_min_depth);
      if (l != left || r != right)
        c = 0; /* the two contig k-mers disagree: purge later */
      else
        c = c < v->count ? c : v->count;
    }
    if (insert_it) {
      memset(v, 0, sizeof *v);
      v->count = (uint16_t)c;
      v->from_ctg = 1;
      ext_inc(v->left, left, c);
      ext_inc(v->right, right, c);
    }
  }
  return 1;
}

/* Read pass + contig pass + finalize. ctg_chars: contigs back to back (case = quality, as for reads),
 * ctg_offs: n_ctgs + 1 offsets, ctg_depths: Contig::get_uint16_t_depth() values (contigs.hpp:65). */
orc_table *orc_kcount_ctgs(const uint8_t *bytes, const uint64_t *offs, uint64_t n_reads, const char *ctg_chars,
                           const uint64_t *ctg_offs, const uint16_t *ctg_depths, uint64_t n_ctgs, int k, int n_longs,
                           int qual_cutoff, int dmin_thres, double dyn_min_depth) {
  static const char nucleotide_map[5] = {'A', 'C', 'G', 'T', 'N'};
  init_tables();
  if (k < 1 || n_longs < (k + 31) / 32 || n_longs > 8) return NULL;
  orc_table *t = (orc_table *)malloc(sizeof(orc_table));
  if (!t || !tbl_init(t, n_longs, 1 << 16)) return NULL;
  char seq[65536];
  for (uint64_t r = 0; r < n_reads; r++) { /* the read pass, as orc_kcount */
    const uint64_t L64 = offs[r + 1] - offs[r];
    if (L64 > 65535) return NULL;
    const int L = (int)L64;
    t->reads++;
    for (int i = 0; i < L; i++) {
      const uint8_t b = bytes[offs[r] + i];
      if ((b & 7) > 4) return NULL;
      seq[i] = nucleotide_map[b & 7];
      if ((b >> 3) < qual_cutoff) seq[i] += 32;
    }
    if (L < k + 2) continue;
    if (!insert_supermer(t, seq, L, k, 1)) return NULL;
  }
  static char cseq[1 << 20];
  for (uint64_t c = 0; c < n_ctgs; c++) { /* add_ctg_kmers, contig order */
    const uint64_t L64 = ctg_offs[c + 1] - ctg_offs[c];
    if (L64 >= sizeof cseq) return NULL;
    const int L = (int)L64;
    if (L < k + 2) continue; /* kcount.cpp:128 */
    memcpy(cseq, ctg_chars + ctg_offs[c], (size_t)L);
    const int depth = ctg_depths[c] ? ctg_depths[c] : 1; /* process_seq: if (!depth) depth = 1 */
    if (!insert_ctg_supermer(t, cseq, L, k, depth, dmin_thres, dyn_min_depth)) return NULL;
  }
  if (!tbl_finalize(t, dmin_thres, dyn_min_depth)) return NULL;
  return t;
}

/* ---------------------------------------------------------------------------------------------
 * Record path used by the multi-rank tests: extraction of (canonical key, ext code) records and
 * counting of a record set. ext code = (left << 3) | right with A0 C1 G2 T3, 4 = none. */

static int ext_to_code(char c) {
  switch (c) {
    case 'A': return 0;
    case 'C': return 1;
    case 'G': return 2;
    case 'T': return 3;
  }
  return 4;
}

/* Returns the number of records written (or -1 on bad input / overflow of cap). */
int64_t orc_extract(const uint8_t *bytes, const uint64_t *offs, uint64_t n_reads, int k, int n_longs, int qual_cutoff,
                    uint64_t *keys_out, uint8_t *ext_out, uint64_t cap) {
  static const char nucleotide_map[5] = {'A', 'C', 'G', 'T', 'N'};
  init_tables();
  char seq[65536], quals[65536];
  uint64_t n = 0;
  uint64_t kmer[8], rc[8];
  for (uint64_t r = 0; r < n_reads; r++) {
    const int L = (int)(offs[r + 1] - offs[r]);
    if (L < k + 2) continue;
    for (int i = 0; i < L; i++) {
      const uint8_t b = bytes[offs[r] + i];
      if ((b & 7) > 4) return -1;
      seq[i] = nucleotide_map[b & 7];
      quals[i] = (b >> 3) >= qual_cutoff;
    }
    for (int i = 1; i < L - k; i++) {
      window_kmer(seq, i, k, n_longs, kmer);
      char left = quals[i - 1] ? seq[i - 1] : '0';
      char right = quals[i + k] ? seq[i + k] : '0';
      orc_kmer_revcomp(kmer, k, n_longs, rc);
      if (kmer_less(rc, kmer, n_longs)) {
        memcpy(kmer, rc, 8 * (size_t)n_longs);
        char tmp = left;
        left = comp_nucleotide(right);
        right = comp_nucleotide(tmp);
      }
      if (n >= cap) return -1;
      memcpy(keys_out + n * n_longs, kmer, 8 * (size_t)n_longs);
      ext_out[n] = (uint8_t)((ext_to_code(left) << 3) | ext_to_code(right));
      n++;
    }
  }
  return (int64_t)n;
}

orc_table *orc_count_records(const uint64_t *keys, const uint8_t *exts, uint64_t n, int n_longs, int dmin_thres,
                             double dyn_min_depth) {
  static const char code_char[5] = {'A', 'C', 'G', 'T', '0'};
  init_tables();
  orc_table *t = (orc_table *)malloc(sizeof(orc_table));
  if (!t || !tbl_init(t, n_longs, 1 << 16)) return NULL;
  for (uint64_t i = 0; i < n; i++) {
    ext_counts *v = tbl_get(t, keys + i * n_longs);
    if (!v) return NULL;
    int c = v->count + 1;
    v->count = (uint16_t)(c > 65535 ? 65535 : c);
    ext_inc(v->left, code_char[exts[i] >> 3 > 4 ? 4 : exts[i] >> 3], 1);
    ext_inc(v->right, code_char[(exts[i] & 7) > 4 ? 4 : (exts[i] & 7)], 1);
    t->occurrences++;
  }
  if (!tbl_finalize(t, dmin_thres, dyn_min_depth)) return NULL;
  return t;
}

/* ---------------------------------------------------------------------------------------------
 * accessors */

uint64_t orc_table_size(const orc_table *t) { return t ? t->n_out : 0; }

void orc_table_fetch(const orc_table *t, uint64_t *keys, uint16_t *counts, char *left, char *right) {
  if (keys) memcpy(keys, t->out_keys, t->n_out * 8 * t->n_longs);
  if (counts) memcpy(counts, t->out_counts, t->n_out * 2);
  if (left) memcpy(left, t->out_left, t->n_out);
  if (right) memcpy(right, t->out_right, t->n_out);
}

/* stats: [0] occurrences, [1] distinct, [2] purged, [3] n_out, [4] reads */
void orc_table_stats(const orc_table *t, uint64_t *s) {
  s[0] = t->occurrences;
  s[1] = t->n;
  s[2] = t->purged;
  s[3] = t->n_out;
  s[4] = t->reads;
}

void orc_table_free(orc_table *t) {
  if (!t) return;
  free(t->keys);
  free(t->vals);
  free(t->used);
  free(t->out_keys);
  free(t->out_counts);
  free(t->out_left);
  free(t->out_right);
  free(t);
}

/* Kmer::hash of n keys (vectorised helper for the multi-rank protocol tests) */
void orc_kmer_hash_many(const uint64_t *keys, uint64_t n, int n_longs, uint64_t *out) {
  for (uint64_t i = 0; i < n; i++) out[i] = orc_kmer_hash(keys + i * n_longs, n_longs);
}

/* ---------------------------------------------------------------------------------------------
 * FASTQ ingest: FastqReader::get_next_fq_record (src/fastq.cpp:504-551) with
 * rtrim (:67-71) and get_fq_name (:73-122), then the PackedRead constructor (src/packed_reads.cpp:73-109).
 * Records are read 4 lines at a time with fgets into a BUF_SIZE = 2047 buffer (src/fastq.hpp:61): a line
 * longer than 2045 characters would be split by fgets and is reported as unsupported here.
 * Error kinds (the first failing record, in file order; within a record in this order), all a DIE in the
 * reference: 1 id line without '@' (:539), 2 third line without '+' (:540), 3 name format (:542),
 * 4 sequence / quality length mismatch (:545), 5 line too long, 6 illegal base (packed_reads.cpp:104),
 * 7 file ends inside a record (:525). rtrim of an all-whitespace line is undefined behaviour in the
 * reference (size_t underflow); here it yields the empty string. */

static int fq_isspace(unsigned char c) { return c == ' ' || (c >= '\t' && c <= '\r'); }

static uint64_t fq_rtrim(const char *s, uint64_t b, uint64_t e) { /* :67-71 */
  while (e > b && fq_isspace((unsigned char)s[e - 1])) e--;
  return e;
}

/* get_fq_name's verdict on the rtrimmed id line [b, e) (which starts with '@') */
static int fq_name_ok(const char *s, uint64_t b, uint64_t e) {
  const char *h = s + b + 1; /* header.erase(0, 1) */
  const uint64_t len = fq_rtrim(s, b + 1, e) - (b + 1);
  if (len >= 3 && h[len - 2] != '/') {
    if (h[len - 2] == 'R') return 1; /* HudsonAlpha -R1 / -R2 */
    uint64_t end_pos = len;
    for (uint64_t i = 0; i < len; i++)
      if (h[i] == '\t') { end_pos = i; break; }
    if (end_pos == len) {
      for (uint64_t i = 0; i < len; i++)
        if (h[i] == ' ') { end_pos = i; break; }
      if (end_pos == len) return 1; /* no comment */
    }
    if (end_pos > 3 && h[end_pos - 2] == '/' && (h[end_pos - 1] == '1' || h[end_pos - 1] == '2')) return 1;
    if (len < end_pos + 7 || h[end_pos + 2] != ':' || h[end_pos + 4] != ':' || h[end_pos + 6] != ':' ||
        (h[end_pos + 1] != '1' && h[end_pos + 1] != '2'))
      return 0;
  }
  return 1;
}

static int fq_code(char c) { /* PackedRead::PackedRead switch, packed_reads.cpp:87-105 */
  switch (c) {
    case 'A': return 0;
    case 'C': return 1;
    case 'G': return 2;
    case 'T': return 3;
    case 'N': case 'U': case 'R': case 'Y': case 'K': case 'M': case 'S': case 'W': case 'B': case 'D':
    case 'H': case 'V': return 4;
  }
  return -1;
}

/* Packs every record of text[0, n). Returns the number of records, or -kind on error with *err_rec = the
 * failing record. out needs room for n bytes, offs for n / 6 + 2 entries. */
int64_t orc_fastq_pack(const char *text, uint64_t n, int qual_offset, uint8_t *out, uint64_t *offs,
                       uint64_t *err_rec) {
  uint64_t pos = 0, r = 0, nb = 0;
  offs[0] = 0;
  while (pos < n) {
    uint64_t lb[4], le[4];
    for (int i = 0; i < 4; i++) {
      if (pos >= n) { *err_rec = r; return -7; }
      const char *nl = memchr(text + pos, '\n', n - pos);
      const uint64_t end = nl ? (uint64_t)(nl - text) : n;
      lb[i] = pos;
      le[i] = end;
      pos = end + 1;
    }
    for (int i = 0; i < 4; i++)
      if (le[i] - lb[i] > 2045) { *err_rec = r; return -5; }
    const uint64_t ide = fq_rtrim(text, lb[0], le[0]);
    const uint64_t se = fq_rtrim(text, lb[1], le[1]);
    const uint64_t qe = fq_rtrim(text, lb[3], le[3]);
    if (ide == lb[0] || text[lb[0]] != '@') { *err_rec = r; return -1; }
    if (le[2] == lb[2] || text[lb[2]] != '+') { *err_rec = r; return -2; }
    if (!fq_name_ok(text, lb[0], ide)) { *err_rec = r; return -3; }
    const uint64_t L = se - lb[1];
    if (L != qe - lb[3]) { *err_rec = r; return -4; }
    for (uint64_t i = 0; i < L; i++) {
      const int c = fq_code(text[lb[1] + i]);
      if (c < 0) { *err_rec = r; return -6; }
      int q = (int)(signed char)text[lb[3] + i] - qual_offset;
      if (q > 31) q = 31;
      out[nb + i] = (uint8_t)(c | (uint8_t)((unsigned char)q << 3));
    }
    nb += L;
    offs[++r] = nb;
  }
  return (int64_t)r;
}
