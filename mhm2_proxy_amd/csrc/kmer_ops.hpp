// k-mer bit operations shared by the HIP kernels and the host code of libmhmkc.
//
// Layout (identical to the reference Kmer<MAX_K>::longs, src/kmer.cpp:178-188,224-232):
//   * 2 bits per base, A=0 C=1 G=2 T=3, MSB-first: base j of word l sits at bits 2*(31-j) of w[l];
//   * NL = k/32 + 1 words (the reference's MAX_K/32 with MAX_K = (k/32+1)*32, src/main.cpp:170);
//   * the unused low bits of the last word are zero.
// k % 32 == 0 is rejected by mhmkc_create: only then can a canonical last word be all ones, which
// the table uses as its EMPTY marker (the reference has the same aliasing, kcount_cpu.cpp:217,236).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define MHM_HD __host__ __device__ __forceinline__
#else
#define MHM_HD static inline
#endif

namespace mhm {

constexpr uint64_t KEY_EMPTY = ~0ull;          // last word of a free table slot
constexpr uint64_t KEY_BUSY = ~0ull - 1ull;    // last word of a slot whose key is being written
constexpr int MAX_NL = 4;                      // k <= 127 (MAX_BUILD_KMER 128)
constexpr int EXT_NONE = 4;                    // no countable extension
constexpr int EXT_BITS = 6;                    // record ext code = (left << 3) | right

MHM_HD uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

// fmix64 of MurmurHash3 (reference src/hash_funcs.c:65-73).
MHM_HD uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

// h1 of MurmurHash3_x64_128(longs, 8*NL, seed 313): Kmer<MAX_K>::hash() (src/kmer.cpp:465-468 ->
// src/hash_funcs.c:77-170,185-190). The key bytes are the little-endian words themselves, so a
// 16-byte block is (w[2b], w[2b+1]) and an odd trailing word is the 8-byte tail k1.
template <int NL>
MHM_HD uint64_t murmur3_h1(const uint64_t *w) {
  const uint64_t c1 = 0x87c37b91114253d5ull, c2 = 0x4cf5ad432745937full;
  uint64_t h1 = 313, h2 = 313;
#pragma unroll
  for (int b = 0; b < NL / 2; b++) {
    uint64_t k1 = w[2 * b], k2 = w[2 * b + 1];
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
  if (NL & 1) {
    uint64_t k1 = w[NL - 1];
    k1 *= c1;
    k1 = rotl64(k1, 31);
    k1 *= c2;
    h1 ^= k1;
  }
  h1 ^= (uint64_t)(8 * NL);
  h2 ^= (uint64_t)(8 * NL);
  h1 += h2;
  h2 += h1;
  h1 = fmix64(h1);
  h2 = fmix64(h2);
  h1 += h2;
  return h1;
}

// Hash that assigns a k-mer of the unmixed record kinds to its rank / coarse bucket / fine bucket: Kmer::hash
// (MurmurHash3 h1). (A two-multiply mixer saved 1.1 ms of extraction at k = 77 and cost 3.4 ms of partition and
// counting through its less even digits, §4.2.)
template <int NL>
MHM_HD uint64_t part_hash(const uint64_t *w) {
  return murmur3_h1<NL>(w);
}

// ------------------------------------------------------------------------------------------------
// Compact records (one key word, 10 <= k <= 21). The partition hash of a compact key is
// a bijection y = cmix(x) of its B = 2k key bits x (20 <= B <= 42), so the coarse and fine bucket digits (the top bits
// of y) need not be stored: a coarse-bucketed record keeps the low B - cb bits of y next to the ext
// code (<= 40 bits: a u32 plane + a byte plane), a fine-bucketed record the low B - cb - fb bits
// (<= 32 bits: one u32 plane), and k_count rebuilds the key as cunmix(bucket digits | stored bits).
// cmix is a Feistel network on the two halves of the B key bits (a = B/2 low bits, b = B - a <= 21 high bits; a
// Feistel round is invertible whatever its round function). The round function takes bits [11, 11 + n) of the low
// 32 bits of a 24 x 24-bit product: one full-rate v_mul_u32_u24, where fmix64's xorshift-multiply chain needs
// quarter-rate 64-bit multiplies. Three rounds: the bucket digits are the top bits of the third round's L
// (L ^ f(R) ^ f(R ^ f(L ^ f(R)))), k_count's home group the bits below them and the top of the second round's R; a
// fourth round only re-mixed R (two rounds: extraction 4.915 -> 4.913 ms, not worth the weaker digits).
constexpr int CMP_MIN_K = 10, CMP_MAX_K = 21;
constexpr uint32_t FEISTEL_K[3] = {0x9E3779u, 0x85EBCAu, 0xC2B2AEu};
// 24 x 24-bit product, low 32 bits (v_mul_u32_u24, full rate; a plain masked product can come out as the
// quarter-rate v_mul_lo_u32 when the compiler loses track of the mask). b must be wave-uniform (an SGPR operand:
// every caller passes a constant).
MHM_HD uint32_t mul24(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t r;  // (inline asm: hipcc turns __umul24 of a non-constant-bounded operand into v_mul_lo_u32)
  asm("v_mul_u32_u24 %0, %1, %2" : "=v"(r) : "v"(a), "s"(b));
  return r;
#else
  return (a & 0xffffffu) * (b & 0xffffffu);
#endif
}
MHM_HD uint32_t feistel_f(uint32_t v, uint32_t c, int n) { return (mul24(v ^ (v >> 9), c) >> 11) & ((1u << n) - 1); }

// The Feistel rounds on the halves (L: b bits, R: a bits) and their inverse.
MHM_HD void cmix_lr(uint32_t &L, uint32_t &R, int a, int b) {
  L ^= feistel_f(R, FEISTEL_K[0], b);
  R ^= feistel_f(L, FEISTEL_K[1], a);
  L ^= feistel_f(R, FEISTEL_K[2], b);
}
MHM_HD void cunmix_lr(uint32_t &L, uint32_t &R, int a, int b) {
  L ^= feistel_f(R, FEISTEL_K[2], b);
  R ^= feistel_f(L, FEISTEL_K[1], a);
  L ^= feistel_f(R, FEISTEL_K[0], b);
}

MHM_HD uint64_t cmix(uint64_t x, int B) {
  const int a = B >> 1, b = B - a;
  uint32_t R = (uint32_t)x & ((1u << a) - 1), L = (uint32_t)(x >> a);
  cmix_lr(L, R, a, b);
  return ((uint64_t)L << a) | R;
}

MHM_HD uint64_t cunmix(uint64_t y, int B) {
  const int a = B >> 1, b = B - a;
  uint32_t R = (uint32_t)y & ((1u << a) - 1), L = (uint32_t)(y >> a);
  cunmix_lr(L, R, a, b);
  return ((uint64_t)L << a) | R;
}

// Partition hash of a compact key word (2k bits, left-aligned): the mixed key, left-aligned, so that the
// coarse / fine digits are taken from its top bits exactly as from part_hash.
MHM_HD uint64_t cpart_hash(uint64_t w, int B) { return cmix(w >> (64 - B), B) << (64 - B); }

MHM_HD bool compact_ok(int k, int nl) { return nl == 1 && k >= CMP_MIN_K && k <= CMP_MAX_K; }

// ------------------------------------------------------------------------------------------------
// Mixed two-word records (33 <= k <= 63, NL = 2). The 2k key bits are split into halves of
// k bits, L (bases 0 .. k/2-ish, the top k bits) and R (the low k bits), and put through a 2-round Feistel
// network, (L', R') = m2_mix(key). The coarse and fine digits are the top bits of L', so a record keeps
//   w[0] = (L' below the digits) << 6 | ext code,   w[1] = R'
// (16 B, no byte plane, no stored hash bits), and k_count rebuilds the key as m2_unmix(digits | w[0] >> 6, w[1]).
// The round functions hash their k-bit input to 32 bits with full-rate 24-bit multiplies and xor them into the 32
// bits that are used downstream: the top 32 bits of L (the bucket digits are the top bits of L'), the low 32 bits
// of R (k_count's home group is the low 16 bits of R'). A Feistel round is a bijection whatever its round function
// and wherever it xors, so the other bits may pass unmixed. Two rounds: the digits are top(L) ^ h(R), R (the last
// ~k/2 bases) being all but unique per k-mer, and the home group is low(R) ^ h(L'); a third round only re-mixed L.
// (Three rounds of a 64-bit multiply folded onto itself, four quarter-rate VALU ops each, were round 2's first mix.)
constexpr int M2_MIN_K = 33, M2_MAX_K = 63;
MHM_HD bool mixed2_ok(int k, int nl) { return nl == 2 && k >= M2_MIN_K && k <= M2_MAX_K; }
constexpr uint32_t M2_C[4] = {0x9E3779u, 0x85EBCBu, 0xC2B2AFu, 0x27D4EBu};
MHM_HD uint32_t m2_h(uint64_t v, uint32_t c1, uint32_t c2) {  // <= 63-bit v -> 32 bits
  const uint32_t hi = (uint32_t)(v >> 32);
  uint32_t u = (uint32_t)v ^ ((hi << 7) | (hi >> 25));
  u ^= u >> 16;
  u = mul24(u, c1);
  u ^= u >> 15;
  u = mul24(u, c2);
  u ^= u >> 16;
  return u;
}

// The rounds on the halves: (L, R) -> (L', R'), k bits each, and back.
MHM_HD void m2_mix_lr(uint64_t &L, uint64_t &R, int k) {
  L ^= (uint64_t)m2_h(R, M2_C[0], M2_C[1]) << (k - 32);
  R ^= (uint64_t)m2_h(L, M2_C[2], M2_C[3]);
}
MHM_HD void m2_unmix_lr(uint64_t &L, uint64_t &R, int k) {
  R ^= (uint64_t)m2_h(L, M2_C[2], M2_C[3]);
  L ^= (uint64_t)m2_h(R, M2_C[0], M2_C[1]) << (k - 32);
}

// key words (Kmer::longs layout, k bases) -> (L', R'), k bits each
MHM_HD void m2_mix(const uint64_t *w, int k, uint64_t &L, uint64_t &R) {
  const uint64_t m = (1ull << k) - 1;
  L = w[0] >> (64 - k);
  R = ((w[0] << (2 * k - 64)) | (w[1] >> (128 - 2 * k))) & m;  // x = L << k | R: x's low 64 bits, masked
  m2_mix_lr(L, R, k);
}

// (L', R') -> key words (the last word's unused low bits zero)
MHM_HD void m2_unmix(uint64_t L, uint64_t R, int k, uint64_t *w) {
  m2_unmix_lr(L, R, k);
  w[0] = (L << (64 - k)) | (R >> (2 * k - 64));
  w[1] = R << (128 - 2 * k);
}

// ------------------------------------------------------------------------------------------------
// Mixed three- and four-word records (64 < k < 128, k % 32 != 0, NL = 3, 4). Two Feistel rounds
// over the key words w[0..NL-1] (Kmer layout; the tail word w[NL-1] holds the last k - 32 (NL - 1) bases):
//   w0' = w0 ^ (h1(w[1..NL-1]) << 32)     the bucket digits are the top bits of w0'
//   X   = w[NL-2] ^ h2(w0')                a full 64-bit word: k_count's examined (last) table word, home group
//                                          from its low bits
// Mixed words r[0] = w0', r[1..NL-3] = w[1..NL-3], r[NL-2] = w[NL-1] (the tail), r[NL-1] = X; a record keeps
// r[0] below the bucket digits << 6 | ext code in its first word (like §3.7b's L'), so three- and four-word keys drop
// the 16 stored MurmurHash3 bits and MurmurHash3 itself (about ten quarter-rate 64-bit multiplies per window in the
// extraction, and a 64-bit slot hash per lookup in k_count). h1 and h2 use full-rate 24-bit multiplies (m2_h).
constexpr uint32_t MX_C[8] = {0x9E3779u, 0x85EBCBu, 0xC2B2AFu, 0x27D4EBu, 0x165667u, 0x3A2659u, 0xD3A2E5u, 0x6B43A9u};
MHM_HD bool mixed3_ok(int k, int nl) { return (nl == 3 || nl == 4) && k % 32 != 0 && k < 32 * nl; }
MHM_HD uint32_t mx_stir(uint32_t u, uint32_t c1, uint32_t c2) {
  u ^= u >> 16;
  u = mul24(u, c1);
  u ^= u >> 15;
  u = mul24(u, c2);
  u ^= u >> 16;
  return u;
}
MHM_HD uint32_t fold64(uint64_t v) {
  const uint32_t hi = (uint32_t)(v >> 32);
  return (uint32_t)v ^ ((hi << 7) | (hi >> 25));
}
template <int NL>
MHM_HD uint32_t mx_h1(const uint64_t *w) {  // w[1..NL-1] -> 32 bits
  uint32_t u = mx_stir(fold64(w[1]), MX_C[0], MX_C[1]);
#pragma unroll
  for (int i = 2; i < NL; i++) u = mx_stir(u ^ fold64(w[i]), MX_C[2 * i - 2], MX_C[2 * i - 1]);
  return u;
}
// key words -> mixed words (r[0] = w0' in full)
template <int NL>
MHM_HD void mx_mix(const uint64_t *w, uint64_t *r) {
  r[0] = w[0] ^ ((uint64_t)mx_h1<NL>(w) << 32);
#pragma unroll
  for (int i = 1; i + 2 < NL; i++) r[i] = w[i];
  r[NL - 2] = w[NL - 1];
  r[NL - 1] = w[NL - 2] ^ (uint64_t)m2_h(r[0], MX_C[6], MX_C[7]);
}
// mixed words (r[0] = w0' in full) -> key words
template <int NL>
MHM_HD void mx_unmix(const uint64_t *r, uint64_t *w) {
  w[NL - 2] = r[NL - 1] ^ (uint64_t)m2_h(r[0], MX_C[6], MX_C[7]);
  w[NL - 1] = r[NL - 2];
#pragma unroll
  for (int i = 1; i + 2 < NL; i++) w[i] = r[i];
  w[0] = r[0] ^ ((uint64_t)mx_h1<NL>(w) << 32);
}

// Reverse the order of the 32 two-bit groups of x.
MHM_HD uint64_t rev2(uint64_t x) {
  x = __builtin_bswap64(x);
  x = ((x >> 4) & 0x0F0F0F0F0F0F0F0Full) | ((x & 0x0F0F0F0F0F0F0F0Full) << 4);
  x = ((x >> 2) & 0x3333333333333333ull) | ((x & 0x3333333333333333ull) << 2);
  return x;
}

// Top 2*n bits set (the reference's ZERO_MASK[n], src/kmer.cpp:81-87), n in [1, 32].
MHM_HD uint64_t top_mask(int n) { return n >= 32 ? ~0ull : ~(~0ull >> (2 * n)); }

// Reverse complement of a k-mer held in NL words (same result as Kmer::revcomp, src/kmer.cpp:485-505):
// complement and reverse every word, reverse the word order, then shift the concatenation left by
// 2*(32*NL - k) bits so the junk from the zero padding falls off the end.
template <int NL>
MHM_HD void revcomp(const uint64_t *w, uint64_t *rc, int k) {
  uint64_t t[NL];
#pragma unroll
  for (int i = 0; i < NL; i++) t[NL - 1 - i] = rev2(~w[i]);
  const int sh = 2 * (32 * NL - k);  // in [2, 62] for k % 32 != 0
#pragma unroll
  for (int i = 0; i < NL; i++) {
    uint64_t v = t[i] << sh;
    if (i + 1 < NL) v |= t[i + 1] >> (64 - sh);
    rc[i] = v;
  }
  rc[NL - 1] &= top_mask(k - 32 * (NL - 1));
}

// Word-wise unsigned lexicographic compare == Kmer::operator< (src/kmer.cpp:265-272).
template <int NL>
MHM_HD bool kmer_less(const uint64_t *a, const uint64_t *b) {
  if (NL == 2) return (a[0] < b[0]) | ((a[0] == b[0]) & (a[1] < b[1]));  // branch-free (walk_windows)
  // branch-free for any NL: an early return per word made the unrolled extraction walk of three- and four-word
  // keys one divergent branch per word and window
  bool lt = false, decided = false;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    lt = decided ? lt : (a[i] < b[i]);
    decided |= a[i] != b[i];
  }
  return lt;
}

// quick_hash (src/hash_funcs.c:332-342)
MHM_HD uint64_t quick_hash(uint64_t v) {
  v = v * 3935559000370003845ull + 2691343689449507681ull;
  v ^= v >> 21;
  v ^= v << 37;
  v ^= v >> 4;
  v *= 4768777513237032717ull;
  v ^= v << 20;
  v ^= v >> 41;
  v ^= v << 5;
  return v;
}

// Kmer::get_minimizer_fast(m, least_complement = true) (src/kmer.cpp:344-393, 395-403): the greatest, over
// the m-mer positions i in [0, k-m], of min(forward m-mer i, its reverse complement), each left-aligned in a
// word with the low bits zero (ZERO_MASK[m], :81-87). The reference reads the reverse-complement candidate
// of position i as the m-mer at k-m-i of revcomp(kmer), which is the reverse complement of forward m-mer
// i; here both are rolled base by base (forward shifts a base in at the bottom, the reverse complement
// shifts the complemented base in at the top), m <= 28.
MHM_HD uint64_t minimizer_fast(const uint64_t *w, int k, int m) {
  const uint64_t mm = (1ull << (2 * m)) - 1;
  const int up = 64 - 2 * m;
  uint64_t f = 0, r = 0, best = 0;
  for (int j = 0; j < k; j++) {
    const uint64_t b = (w[j >> 5] >> (62 - 2 * (j & 31))) & 3u;
    f = ((f << 2) | b) & mm;
    r = (r >> 2) | ((3u - b) << (2 * m - 2));
    if (j >= m - 1) {
      const uint64_t fl = f << up, rl = r << up;
      const uint64_t least = fl < rl ? fl : rl;
      best = least > best ? least : best;
    }
  }
  return best;
}

// Packed-record mode: the 6-bit ext code fits into the zero low bits of the last key word.
MHM_HD bool ext_packs(int k, int nl) { return 2 * (k - 32 * (nl - 1)) + EXT_BITS <= 64; }

// get_ext of the reference (src/kcount/kcount_cpu.cpp:173-182): 'X' when the top count is below the
// dynamic threshold, 'F' when the runner-up reaches it, otherwise the (then unique) top base.
// thr = max((int)((1.0 - DYN_MIN_DEPTH) * count), dmin_thres).
MHM_HD char ext_choice(uint32_t a, uint32_t c, uint32_t g, uint32_t t, int thr) {
  uint32_t v[4] = {a, c, g, t};
  uint32_t top = 0, second = 0;
  int arg = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    if (v[i] > top) {
      second = top;
      top = v[i];
      arg = i;
    } else if (v[i] > second) {
      second = v[i];
    }
  }
  if ((int)top < thr) return 'X';
  if ((int)second >= thr) return 'F';
  // 'A' 'C' 'G' 'T' = 0x41 0x43 0x47 0x54, one byte each of a constant (a char array here was compiled into a
  // global-memory table: two dependent loads per decided k-mer in k_count's finalize)
  return (char)((0x54474341u >> (8 * arg)) & 0xffu);
}

MHM_HD int dyn_threshold(uint32_t count16, double dyn_mult, int dmin_thres) {
  int t = (int)(dyn_mult * (double)count16);
  return t > dmin_thres ? t : dmin_thres;
}

}  // namespace mhm
