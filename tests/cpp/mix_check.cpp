// Host check of the mixed-record bijections (kmer_ops.hpp cmix / cunmix for compact records, DESIGN.md §3.7, and
// m2_mix / m2_unmix for mixed two-word records, §3.7b, mx_mix / mx_unmix for three- and four-word records, §3.7c):
//   1. the inverse undoes the mix and the mixed key stays in its bits, for random keys at every k in 10..21, 33..63
//      and 65..127 (k % 32 != 0);
//   2. the bucket digits (top bits of L') and k_count's home group (low 16 bits of R') of the canonical windows of
//      one random sequence (consecutive windows: correlated inputs) are flat: prints the max / mean bin ratio of
//      the coarse digit (256 bins), the coarse+fine digits (2^17 bins) and the home group (1000 groups).
// Usage: mix_check [n_windows]   -> "k <k> coarse <r> fine <r> group <r>" lines, "roundtrip ok"
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../mhm2_proxy_amd/csrc/kmer_ops.hpp"

static uint64_t sm_state = 0x1234567ull;
static uint64_t splitmix() {
  uint64_t z = (sm_state += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static double max_over_mean(const std::vector<uint32_t> &h, uint64_t n) {
  uint32_t mx = 0;
  for (uint32_t v : h) mx = v > mx ? v : mx;
  return (double)mx / ((double)n / (double)h.size());
}

int main(int argc, char **argv) {
  const uint64_t nw = argc > 1 ? strtoull(argv[1], nullptr, 10) : 4000000;
  // 1. round trips
  for (int k = 33; k <= 63; k++) {
    if (k == 64) continue;
    const uint64_t m1 = ~(~0ull >> (2 * (k - 32)));  // the used top bits of the last word
    for (int i = 0; i < 20000; i++) {
      uint64_t w[2] = {splitmix(), splitmix() & m1}, L, R, b[2];
      mhm::m2_mix(w, k, L, R);
      if ((L >> k) || (R >> k)) {
        printf("range k=%d\n", k);
        return 1;
      }
      mhm::m2_unmix(L, R, k, b);
      if (b[0] != w[0] || b[1] != w[1]) {
        printf("roundtrip k=%d\n", k);
        return 1;
      }
    }
  }
  for (int k = 10; k <= 21; k++) {
    const int B = 2 * k;
    for (int i = 0; i < 20000; i++) {
      const uint64_t x = splitmix() >> (64 - B), y = mhm::cmix(x, B);
      if ((y >> B) || mhm::cunmix(y, B) != x) {
        printf("compact roundtrip k=%d\n", k);
        return 1;
      }
    }
  }
  for (int k = 65; k <= 127; k++) {
    if (k % 32 == 0) continue;
    const int nl = k / 32 + 1;
    const uint64_t m1 = ~(~0ull >> (2 * (k - 32 * (nl - 1))));
    for (int i = 0; i < 20000; i++) {
      uint64_t w[4] = {splitmix(), splitmix(), splitmix(), splitmix()}, r[4], b[4];
      w[nl - 1] &= m1;
      if (nl == 3) {
        mhm::mx_mix<3>(w, r);
        mhm::mx_unmix<3>(r, b);
      } else {
        mhm::mx_mix<4>(w, r);
        mhm::mx_unmix<4>(r, b);
      }
      if (r[nl - 2] != w[nl - 1]) {  // the tail word passes unchanged (its unused low bits stay zero)
        printf("mx tail k=%d\n", k);
        return 1;
      }
      for (int j = 0; j < nl; j++)
        if (b[j] != w[j]) {
          printf("mx roundtrip k=%d\n", k);
          return 1;
        }
    }
  }
  printf("roundtrip ok\n");
  // 2. digit / group flatness over consecutive canonical windows of one sequence
  std::vector<uint8_t> seq(nw + 64);
  for (auto &c : seq) c = (uint8_t)(splitmix() & 3);
  for (int k : {21, 15}) {  // compact: digits are the top bits of y = cmix(x), k_count's group the 16 bits below
    const int B = 2 * k, cb = 8, fb = k == 21 ? 9 : 4;
    std::vector<uint32_t> hc(256, 0), hf(1u << (cb + fb), 0), hg(1000, 0);
    for (uint64_t p = 0; p < nw; p++) {
      uint64_t f = 0, r = 0;
      for (int j = 0; j < k; j++) {
        f = (f << 2) | seq[p + j];
        r = (r << 2) | (3 - seq[p + k - 1 - j]);
      }
      const uint64_t y = mhm::cmix(r < f ? r : f, B);
      hc[y >> (B - cb)]++;
      hf[y >> (B - cb - fb)]++;
      hg[(((y >> (B - cb - fb - 16)) & 0xffff) * 1000) >> 16]++;
    }
    printf("k %d coarse %.4f fine %.4f group %.4f\n", k, max_over_mean(hc, nw), max_over_mean(hf, nw),
           max_over_mean(hg, nw));
  }
  for (int k : {33, 47, 55, 63}) {
    std::vector<uint32_t> hc(256, 0), hf(1u << 17, 0), hg(1000, 0);
    for (uint64_t p = 0; p < nw; p++) {
      uint64_t f[2] = {0, 0}, r[2] = {0, 0};
      for (int j = 0; j < k; j++) {
        const uint64_t c = seq[p + j], rcb = 3 - seq[p + k - 1 - j];
        f[j >> 5] |= c << (62 - 2 * (j & 31));
        r[j >> 5] |= rcb << (62 - 2 * (j & 31));
      }
      const bool use_rc = r[0] < f[0] || (r[0] == f[0] && r[1] < f[1]);
      const uint64_t *key = use_rc ? r : f;
      uint64_t L, R;
      mhm::m2_mix(key, k, L, R);
      hc[L >> (k - 8)]++;
      hf[L >> (k - 17)]++;
      hg[((R & 0xffff) * 1000) >> 16]++;
    }
    printf("k %d coarse %.4f fine %.4f group %.4f\n", k, max_over_mean(hc, nw), max_over_mean(hf, nw),
           max_over_mean(hg, nw));
  }
  for (int k : {65, 77, 95, 99, 127}) {  // three- and four-word: digits = top bits of w0', group = low 16 bits of X
    const int nl = k / 32 + 1;
    std::vector<uint32_t> hc(256, 0), hf(1u << 17, 0), hg(1000, 0);
    for (uint64_t p = 0; p < nw; p++) {
      uint64_t f[4] = {0, 0, 0, 0}, r[4] = {0, 0, 0, 0}, m[4];
      for (int j = 0; j < k; j++) {
        const uint64_t c = seq[p + j], rcb = 3 - seq[p + k - 1 - j];
        f[j >> 5] |= c << (62 - 2 * (j & 31));
        r[j >> 5] |= rcb << (62 - 2 * (j & 31));
      }
      bool lt = false, decided = false;
      for (int i = 0; i < nl; i++) {
        lt = decided ? lt : r[i] < f[i];
        decided |= r[i] != f[i];
      }
      const uint64_t *key = lt ? r : f;
      if (nl == 3)
        mhm::mx_mix<3>(key, m);
      else
        mhm::mx_mix<4>(key, m);
      hc[m[0] >> 56]++;
      hf[m[0] >> 47]++;
      hg[((m[nl - 1] & 0xffff) * 1000) >> 16]++;
    }
    printf("k %d coarse %.4f fine %.4f group %.4f\n", k, max_over_mean(hc, nw), max_over_mean(hf, nw),
           max_over_mean(hg, nw));
  }
  return 0;
}
