// The contig pass of the kcount stage on gfx950.
//
// Reference: analyze_kmers runs add_ctg_kmers after the read pass (src/kcount/kcount.cpp:140-157,
// 100-138): every contig of length >= k+2 is one supermer with count = depth
// (SeqBlockInserter::process_seq, src/kcount/kcount_cpu.cpp:73-103), inserted by
// insert_supermer_from_ctg (kcount_cpu.cpp:356-406). Per canonical k-mer that rule is a fold over the
// k-mer's contig occurrences in contig order, started from the read entry:
//   * a read entry that exists with count >= 2 and unique extensions on both sides (UU) is kept and every
//     contig occurrence is ignored;
//   * otherwise (no read entry, a singleton, or non-UU) the first occurrence replaces it: {count = depth,
//     ext counter [left] = [right] = depth, from_ctg};
//   * a later occurrence meets a contig entry: count 0 stays 0; else if the entry's extension choices
//     (get_ext) differ from the occurrence's raw extensions the count becomes 0 (purged later), otherwise
//     min(depth, count); the extensions become the occurrence's.
// The fold is order dependent (a depth below dmin_thres makes the entry's choice 'X'), so this pass keeps
// the order: contig windows are extracted in contig order, stably sorted by key, and one lane folds each
// key's run. The result per key does not depend on the read entry except through "kept or not", which
// k_count decides when it meets the key in its bucket (kcount_kernels.hip, ctg_apply).
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>

#include "kcount_launch.hpp"
#include "kmer_ops.hpp"

namespace mhm {

namespace {

constexpr int G_THREADS = 256;

inline unsigned grid_for(uint64_t n) { return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(4096, (n + 255) / 256)); }

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// Counted windows i in [1, L-k-1] of contig c, in contig order: window w of the batch.
template <int NL>
__global__ __launch_bounds__(G_THREADS) void k_ctg_extract(CtgView cv, int k, int qcut, PlaneSet keys, uint32_t *aux,
                                                            unsigned int *err) {
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < cv.n_windows;
       w += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t lo = 0, hi = cv.n_ctgs;  // last contig c with win_prefix[c] <= w (never an empty one)
    while (hi - lo > 1) {
      const uint64_t mid = (lo + hi) >> 1;
      if (cv.win_prefix[mid] <= w)
        lo = mid;
      else
        hi = mid;
    }
    const uint64_t c = lo;
    const uint64_t p = cv.offs[c] + 1 + (w - cv.win_prefix[c]);
    uint64_t fw[NL], rc[NL];
#pragma unroll
    for (int m = 0; m < NL; m++) fw[m] = 0;
    unsigned bad = 0;
    for (int j = 0; j < k; j++) {
      const uint32_t code = cv.bytes[p + j] & 7u;
      bad |= code > 4;
      const uint64_t t = (code & 3u) | ((code >> 1) & 2u);  // N -> G (src/kmer.cpp:169,187-188)
      fw[j >> 5] |= t << (62 - 2 * (j & 31));
    }
    const uint8_t lb = cv.bytes[p - 1], rb = cv.bytes[p + k];
    bad |= ((lb & 7u) > 4) | ((rb & 7u) > 4);
    if (bad) atomicOr(err, 1u);
    // extensions: the neighbour base when it is A/C/G/T of good quality, else none
    // (get_kmers_and_exts, kcount_cpu.cpp:319-324; ExtCounts::inc ignores N and '0')
    uint32_t l = ((lb & 7u) < 4 && (int)(lb >> 3) >= qcut) ? (lb & 7u) : (uint32_t)EXT_NONE;
    uint32_t r = ((rb & 7u) < 4 && (int)(rb >> 3) >= qcut) ? (rb & 7u) : (uint32_t)EXT_NONE;
    revcomp<NL>(fw, rc, k);
    const bool use_rc = kmer_less<NL>(rc, fw);  // kcount_cpu.cpp:326-332
    if (use_rc) {
      const uint32_t nl_ = r < 4 ? 3 - r : (uint32_t)EXT_NONE, nr_ = l < 4 ? 3 - l : (uint32_t)EXT_NONE;
      l = nl_;
      r = nr_;
    }
#pragma unroll
    for (int m = 0; m < NL; m++) keys.w[m][w] = use_rc ? rc[m] : fw[m];
    const uint32_t depth = cv.depth[c] ? cv.depth[c] : 1u;  // process_seq: if (!depth) depth = 1
    aux[w] = ((l << 3) | r) | (depth << 16);
  }
}

__global__ __launch_bounds__(G_THREADS) void k_iota(uint32_t *a, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    a[i] = (uint32_t)i;
}

__global__ __launch_bounds__(G_THREADS) void k_gather_u64(const uint64_t *src, const uint32_t *idx, uint64_t *dst,
                                                          uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = src[idx[i]];
}

__global__ __launch_bounds__(G_THREADS) void k_gather_u32(const uint32_t *src, const uint32_t *idx, uint32_t *dst,
                                                          uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = src[idx[i]];
}

// The contig entry's choice on one side: its only counter is [code] = count (ExtCounts::get_ext,
// kcount_cpu.cpp:173-182). 0-3 = the base, 5 = 'X', 6 = 'F'.
__device__ __forceinline__ uint32_t single_choice(uint32_t code, uint32_t count, int thr) {
  const int top = code < 4 ? (int)count : 0;
  if (top < thr) return 5;
  if (0 >= thr) return 6;
  return code;
}

// One lane per run of equal keys in sorted order: fold the run's occurrences (contig order, the sort is
// stable) and emit the k-mer's contig entry with its local fine bucket.
template <int NL>
__global__ __launch_bounds__(G_THREADS) void k_ctg_fold(PlaneSet keys, const uint32_t *aux, const uint32_t *perm,
                                                         uint64_t n, int dmin, double dyn_mult, int cb, int fb,
                                                         uint32_t own_lo, uint32_t own_hi, int cmpB, int k, CtgOwner ow,
                                                         PlaneSet fkeys, uint32_t *fstate,
                                                         uint32_t *fbucket, uint32_t *fidx,
                                                         unsigned long long *counter) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t key[NL];
    const uint32_t pi = perm[i];
#pragma unroll
    for (int m = 0; m < NL; m++) key[m] = keys.w[m][pi];
    if (i > 0) {
      const uint32_t pp = perm[i - 1];
      bool same = true;
#pragma unroll
      for (int m = 0; m < NL; m++) same &= keys.w[m][pp] == key[m];
      if (same) continue;  // not the head of its run
    }
    bool active = false;
    uint32_t C = 0, L = EXT_NONE, R = EXT_NONE;
    for (uint64_t j = i; j < n; j++) {
      const uint32_t pj = perm[j];
      if (j > i) {
        bool same = true;
#pragma unroll
        for (int m = 0; m < NL; m++) same &= keys.w[m][pj] == key[m];
        if (!same) break;
      }
      const uint32_t a = aux[pj];
      const uint32_t c = a >> 16, l = (a >> 3) & 7u, r = a & 7u;
      if (!active) {  // the first contig occurrence: insert (the read entry question is k_count's)
        active = true;
        C = c;
        L = l;
        R = r;
      } else if (C != 0) {  // an existing contig entry (kcount_cpu.cpp:381-398)
        const int thr = dyn_threshold(C, dyn_mult, dmin);
        const bool agree = single_choice(L, C, thr) == l && single_choice(R, C, thr) == r;
        C = agree ? (c < C ? c : C) : 0u;
        L = l;
        R = r;
      }
    }
    uint64_t h;  // the partition hash of k_extract_scatter
    if (NL == 1 && cmpB) {
      h = cpart_hash(key[0], cmpB);
    } else if (NL == 2 && cmpB) {  // mixed two-word records: L' of m2_mix, left-aligned
      uint64_t L, R;
      m2_mix(key, cmpB / 2, L, R);
      h = L << (64 - cmpB / 2);
    } else if (NL >= 3 && cmpB) {  // mixed three- and four-word records: w0' of mx_mix
      uint64_t r[NL];
      mx_mix<NL>(key, r);
      h = r[0];
    } else {
      h = part_hash<NL>(key);
    }
    const uint32_t coarse = (uint32_t)(h >> (64 - cb));
    if (coarse < own_lo || coarse >= own_hi) continue;  // another rank's hash range (it folds this key itself)
    // supermer exchange: this rank holds the k-mers of its get_kmer_target_rank (kmer_dht.cpp:193-196)
    if (ow.n_ranks && (int)(quick_hash(minimizer_fast(key, k, ow.m)) % (uint64_t)ow.n_ranks) != ow.rank) continue;
    const uint32_t fine = fb ? (uint32_t)((h >> (64 - cb - fb)) & ((1ull << fb) - 1)) : 0u;
    const unsigned long long o = atomicAdd(counter, 1ull);
#pragma unroll
    for (int m = 0; m < NL; m++) fkeys.w[m][o] = key[m];
    fstate[o] = ctg_state_word(C, L, R);
    fbucket[o] = ((coarse - own_lo) << fb) | fine;
    fidx[o] = (uint32_t)o;
  }
}

struct Scratch {
  PlaneSet keys, fkeys;
  uint32_t *aux, *perm, *perm2, *fstate, *fbucket, *fbucket2, *fidx, *fidx2;
  uint64_t *tmp, *tmp2;
  unsigned long long *counter;
  void *sort_tmp;
  size_t sort_bytes;
};

size_t sort_temp_bytes(uint64_t n) {
  size_t a = 0, b = 0;
  (void)rocprim::radix_sort_pairs(nullptr, a, (const uint64_t *)nullptr, (uint64_t *)nullptr,
                                  (const uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)n);
  (void)rocprim::radix_sort_pairs(nullptr, b, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                  (const uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)n);
  return std::max(a, b);
}

// Carve the scratch (or just measure it when base is null).
size_t carve(void *base, uint64_t n, int nl, Scratch *sc) {
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char *p = base ? (char *)base + off : nullptr;
    off += align256(std::max<size_t>(bytes, 1));
    return p;
  };
  Scratch s{};
  for (int m = 0; m < 4; m++) s.keys.w[m] = m < nl ? (uint64_t *)take(n * 8) : nullptr;
  for (int m = 0; m < 4; m++) s.fkeys.w[m] = m < nl ? (uint64_t *)take(n * 8) : nullptr;
  s.aux = (uint32_t *)take(n * 4);
  s.perm = (uint32_t *)take(n * 4);
  s.perm2 = (uint32_t *)take(n * 4);
  s.fstate = (uint32_t *)take(n * 4);
  s.fbucket = (uint32_t *)take(n * 4);
  s.fbucket2 = (uint32_t *)take(n * 4);
  s.fidx = (uint32_t *)take(n * 4);
  s.fidx2 = (uint32_t *)take(n * 4);
  s.tmp = (uint64_t *)take(n * 8);
  s.tmp2 = (uint64_t *)take(n * 8);
  s.counter = (unsigned long long *)take(8);
  s.sort_bytes = sort_temp_bytes(n);
  s.sort_tmp = take(s.sort_bytes);
  if (sc) *sc = s;
  return off;
}

template <int NL>
hipError_t prepare(const CtgView &cv, int k, int qcut, int dmin, double dyn_mult, int cb, int fb, uint32_t own_lo,
                   uint32_t own_hi, int cmpB, const CtgOwner &ow, const Scratch &sc, uint64_t *const out_keys[4],
                   uint32_t *out_state, uint32_t *out_bucket, uint64_t *n_out, unsigned int *err, hipStream_t s) {
  const uint64_t n = cv.n_windows;
  hipError_t e;
  k_ctg_extract<NL><<<grid_for(n), G_THREADS, 0, s>>>(cv, k, qcut, sc.keys, sc.aux, err);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  k_iota<<<grid_for(n), G_THREADS, 0, s>>>(sc.perm, n);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  // LSD: stable radix sorts by the key words, last word first; the value is the window index
  uint32_t *perm = sc.perm, *perm2 = sc.perm2;
  for (int m = NL - 1; m >= 0; m--) {
    k_gather_u64<<<grid_for(n), G_THREADS, 0, s>>>(sc.keys.w[m], perm, sc.tmp, n);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    size_t bytes = sc.sort_bytes;
    if ((e = rocprim::radix_sort_pairs(sc.sort_tmp, bytes, sc.tmp, sc.tmp2, perm, perm2, (size_t)n, 0, 64, s)) !=
        hipSuccess)
      return e;
    std::swap(perm, perm2);
  }
  if ((e = hipMemsetAsync(sc.counter, 0, 8, s)) != hipSuccess) return e;
  k_ctg_fold<NL><<<grid_for(n), G_THREADS, 0, s>>>(sc.keys, sc.aux, perm, n, dmin, dyn_mult, cb, fb, own_lo, own_hi, cmpB,
                                                   k, ow, sc.fkeys,
                                                   sc.fstate, sc.fbucket, sc.fidx, sc.counter);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  unsigned long long f = 0;
  if ((e = hipMemcpyAsync(&f, sc.counter, 8, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
  *n_out = f;
  if (!f) return hipSuccess;
  size_t bytes = sc.sort_bytes;
  if ((e = rocprim::radix_sort_pairs(sc.sort_tmp, bytes, sc.fbucket, out_bucket, sc.fidx, sc.fidx2, (size_t)f, 0, 32,
                                     s)) != hipSuccess)
    return e;
  for (int m = 0; m < NL; m++) {
    k_gather_u64<<<grid_for(f), G_THREADS, 0, s>>>(sc.fkeys.w[m], sc.fidx2, out_keys[m], f);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  k_gather_u32<<<grid_for(f), G_THREADS, 0, s>>>(sc.fstate, sc.fidx2, out_state, f);
  return hipGetLastError();
}

}  // namespace

size_t ctg_scratch_bytes(uint64_t n_windows, int nl) { return carve(nullptr, n_windows, nl, nullptr); }

hipError_t ctg_prepare(const CtgView &cv, int k, int nl, bool mixed, int qual_cutoff, int dmin_thres,
                       double dyn_mult, int coarse_bits, int fine_bits, uint32_t own_lo, uint32_t own_hi,
                       const CtgOwner &ow, void *scratch, size_t scratch_bytes,
                       uint64_t *const out_keys[4], uint32_t *out_state, uint32_t *out_bucket, uint64_t *n_out,
                       unsigned int *err, hipStream_t s) {
  *n_out = 0;
  if (!cv.n_windows) return hipSuccess;
  if (cv.n_windows >= 0xffffffffull) return hipErrorInvalidValue;  // 32-bit window indices
  Scratch sc;
  if (carve(scratch, cv.n_windows, nl, &sc) > scratch_bytes) return hipErrorInvalidValue;
  const int cmpB = mixed ? 2 * k : 0;  // compact (NL = 1) or mixed two-word (NL = 2) records
  switch (nl) {
    case 1: return prepare<1>(cv, k, qual_cutoff, dmin_thres, dyn_mult, coarse_bits, fine_bits, own_lo, own_hi, cmpB, ow, sc, out_keys,
                              out_state, out_bucket, n_out, err, s);
    case 2: return prepare<2>(cv, k, qual_cutoff, dmin_thres, dyn_mult, coarse_bits, fine_bits, own_lo, own_hi, cmpB, ow, sc, out_keys,
                              out_state, out_bucket, n_out, err, s);
    case 3: return prepare<3>(cv, k, qual_cutoff, dmin_thres, dyn_mult, coarse_bits, fine_bits, own_lo, own_hi, cmpB, ow, sc, out_keys,
                              out_state, out_bucket, n_out, err, s);
    case 4: return prepare<4>(cv, k, qual_cutoff, dmin_thres, dyn_mult, coarse_bits, fine_bits, own_lo, own_hi, cmpB, ow, sc, out_keys,
                              out_state, out_bucket, n_out, err, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace mhm
