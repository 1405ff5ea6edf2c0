// gfx950 kernels of the MI355X-native kcount stage.
//
// Pipeline per rank:
//   tile_first_read  per extract tile, first read starting at/after the tile (binary search)
//   extract_hist     PackedRead bytes -> canonical k-mer + ext code + MurmurHash3 -> coarse histogram
//   extract_scatter  same records, LDS-staged scatter into coarse buckets (hash range)
//   [RCCL all-to-all of coarse buckets to their owner rank]
//   part_hist        coarse bucket chunks -> fine histogram
//   scan             fine bucket bases
//   part_scatter     LDS-staged scatter into fine buckets
//   count            one workgroup per fine bucket: open-addressing hash table in LDS, count and
//                    extension counters, then the reference finalize rule (count >= 2, get_ext, X/X)
//                    and compaction into the output table.
// Semantics follow the reference CPU kcount at one rank, cited per function.
#include <hip/hip_runtime.h>
#include <type_traits>

#include <algorithm>

#include "kcount_launch.hpp"
#include "kmer_ops.hpp"

namespace mhm {

template <int NL>
constexpr int kTile() {  // bases per extract tile
  return TILE_BASES[NL];
}
template <int NL>
constexpr int kEThreads() {  // threads per extract workgroup
  return E_THREADS_NL[NL];
}
template <int NL>
constexpr int kPTile() {  // records per partition chunk (kPThreads threads)
  return P_TILE[NL];
}
template <int NL>
constexpr int kPThreads() {  // threads per partition workgroup
  return P_THREADS[NL];
}
template <int NL>
constexpr int kGroups() {
  return kTile<NL>() / 32 + NL + 2;
}

constexpr size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

// Load through a pointer known to be global memory. Pointers read from device tables (PlaneSet of a
// partition source) lose their address space and would otherwise become flat loads, which also count
// against lgkmcnt and are waited for together with LDS operations.
template <typename T>
__device__ __forceinline__ T gload(const T *p) {
  return *(const __attribute__((address_space(1))) T *)p;
}
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4 gload4(const uint32_t *p) {  // one 16-byte global load (p 16-byte aligned)
  return *(const __attribute__((address_space(1))) u32x4 *)p;
}

// All LDS is carved from the one dynamic region at 16-byte aligned offsets (cdna_hip_programming.md
// Guideline 17): fwd[NG] u64 | good[NG] u32 | start[NG] u32 | rest.
template <int NL>
__host__ __device__ constexpr size_t tile_lds_bytes() {
  return align16((size_t)kGroups<NL>() * 8) + 2 * align16((size_t)kGroups<NL>() * 4);
}
template <int NL>
__device__ __forceinline__ unsigned char *carve_tile(unsigned char *smem, uint64_t *&fwd, uint32_t *&good,
                                                     uint32_t *&start) {
  constexpr int NG = kGroups<NL>();
  fwd = (uint64_t *)smem;
  good = (uint32_t *)(smem + align16(NG * 8));
  start = (uint32_t *)(smem + align16(NG * 8) + align16(NG * 4));
  return smem + tile_lds_bytes<NL>();
}

// ------------------------------------------------------------------------------------------------
// block helpers

// Exclusive scan of a[0..n) in LDS by NT threads; returns the total. Uses wsum[NT/64 + 1].
template <int NT>
__device__ uint32_t block_excl_scan(uint32_t *a, int n, uint32_t *wsum) {
  const int per = (n + NT - 1) / NT;
  const int tid = threadIdx.x;
  const int lo = tid * per;
  const int hi = min(lo + per, n);
  uint32_t s = 0;
  for (int i = lo; i < hi; i++) s += a[i];
  uint32_t x = s;
  const int lane = tid & 63, wid = tid >> 6;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  if (tid == 0) {
    uint32_t acc = 0;
    for (int w = 0; w < NT / 64; w++) {
      uint32_t t = wsum[w];
      wsum[w] = acc;
      acc += t;
    }
    wsum[NT / 64] = acc;
  }
  __syncthreads();
  uint32_t run = wsum[wid] + x - s;
  for (int i = lo; i < hi; i++) {
    uint32_t t = a[i];
    a[i] = run;
    run += t;
  }
  const uint32_t total = wsum[NT / 64];
  __syncthreads();
  return total;
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}
__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// ------------------------------------------------------------------------------------------------
// read tile staging

// Stage one extract tile in LDS: for every 32-base group the 2-bit codes (N -> G, the reference's
// get_kmers bit trick, src/kmer.cpp:169,187-188), the "extension countable" bit (quality >= cutoff,
// i.e. the base was not lowercased by count_kmers, src/kcount/kcount.cpp:80-85, and it is not N,
// which ExtCounts::inc ignores, src/kcount/kcount_cpu.cpp:157-164) and the read-start bit.
// Group g of the tile is global group tile*T/32 - 1 + g (one group of left halo).
template <int NL>
__device__ void load_tile(const ReadsView &rv, uint32_t tile, uint32_t first_read, int qcut, uint64_t *fwd,
                          uint32_t *good, uint32_t *start, unsigned int *err, const uint32_t *tile_starts = nullptr) {
  constexpr int T = kTile<NL>(), NG = kGroups<NL>();
  const int64_t gA = (int64_t)tile * (T / 32) - 1;
  for (int g = threadIdx.x; g < NG; g += blockDim.x) {
    const int64_t gi = gA + g;
    // the group's read-start word first, so that its load is in flight with the bases' (issued after them it was
    // a second global round trip per tile: the bases' loads are waited for and decoded before it)
    const uint32_t sw = tile_starts ? gload(tile_starts + (uint64_t)tile * (T / 32) + g) : 0u;
    uint64_t f = 0;
    uint32_t gd = 0;
    if (gi >= 0 && (uint64_t)gi * 32 < rv.n_bases) {
      const uint64_t pos = (uint64_t)gi * 32;
      const uint64_t rem = rv.n_bases - pos;
      uint32_t wv[8];
      if (rem >= 32 && ((((uintptr_t)(rv.bytes + pos)) & 15) == 0)) {
        const uint4 *q = (const uint4 *)(rv.bytes + pos);
        const uint4 v0 = q[0], v1 = q[1];
        wv[0] = v0.x, wv[1] = v0.y, wv[2] = v0.z, wv[3] = v0.w;
        wv[4] = v1.x, wv[5] = v1.y, wv[6] = v1.z, wv[7] = v1.w;
      } else {
#pragma unroll
        for (int i = 0; i < 8; i++) {
          uint32_t x = 0;
#pragma unroll
          for (int bj = 0; bj < 4; bj++) {
            const uint64_t j = 4 * i + bj;
            if (j < rem) x |= (uint32_t)rv.bytes[pos + j] << (8 * bj);
          }
          wv[i] = x;
        }
      }
      // SWAR over 4 bytes: c = base code (A,C,G,T,N = 0..4; 5..7 bad), q = min(quality, 31).
      // Bytes past the data are zero (code A, quality 0) and are never inside a counted window.
      // bit 7 of each byte of q + qbias is q >= qcut (qcut clamped to [0, 32]: q <= 31)
      const uint32_t qbias = 0x80808080u - 0x01010101u * (uint32_t)min(max(qcut, 0), 32);
      uint32_t bad = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const uint32_t c = wv[i] & 0x07070707u, q = (wv[i] >> 3) & 0x1f1f1f1fu;
        const uint32_t t = (c & 0x03030303u) | ((c >> 1) & 0x02020202u);  // N (4) -> G (2)
        const uint32_t ok = (~c >> 2) & ((q + qbias) >> 7) & 0x01010101u;  // code < 4 && q >= qcut
        bad |= (c + 0x03030303u) & 0x08080808u;                            // code > 4
        const uint32_t t8 = ((t & 3u) << 6) | ((t >> 4) & 0x30u) | ((t >> 14) & 0x0cu) | ((t >> 24) & 3u);
        const uint32_t g4 = ((ok & 1u) << 3) | ((ok >> 6) & 4u) | ((ok >> 15) & 2u) | ((ok >> 24) & 1u);
        f |= (uint64_t)t8 << (56 - 8 * i);
        gd |= g4 << (28 - 4 * i);
      }
      if (bad) atomicOr(err, 1u);
    }
    fwd[g] = f;
    good[g] = gd;
    start[g] = sw;
  }
  __syncthreads();
  if (tile_starts) return;  // (uniform) the bitmap came precomputed: no dependent load of the tile's first read
  const int64_t lo = gA * 32, hi = (gA + NG) * 32;
  for (uint64_t r = (uint64_t)first_read + threadIdx.x; r <= rv.n_reads; r += blockDim.x) {
    const int64_t s = (int64_t)(rv.offs[r] - rv.obase);
    if (s >= hi) break;
    if (s >= lo) {
      const int64_t d = s - lo;
      atomicOr(&start[d >> 5], 1u << (31 - (d & 31)));
    }
  }
  __syncthreads();
}

// First read start at or after tile-local position q (LARGE when none in the staged groups).
template <int NL>
__device__ __forceinline__ int next_start(const uint32_t *start, int q) {
  constexpr int NG = kGroups<NL>();
  int g = q >> 5;
  uint32_t m = start[g] & (~0u >> (q & 31));
  while (m == 0) {
    if (++g >= NG) return 1 << 30;
    m = start[g];
  }
  return g * 32 + __clz(m);
}

// Walk the W consecutive windows of this thread (tile positions W*tid .. W*tid + W-1), rolling the
// forward and reverse-complement words by one base per window instead of re-extracting them.
// A window is counted iff it and both neighbours lie in one read: the interior windows i in [1, L-k-1]
// of get_kmers_and_exts (src/kcount/kcount_cpu.cpp:316-334); at one rank the supermer is the read
// (kcount_cpu.cpp:84-101). Canonical = min(fwd, revcomp) (kcount_cpu.cpp:326-332);
// extensions are the neighbour bases, '0' (none) when low quality, complemented and swapped when the
// reverse complement is used (comp_nucleotide, src/utils.cpp:121-143).
//
// Branch-free: the incoming bases, their quality bits and the read starts of the thread's span are
// funnel-loaded into registers once, so the fully unrolled loop is straight-line ALU work with
// constant shifts. Window p (tile position) is valid iff the last read start at or before p + k
// (tracked in `last`) is before p, and p + k is inside the data. emit(i, key, ext, valid) is called for
// every window; key/ext are meaningless when !valid.
template <int NL, int KC = 0, typename Emit>
__device__ __forceinline__ void walk_windows(const uint64_t *fwd, const uint32_t *good, const uint32_t *start,
                                             uint32_t tile, uint64_t n_bases, uint32_t head, int k_rt, Emit &&emit) {
  constexpr int T = kTile<NL>(), W = T / kEThreads<NL>();
  const int k = KC ? KC : k_rt;  // (KC > 0: k as a compile-time constant)
  static_assert(W <= 32, "one 32-bit mask per thread span");
  const int klast = k - 32 * (NL - 1);
  const uint64_t tmask = top_mask(klast);
  const int lp0 = 32 + W * (int)threadIdx.x;
  auto codes64 = [&](int q) {  // the 32 codes from tile position q, first in the top bits
    const int g = q >> 5, sh = (q & 31) * 2;
    uint64_t v = fwd[g];
    if (sh) v = (v << sh) | (fwd[g + 1] >> (64 - sh));
    return v;
  };
  auto bits32 = [&](const uint32_t *a, int q) {  // the 32 bits from tile position q, first in bit 31
    const int g = q >> 5, sh = q & 31;
    uint32_t v = a[g];
    if (sh) v = (v << sh) | (a[g + 1] >> (32 - sh));
    return v;
  };
  uint64_t fw[NL], rc[NL];
#pragma unroll
  for (int m = 0; m < NL; m++) fw[m] = codes64(lp0 + 32 * m);
  fw[NL - 1] &= tmask;
  revcomp<NL>(fw, rc, k);
  const uint64_t incoming = codes64(lp0 + k);         // base entering at window i: lp0 + k + i
  const uint32_t gl_bits = bits32(good, lp0 - 1);      // left neighbour of window i: lp0 - 1 + i
  const uint32_t gr_bits = bits32(good, lp0 + k);      // right neighbour: lp0 + k + i
  const uint32_t st_bits = bits32(start, lp0 + k);     // read starts at lp0 + k + i
  // last read start in [lp0, lp0 + k - 1] (at most 5 groups), else lp0 - 1
  int last = lp0 - 1;
  {
    const int q0 = lp0, q1 = lp0 + k - 1;
    for (int g = q1 >> 5; g >= (q0 >> 5); g--) {
      uint32_t m = start[g];
      const int lo = max(q0, g * 32), hi = min(q1, g * 32 + 31);
      m &= (~0u >> (lo - g * 32)) & (~0u << (31 - (hi - g * 32)));
      if (m) {
        last = g * 32 + 31 - (__ffs(m) - 1);
        break;
      }
    }
  }
  // data end in tile positions: window p needs p + k < end (p + k is the right neighbour)
  const int64_t end64 = (int64_t)n_bases - ((int64_t)tile * T - 32);
  const int end = end64 > (int64_t)(1 << 30) ? (1 << 30) : (int)end64;
  // data begin (a slice view): window p needs its left neighbour p - 1 at or after the view's head
  const int beg = tile == 0 ? (int)head + 32 : -(1 << 30);
  uint32_t cl = (uint32_t)(codes64(lp0 - 1) >> 62);
#pragma unroll
  for (int i = 0; i < W; i++) {
    const int lp = lp0 + i;
    const uint32_t cr = (uint32_t)(incoming >> (62 - 2 * i)) & 3u;
    const uint32_t gl = (gl_bits >> (31 - i)) & 1u, gr = (gr_bits >> (31 - i)) & 1u;
    if ((st_bits >> (31 - i)) & 1u) last = lp + k;
    const bool valid = (last < lp) && (lp + k < end) && (lp > beg);
    int l = gl ? (int)cl : EXT_NONE, r = gr ? (int)cr : EXT_NONE;
    const bool use_rc = kmer_less<NL>(rc, fw);
    uint64_t key[NL];
#pragma unroll
    for (int m = 0; m < NL; m++) key[m] = use_rc ? rc[m] : fw[m];
    const int lr = (r == EXT_NONE) ? EXT_NONE : 3 - r, rr = (l == EXT_NONE) ? EXT_NONE : 3 - l;
    if (use_rc) {
      l = lr;
      r = rr;
    }
    emit(i, key, (uint32_t)((l << 3) | r), valid);
    // roll to the next window: base lp leaves, base lp + k (cr) enters
    cl = (uint32_t)(fw[0] >> 62);
#pragma unroll
    for (int m = 0; m < NL - 1; m++) fw[m] = (fw[m] << 2) | (fw[m + 1] >> 62);
    fw[NL - 1] = (fw[NL - 1] << 2) | ((uint64_t)cr << (64 - 2 * klast));
#pragma unroll
    for (int m = NL - 1; m > 0; m--) rc[m] = (rc[m] >> 2) | (rc[m - 1] << 62);
    rc[0] = (rc[0] >> 2) | ((uint64_t)(3u - cr) << 62);
    rc[NL - 1] &= tmask;
  }
}

// The per-thread span of walk_windows, for the mixed-record walks below: the bits of the W windows' neighbours
// and read starts, the last read start before the span and the data bounds (see walk_windows).
template <int NL>
struct WalkSpan {
  int lp0, last, end, beg;
  uint64_t incoming;                 // the base entering at window i: bits 63 - 2i, 62 - 2i
  uint32_t gl_bits, gr_bits, st_bits, cl;
  __device__ __forceinline__ WalkSpan(const uint64_t *fwd, const uint32_t *good, const uint32_t *start, uint32_t tile,
                                      uint64_t n_bases, uint32_t head, int k) {
    constexpr int T = kTile<NL>(), W = T / kEThreads<NL>();
    lp0 = 32 + W * (int)threadIdx.x;
    incoming = codes64(fwd, lp0 + k);
    gl_bits = bits32(good, lp0 - 1);
    gr_bits = bits32(good, lp0 + k);
    st_bits = bits32(start, lp0 + k);
    last = lp0 - 1;
    const int q0 = lp0, q1 = lp0 + k - 1;
    for (int g = q1 >> 5; g >= (q0 >> 5); g--) {
      uint32_t m = start[g];
      const int lo = max(q0, g * 32), hi = min(q1, g * 32 + 31);
      m &= (~0u >> (lo - g * 32)) & (~0u << (31 - (hi - g * 32)));
      if (m) {
        last = g * 32 + 31 - (__ffs(m) - 1);
        break;
      }
    }
    const int64_t end64 = (int64_t)n_bases - ((int64_t)tile * T - 32);
    end = end64 > (int64_t)(1 << 30) ? (1 << 30) : (int)end64;
    beg = tile == 0 ? (int)head + 32 : -(1 << 30);
    cl = (uint32_t)(codes64(fwd, lp0 - 1) >> 62);
  }
  static __device__ __forceinline__ uint64_t codes64(const uint64_t *fwd, int q) {  // 32 codes from q, first on top
    const int g = q >> 5, sh = (q & 31) * 2;
    uint64_t v = fwd[g];
    if (sh) v = (v << sh) | (fwd[g + 1] >> (64 - sh));
    return v;
  }
  static __device__ __forceinline__ uint32_t bits32(const uint32_t *a, int q) {  // 32 bits from q, first in bit 31
    const int g = q >> 5, sh = q & 31;
    uint32_t v = a[g];
    if (sh) v = (v << sh) | (a[g + 1] >> (32 - sh));
    return v;
  }
  // window i: the entering base (its right neighbour), the ext code in both orientations, validity
  __device__ __forceinline__ bool step(int i, int k, uint32_t &cr, uint32_t &e_f, uint32_t &e_r) {
    const int lp = lp0 + i;
    cr = (uint32_t)(incoming >> (62 - 2 * i)) & 3u;
    const bool gl = (gl_bits >> (31 - i)) & 1u, gr = (gr_bits >> (31 - i)) & 1u;
    if ((st_bits >> (31 - i)) & 1u) last = lp + k;
    const uint32_t l = gl ? cl : (uint32_t)EXT_NONE, r = gr ? cr : (uint32_t)EXT_NONE;
    const uint32_t lr = gr ? cr ^ 3u : (uint32_t)EXT_NONE, rr = gl ? cl ^ 3u : (uint32_t)EXT_NONE;
    e_f = (l << 3) | r;   // forward: (left << 3) | right
    e_r = (lr << 3) | rr;  // reverse complement: complemented and swapped
    return (last < lp) && (lp + k < end) && (lp > beg);
  }
  // The validity of all W windows at once (W + k + 1 <= 64): window i is valid iff no read starts in
  // [lp0 + i, lp0 + i + k] (then `last` < lp in step) and it is inside the data. One OR-window of width k + 1 over the
  // span's read-start bits (log steps) replaces step's per-window start test, compare and select (the extraction is
  // VALU-issue bound).
  __device__ __forceinline__ uint32_t valid_mask(const uint32_t *start, int k) const {
    const uint64_t X = __brevll(((uint64_t)bits32(start, lp0) << 32) | bits32(start, lp0 + 32));  // bit j: lp0 + j
    uint64_t A = X | (X >> 1);
    A |= A >> 2;
    A |= A >> 4;  // bit j: a start in [j, j + 8)
    const int w = k + 1;
    if (w > 16) {
      A |= A >> 8;
      A |= A >> (w - 16);
    } else {
      A |= A >> (w - 8);
    }
    uint32_t m = ~(uint32_t)A;
    const int hi = end - lp0 - k, lo = beg - lp0;  // valid iff lo < i < hi
    m &= hi >= 32 ? ~0u : hi <= 0 ? 0u : (1u << hi) - 1u;
    m &= lo < 0 ? ~0u : lo >= 31 ? 0u : ~0u << (lo + 1);
    return m;
  }
  // valid_mask for 32 < k < 64 (two-word keys: W + k + 1 <= 80 positions): the OR-window over the span's first 64
  // positions, and a start at lp0 + 64 + j in the next 32 invalidates the windows i >= 64 + j - k
  __device__ __forceinline__ uint32_t valid_mask_wide(const uint32_t *start, int k) const {
    const uint64_t X = __brevll(((uint64_t)bits32(start, lp0) << 32) | bits32(start, lp0 + 32));
    uint64_t A = X | (X >> 1);
    A |= A >> 2;
    A |= A >> 4;
    A |= A >> 8;
    A |= A >> 16;  // bit j: a start in [j, j + 32)
    A |= A >> (k + 1 - 32);
    uint32_t P = __brev(bits32(start, lp0 + 64));  // bit j: a start at lp0 + 64 + j
    P |= P << 1;
    P |= P << 2;
    P |= P << 4;
    P |= P << 8;
    P |= P << 16;  // bit j: a start in [lp0 + 64, lp0 + 64 + j]
    uint32_t m = ~(uint32_t)(A | ((uint64_t)P << (64 - k)));
    const int hi = end - lp0 - k, lo = beg - lp0;
    m &= hi >= 32 ? ~0u : hi <= 0 ? 0u : (1u << hi) - 1u;
    m &= lo < 0 ? ~0u : lo >= 31 ? 0u : ~0u << (lo + 1);
    return m;
  }
  // step without the validity (valid_mask)
  __device__ __forceinline__ void step_ext(int i, uint32_t &cr, uint32_t &e_f, uint32_t &e_r) {
    cr = (uint32_t)(incoming >> (62 - 2 * i)) & 3u;
    const bool gl = (gl_bits >> (31 - i)) & 1u, gr = (gr_bits >> (31 - i)) & 1u;
    const uint32_t l = gl ? cl : (uint32_t)EXT_NONE, r = gr ? cr : (uint32_t)EXT_NONE;
    const uint32_t lr = gr ? cr ^ 3u : (uint32_t)EXT_NONE, rr = gl ? cl ^ 3u : (uint32_t)EXT_NONE;
    e_f = (l << 3) | r;
    e_r = (lr << 3) | rr;
  }
};

// Compact-record walk (10 <= k <= 21, §3.7): the windows of walk_windows with the key kept right-aligned in its
// B = 2k bits, the form cmix takes, so no Kmer-layout word is built or shifted into the mix; the record is
// (y below the coarse digit) << 6 | ext with y = cmix(canonical key), the bin the coarse digit (y's top cb bits).
// Each window's record is held in two u32 registers instead of a u64 and an info word: lo = the record's low 32
// bits, hi = valid << 31 | (the record's bits 32..39) << 11 | bin (bits 19..30 stay free for the window's rank in its
// bin, scatter_staged_c40). 48 -> 32 VGPRs of records per thread, so the kernel fits 96 VGPRs (five workgroups per
// CU) without spilling.
template <int W, int KC = 0, int CBC = 0>
__device__ __forceinline__ void walk_c32_lh(const uint64_t *fwd, const uint32_t *good, const uint32_t *start,
                                            uint32_t tile, uint64_t n_bases, uint32_t head, int k_rt, int cb_rt,
                                            uint32_t (&lo)[W], uint32_t (&hi)[W]) {
  // (KC, CBC > 0: k and the coarse bits as compile-time constants)
  const int k = KC ? KC : k_rt, cb = CBC ? CBC : cb_rt;
  WalkSpan<1> sp(fwd, good, start, tile, n_bases, head, k);
  const int B = 2 * k, a = B >> 1, b = B - a, rb = B - cb;
  const uint64_t mB = (1ull << B) - 1, rmask = (1ull << rb) - 1;
  uint64_t fw = WalkSpan<1>::codes64(fwd, sp.lp0) >> (64 - B);
  uint64_t rc = rev2(~fw) >> (64 - B);
  static_assert(W + 21 + 1 <= 64, "valid_mask covers the span");
  const uint32_t vm = sp.valid_mask(start, k);
#pragma unroll
  for (int i = 0; i < W; i++) {
    uint32_t cr, e_f, e_r;
    sp.step_ext(i, cr, e_f, e_r);
    const bool valid = (vm >> i) & 1u;
    const bool use_rc = rc < fw;
    const uint64_t x = use_rc ? rc : fw;
    const uint32_t e = use_rc ? e_r : e_f;
    uint32_t R = (uint32_t)x & ((1u << a) - 1), L = (uint32_t)(x >> a);
    cmix_lr(L, R, a, b);
    const uint64_t y = ((uint64_t)L << a) | R;
    const uint64_t r = ((y & rmask) << EXT_BITS) | e;
    lo[i] = (uint32_t)r;
    hi[i] = valid ? (1u << 31) | (((uint32_t)(r >> 32) & 0xffu) << 11) | (uint32_t)(y >> rb) : 0u;
    asm volatile("" : "+v"(lo[i]), "+v"(hi[i]));
    sp.cl = (uint32_t)(fw >> (B - 2));
    fw = ((fw << 2) | cr) & mB;
    rc = (rc >> 2) | ((uint64_t)(cr ^ 3u) << (B - 2));
  }
}

// Mixed two-word walk (33 <= k <= 63, §3.7b): the 2k-bit key kept as its two k-bit halves (L = the top k bits,
// R = the low k bits), the form m2_mix_lr takes, rolled and compared as halves; record w[0] = (L' below the coarse
// digit) << 6 | ext, w[1] = R', bin = the coarse digit (L''s top cb bits).
template <int W, int KC = 0, int CBC = 0>
__device__ __forceinline__ void walk_m2(const uint64_t *fwd, const uint32_t *good, const uint32_t *start,
                                        uint32_t tile, uint64_t n_bases, uint32_t head, int k_rt, int cb_rt,
                                        uint64_t (&rk)[W][2], uint32_t (&inf)[W]) {
  // (KC, CBC > 0: k and the coarse bits as compile-time constants)
  const int k = KC ? KC : k_rt, cb = CBC ? CBC : cb_rt;
  WalkSpan<2> sp(fwd, good, start, tile, n_bases, head, k);
  const uint64_t mk = (1ull << k) - 1;
  const int csh = k - cb;
  const uint64_t cmask = (1ull << csh) - 1;
  uint64_t fL, fR, rL, rR;
  {
    uint64_t w[2], rw[2];
    w[0] = WalkSpan<2>::codes64(fwd, sp.lp0);
    w[1] = WalkSpan<2>::codes64(fwd, sp.lp0 + 32) & top_mask(k - 32);
    revcomp<2>(w, rw, k);
    fL = w[0] >> (64 - k);
    fR = ((w[0] << (2 * k - 64)) | (w[1] >> (128 - 2 * k))) & mk;
    rL = rw[0] >> (64 - k);
    rR = ((rw[0] << (2 * k - 64)) | (rw[1] >> (128 - 2 * k))) & mk;
  }
  static_assert(W + 63 + 1 <= 96, "valid_mask_wide covers the span");
  const uint32_t vm = sp.valid_mask_wide(start, k);
#pragma unroll
  for (int i = 0; i < W; i++) {
    uint32_t cr, e_f, e_r;
    sp.step_ext(i, cr, e_f, e_r);
    const bool valid = (vm >> i) & 1u;
    const bool use_rc = (rL < fL) | ((rL == fL) & (rR < fR));
    uint64_t L = use_rc ? rL : fL, R = use_rc ? rR : fR;
    const uint32_t e = use_rc ? e_r : e_f;
    m2_mix_lr(L, R, k);
    rk[i][0] = ((L & cmask) << EXT_BITS) | e;
    rk[i][1] = R;
    inf[i] = valid ? (1u << 31) | (e << 16) | (uint32_t)(L >> csh) : 0u;
    asm volatile("" : "+v"(rk[i][0]), "+v"(rk[i][1]), "+v"(inf[i]));
    // roll the halves: the 2k-bit forward key shifts left by one base, the reverse complement right
    sp.cl = (uint32_t)(fL >> (k - 2));
    fL = ((fL << 2) | (fR >> (k - 2))) & mk;
    fR = ((fR << 2) | cr) & mk;
    rR = (rR >> 2) | ((rL & 3u) << (k - 2));
    rL = (rL >> 2) | ((uint64_t)(cr ^ 3u) << (k - 2));
  }
}

// ------------------------------------------------------------------------------------------------
// tile index

__global__ void k_tile_first_read(ReadsView rv, uint32_t *out, uint32_t n_tiles, int tile) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_tiles) return;
  const int64_t lo64 = (int64_t)t * tile - 32;
  const uint64_t lo = lo64 < 0 ? 0 : (uint64_t)lo64;
  uint64_t a = 0, b = rv.n_reads + 1;  // lower_bound over offs[0..n_reads]
  while (a < b) {
    const uint64_t m = (a + b) >> 1;
    if (rv.offs[m] - rv.obase < lo)
      a = m + 1;
    else
      b = m;
  }
  out[t] = (uint32_t)a;
}

// Read-start bits of a batch (or slice view), flat: bit 31 - (s & 31) of word (s >> 5) + 1 for every read start (and
// the end) at position s from the view's base; word 0 is the group left of position 0 (tile 0's halo), so a tile's
// kGroups<NL>() staged groups are words [tile T / 32, tile T / 32 + kGroups) (load_tile). The extraction then loads its
// tile's start words beside the bases instead of first loading the tile's first read and then the offsets after it,
// two dependent global round trips per tile. Every word is written once, by the read that starts first in it or whose
// start precedes it: thread r writes its start's word (with the bits of the later reads starting in it) and zeros up
// to the next start's word; the first read also the words before its own, the end the words after. (Per-tile bitmaps
// by one wave per tile from a searched first read took 37 + 87 us at C2; a zeroed array and one atomicOr per read
// 26 + 118 us.)
__global__ __launch_bounds__(256) void k_read_start_bits(ReadsView rv, uint32_t *bits, uint64_t n_words) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r <= rv.n_reads; r += stride) {
    const uint64_t s = rv.offs[r] - rv.obase, w = (s >> 5) + 1;
    if (r > 0 && ((rv.offs[r - 1] - rv.obase) >> 5) + 1 == w) continue;  // an earlier read starts in this word
    uint32_t v = 1u << (31 - (uint32_t)(s & 31));
    uint64_t wn = n_words;  // the next word holding a start
    for (uint64_t q = r + 1; q <= rv.n_reads; q++) {
      const uint64_t sq = rv.offs[q] - rv.obase, wq = (sq >> 5) + 1;
      if (wq != w) {
        wn = wq;
        break;
      }
      v |= 1u << (31 - (uint32_t)(sq & 31));
    }
    bits[w] = v;
    for (uint64_t x = w + 1; x < wn; x++) bits[x] = 0;
    if (r == 0)
      for (uint64_t x = 0; x < w; x++) bits[x] = 0;
  }
}

// ------------------------------------------------------------------------------------------------
// extract: histogram

// Partition hash of a window's key: MurmurHash3 h1 (part_hash), or the key bijection of mixed records
// (compact: cmix; two words: L' of m2_mix), left-aligned so that the digits are its top bits.
template <int NL, bool CMP>
__device__ __forceinline__ uint64_t window_hash(const uint64_t *key, int k) {
  if (CMP && NL == 1) return cpart_hash(key[0], 2 * k);
  if (CMP && NL == 2) {
    uint64_t L, R;
    m2_mix(key, k, L, R);
    return L << (64 - k);
  }
  if (CMP && NL >= 3) {  // mixed three- and four-word records: w0' of mx_mix
    uint64_t r[NL];
    mx_mix<NL>(key, r);
    return r[0];
  }
  return part_hash<NL>(key);
}

// Record layout traits: compact (one u32 word, NL = 1), mixed two-word records (NL = 2, ext code in w[0],
// kmer_ops.hpp m2_mix) and mixed three- and four-word records (NL = 3, 4, ext code in w[0], mx_mix) are the kinds
// of "mixed" records (CMP) whose bucket digits are implicit. LW: bits of the mixed first word whose top bits are the
// digits (L' of k bits, w0' of 64).
template <int NL, bool CMP>
struct RecKind {
  static constexpr bool C32 = CMP && NL == 1;
  static constexpr bool M2 = CMP && NL == 2;
  static constexpr bool MX = CMP && NL >= 3;
  static constexpr bool MW = M2 || MX;  // multi-word mixed: w[0] = (first mixed word below the digits) << 6 | ext
  static constexpr int XW = MW ? 0 : NL - 1;  // the word holding the ext code of a packed record
  static __host__ __device__ constexpr int lw(int k) { return M2 ? k : 64; }
};

template <int NL, bool PACKED, bool CMP>
__global__ __launch_bounds__(kEThreads<NL>()) void k_extract_hist(ExtractParams p) {
  constexpr int ET = kEThreads<NL>(), T = kTile<NL>(), W = T / ET;
  extern __shared__ __align__(16) unsigned char smem[];
  uint64_t *fwd;
  uint32_t *good, *start;
  unsigned char *rest = carve_tile<NL>(smem, fwd, good, start);
  uint32_t *hist = (uint32_t *)rest;
  for (uint32_t b = threadIdx.x; b < p.n_bins; b += ET) hist[b] = 0;
  const uint32_t tile = blockIdx.x;
  load_tile<NL>(p.reads, tile, p.tile_starts ? 0u : p.tile_first_read[tile], p.qual_cutoff, fwd, good, start, p.err,
                p.tile_starts);
  const int sh = 64 - p.coarse_bits;
  walk_windows<NL>(fwd, good, start, tile, p.reads.n_bases, p.reads.head, p.k, [&](int, const uint64_t *key, uint32_t, bool valid) {
    if (valid) atomicAdd(&hist[(uint32_t)(window_hash<NL, CMP>(key, p.k) >> sh)], 1u);
  });
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < p.n_bins; b += ET) {
    const uint32_t c = hist[b];
    if (c) atomicAdd(&p.hist[b], (unsigned long long)c);
  }
}

// ------------------------------------------------------------------------------------------------
// Register-resident scatter shared by extract_scatter and part_scatter.
// Each thread holds its W records (rk, inf = valid<<31 | e<<16 | bin). LDS only holds per-bin counters:
// a returning LDS atomic ranks every record inside its bin, one global atomic per non-empty bin reserves
// the workgroup's run, and every lane stores its own records. The stores of one bin land in the same
// segment, which is written by blocks of one XCD only (E_NSUB segments per coarse bucket, fine buckets
// per coarse bucket), so partial lines merge in that XCD's L2 before they reach HBM.
// LDS: lcnt[nb] u32 | pad to 16 B | goff[nb] u64.

// Global store formats of a scatter: the record words (+ the ext byte plane when not packed), or a
// compact record (kmer_ops.hpp cmix) split into a u32 plane w[0] + a byte plane ext (coarse buckets,
// <= 40 bits) or a u32 plane alone (fine buckets, <= 32 bits).
// SF_AOS2: two-word records as one 16-byte record (the records of mixed two-word keys: a bucket's run of a tile or
// chunk is one contiguous span, and a record one 16-byte load), staged in LDS as 16-byte records too
enum { SF_WORDS = 0, SF_C40 = 1, SF_C32 = 2, SF_AOS2 = 3 };

template <int NL, bool PACKED, int SF>
__device__ __forceinline__ void store_out(const PlaneSet &out, uint64_t dst, const uint64_t *v, uint32_t ext) {
  if (SF == SF_C40) {
    ((uint32_t *)out.w[0])[dst] = (uint32_t)v[0];
    out.ext[dst] = (uint8_t)(v[0] >> 32);
  } else if (SF == SF_C32) {
    ((uint32_t *)out.w[0])[dst] = (uint32_t)v[0];
  } else if (SF == SF_AOS2) {
    ((ulonglong2 *)out.w[0])[dst] = make_ulonglong2(v[0], v[1]);
  } else {
#pragma unroll
    for (int w = 0; w < NL; w++) out.w[w][dst] = v[w];
    if (!PACKED) out.ext[dst] = (uint8_t)ext;
  }
}

// Bin limits of capped layouts: bin b may use [.., lim.base + b * lim.stride + lim.cap); lim.cap == 0: none.
struct BinLimit {
  uint64_t base, stride, cap;
  __device__ __forceinline__ uint64_t end(uint32_t b) const { return base + (uint64_t)b * stride + cap; }
};

__host__ __device__ constexpr size_t scatter_cnt_bytes(uint32_t nb) { return ((size_t)nb * 4 + 15) & ~(size_t)15; }
__host__ __device__ constexpr size_t scatter_lds_bytes(uint32_t nb) { return scatter_cnt_bytes(nb) + (size_t)nb * 8; }

template <int NT = E_THREADS>
__device__ __forceinline__ void scatter_clear(uint32_t *lcnt, uint32_t nb) {
  for (uint32_t b = threadIdx.x; b < nb; b += NT) lcnt[b] = 0;
}

constexpr size_t WSUM_BYTES = ((1024 / 64 + 1) * 4 + 15) & ~(size_t)15;  // block_excl_scan's wave sums (<= 1024 threads)

// The scatter of extraction and partition. Every thread holds its W records (rk, inf = valid<<31 | e<<16 | bin); a
// returning LDS atomic ranks every record inside its bin, one global atomic per non-empty bin reserves the
// workgroup's run, the records are written to LDS in bin order, and then copied out so that consecutive lanes store
// consecutive addresses of one bin (runs of ~T/nb records instead of one line per lane; a register scatter took
// extraction 8.1 -> 14.3 ms, §4.2). The stores of one bin land in the same segment, which is written by workgroups
// of one XCD only (E_NSUB segments per coarse bucket, fine buckets per coarse bucket), so partial lines merge in that
// XCD's L2 before they reach HBM. Bin b's cursor is cursor[b * cstride]; in a capped layout a bin that would
// overflow sets err bit 1 and its records are not written (the host then redoes the pass with exact bin sizes).
// LDS: counters [lcnt | goff | wsum] then the stage area [NL][T] u64 | sbin[T] u16 | sext[T] u8, which may alias
// the tile (the first barrier below is after every thread's walk). The bins' run starts reuse the rank counters
// (lcnt): each thread reads its bins' counts, then overwrites the same entries. At k = 21 this keeps an extraction
// workgroup's LDS (counters + the staged tile) under 32 KiB, five per CU.
__host__ __device__ constexpr size_t staged_cnt_bytes(uint32_t nb) { return scatter_lds_bytes(nb) + WSUM_BYTES; }
// Compact records are staged at their stored width: u32 (+ the high byte for SF_C40).
__host__ __device__ constexpr size_t staged_area_bytes(int nl, int T, bool packed, int sf = SF_WORDS) {
  return sf == SF_C40   ? (size_t)T * (4 + 1 + 2)
         : sf == SF_C32 ? (size_t)T * (4 + 2)
                        : (size_t)nl * T * 8 + (size_t)T * 2 + (packed ? 0 : (size_t)T);
}

// CAP < W * NT: the stage area holds CAP records and the records go out in rounds of CAP (bin order), so a
// workgroup whose windows are mostly not counted (k = 77, 99 on 150-base reads: 48 %, 33 % counted) needs LDS for
// the records it has, not for one per window.
template <int NL, bool PACKED, int W, int SF, int NT = E_THREADS, int CAP = W * NT, int BPT = 8>  // BPT: as scatter_staged_c40
__device__ __forceinline__ void scatter_staged(const uint64_t (&rk)[W][NL], const uint32_t (&inf)[W], uint32_t nb,
                                               unsigned char *smem, unsigned char *area,
                                               unsigned long long *cursor, uint32_t cstride, const PlaneSet &out,
                                               const BinLimit lim, unsigned int *err) {
  constexpr int T = CAP;
  static_assert(CAP <= W * NT && CAP % NT == 0, "stage capacity: whole rows of the workgroup");
  uint32_t *lcnt = (uint32_t *)smem;
  unsigned long long *goff = (unsigned long long *)(smem + scatter_cnt_bytes(nb));
  uint32_t *lstart = lcnt;
  uint32_t *wsum = (uint32_t *)(smem + staged_cnt_bytes(nb) - WSUM_BYTES);
  constexpr bool C32 = SF == SF_C40 || SF == SF_C32;  // compact: low 32 bits in stage32, the high byte (SF_C40) in sext
  uint64_t *stage = (uint64_t *)area;
  uint32_t *stage32 = (uint32_t *)area;
  uint16_t *sbin = C32 ? (uint16_t *)(stage32 + T) : (uint16_t *)(stage + NL * T);
  uint8_t *sext = (uint8_t *)(sbin + T);
  // One- and two-word records (BATCH): every rank atomic issued before any result is used (see scatter_staged_c40);
  // uncounted windows add 0 to a word of their own lane in goff (free until the bins' offsets are written). Three- and
  // four-word records keep one atomic per counted window: the batched phases cost their kernels a wave per SIMD.
  constexpr bool BATCH = NL <= 2;
  uint32_t rank[W];
  if constexpr (BATCH) {
    uint32_t *const dummy = (uint32_t *)goff + (threadIdx.x & 63u);
#pragma unroll
    for (int j = 0; j < W; j++) {
      const bool v = inf[j] >> 31;
      rank[j] = atomicAdd(v ? &lcnt[inf[j] & 0xffffu] : dummy, v ? 1u : 0u);
    }
  } else {
#pragma unroll
    for (int j = 0; j < W; j++) rank[j] = (inf[j] >> 31) ? atomicAdd(&lcnt[inf[j] & 0xffffu], 1u) : 0u;
  }
  __syncthreads();
  // Reserve each bin's run in the global layout. The returned offsets stay in registers while the bins are
  // scanned and the records staged, so the atomics' round trip overlaps that LDS work (a bin count up to
  // SCATTER_MAX_BINS = 8 * NT).
  unsigned long long off[BPT];
  uint32_t cnt[BPT];
#pragma unroll
  for (int i = 0; i < BPT; i++) {
    const uint32_t b = threadIdx.x + i * NT;
    off[i] = 0;
    cnt[i] = 0;
    if (b < nb) {
      const uint32_t c = lcnt[b];
      cnt[i] = c;
      if (c) off[i] = atomicAdd(&cursor[(uint64_t)b * cstride], (unsigned long long)c);
      lstart[b] = c;
    }
  }
  __syncthreads();
  const uint32_t total = block_excl_scan<NT>(lstart, (int)nb, wsum);
  for (uint32_t r0 = 0; r0 < total; r0 += CAP) {  // (uniform) one round when CAP = W * NT
  if (r0) __syncthreads();  // the previous round's copy-out has read the stage area
  // the bins' run starts of all W records read first (BATCH, see scatter_staged_c40)
  uint32_t st_[BATCH ? W : 1];
  if constexpr (BATCH) {
#pragma unroll
    for (int j = 0; j < W; j++) st_[j] = lstart[inf[j] & 0xffffu];
  }
#pragma unroll
  for (int j = 0; j < W; j++) {
    if (inf[j] >> 31) {
      const uint32_t d = inf[j] & 0xffffu;
      const uint32_t pos = (BATCH ? st_[BATCH ? j : 0] : lstart[d]) + rank[j] - r0;  // (earlier rounds' records wrap to >= CAP)
      if (CAP < W * NT && pos >= (uint32_t)CAP) continue;
      if (C32) {
        stage32[pos] = (uint32_t)rk[j][0];
        if (SF == SF_C40) sext[pos] = (uint8_t)(rk[j][0] >> 32);
      } else if (SF == SF_AOS2) {  // one 16-byte LDS write per record
        ((ulonglong2 *)stage)[pos] = make_ulonglong2(rk[j][0], rk[j][NL - 1]);
      } else {
#pragma unroll
        for (int w = 0; w < NL; w++) stage[w * T + pos] = rk[j][w];
      }
      sbin[pos] = (uint16_t)d;
      if (!PACKED) sext[pos] = (uint8_t)((inf[j] >> 16) & 63u);
    }
  }
  // A bin that overflows its capped segment flags the pass (the host redoes it with exact sizes) and writes
  // nothing: its run offset becomes ~0, so the copy-out below tests one loaded word per record instead of
  // recomputing the segment end (a 64-bit multiply per record)
  if (r0 == 0) {
#pragma unroll
  for (int i = 0; i < BPT; i++) {
    const uint32_t b = threadIdx.x + i * NT;
    if (b < nb) {
      const bool over = lim.cap && cnt[i] && off[i] + cnt[i] > lim.end(b);
      if (over) atomicOr(err, 2u);
      goff[b] = over ? ~0ull : off[i];
    }
  }
  }
  __syncthreads();
  // the copy-out in batches of CB records whose LDS reads are all issued before the first global store (see
  // scatter_staged_c40)
  constexpr int NJ = CAP / NT, CB = !BATCH ? 1 : NJ % 4 == 0 ? 4 : NJ % 2 == 0 ? 2 : 1;
#pragma unroll
  for (int j0 = 0; j0 < NJ; j0 += CB) {
    uint32_t d[CB], ls[CB], xe[CB];
    unsigned long long go[CB];
    uint64_t v[CB][NL];
#pragma unroll
    for (int jj = 0; jj < CB; jj++) d[jj] = sbin[threadIdx.x + (j0 + jj) * NT];  // (past total: stale, unused)
#pragma unroll
    for (int jj = 0; jj < CB; jj++) {
      const uint32_t sp = threadIdx.x + (j0 + jj) * NT;
      const uint32_t dd = d[jj] < nb ? d[jj] : 0u;
      go[jj] = goff[dd];
      ls[jj] = lstart[dd];
      if (C32) {
        v[jj][0] = (uint64_t)stage32[sp] | (SF == SF_C40 ? (uint64_t)sext[sp] << 32 : 0ull);
      } else if (SF == SF_AOS2) {
        const ulonglong2 q = ((const ulonglong2 *)stage)[sp];
        v[jj][0] = q.x;
        v[jj][NL - 1] = q.y;
      } else {
#pragma unroll
        for (int w = 0; w < NL; w++) v[jj][w] = stage[w * T + sp];
      }
      xe[jj] = PACKED ? 0u : sext[sp];
    }
#pragma unroll
    for (int jj = 0; jj < CB; jj++) {
      const uint32_t sp = threadIdx.x + (j0 + jj) * NT, pos = sp + r0;  // stage slot, position in the workgroup's run
      if (pos < total && go[jj] != ~0ull) store_out<NL, PACKED, SF>(out, go[jj] + (pos - ls[jj]), v[jj], xe[jj]);
    }
  }
  }  // rounds
}

// scatter_staged for compact 40-bit records held as lo / hi words (walk_c32_lh): the window's rank in its bin
// goes into hi's free bits 19..30 instead of a register of its own (bins <= 2048, T <= 4096).
template <int W, int NT, bool HB = true, int BPT = 8>  // HB: the record's top byte goes to the ext plane (false: u32
// records); BPT: bins per thread, nb <= BPT * NT (1: the usual 256 fine bins over 256 threads in 21 fewer VGPRs)
__device__ __forceinline__ void scatter_staged_c40(uint32_t (&lo)[W], uint32_t (&hi)[W], uint32_t nb,
                                                   unsigned char *smem, unsigned char *area,
                                                   unsigned long long *cursor, const PlaneSet &out,
                                                   const BinLimit lim, unsigned int *err) {
  constexpr int T = W * NT;
  static_assert(T <= 4096 && 8 * NT <= 2048, "rank in 12 bits, bin in 11");
  uint32_t *lcnt = (uint32_t *)smem;
  unsigned long long *goff = (unsigned long long *)(smem + scatter_cnt_bytes(nb));
  uint32_t *lstart = lcnt;
  uint32_t *wsum = (uint32_t *)(smem + staged_cnt_bytes(nb) - WSUM_BYTES);
  uint32_t *stage32 = (uint32_t *)area;
  uint16_t *sbin = (uint16_t *)(stage32 + T);
  uint8_t *sext = (uint8_t *)(sbin + T);
#pragma unroll
  for (int j = 0; j < W; j++)
    if (hi[j] >> 31) hi[j] |= atomicAdd(&lcnt[hi[j] & 0x7ffu], 1u) << 19;
  __syncthreads();
  unsigned long long off[BPT];
  uint32_t cnt[BPT];
#pragma unroll
  for (int i = 0; i < BPT; i++) {
    const uint32_t b = threadIdx.x + i * NT;
    off[i] = 0;
    cnt[i] = 0;
    if (b < nb) {
      const uint32_t c = lcnt[b];
      cnt[i] = c;
      if (c) off[i] = atomicAdd(&cursor[b], (unsigned long long)c);
      lstart[b] = c;
    }
  }
  __syncthreads();
  const uint32_t total = block_excl_scan<NT>(lstart, (int)nb, wsum);
#pragma unroll
  for (int j = 0; j < W; j++) {
    if (hi[j] >> 31) {
      const uint32_t d = hi[j] & 0x7ffu;
      const uint32_t pos = lstart[d] + ((hi[j] >> 19) & 0xfffu);
      stage32[pos] = lo[j];
      if (HB) sext[pos] = (uint8_t)(hi[j] >> 11);
      sbin[pos] = (uint16_t)d;
    }
  }
#pragma unroll
  for (int i = 0; i < BPT; i++) {
    const uint32_t b = threadIdx.x + i * NT;
    if (b < nb) {
      const bool over = lim.cap && cnt[i] && off[i] + cnt[i] > lim.end(b);
      if (over) atomicOr(err, 2u);
      goff[b] = over ? ~0ull : off[i];
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < W; j++) {
    const uint32_t pos = threadIdx.x + j * NT;
    if (pos < total) {
      const uint32_t d = sbin[pos];
      const unsigned long long go = goff[d];
      if (go == ~0ull) continue;
      const unsigned long long dst = go + (pos - lstart[d]);
      ((uint32_t *)out.w[0])[dst] = stage32[pos];
      if (HB) out.ext[dst] = sext[pos];
    }
  }
}

// ------------------------------------------------------------------------------------------------
// extract: scatter into coarse buckets

// Records the extraction stages at once (scatter_staged CAP; more go out in further rounds): fewer than the tile's
// windows for keys of two or more words, whose tiles count 57-77 % (k = 63..33), 48 % (k = 77) and 33 % (k = 99) of
// their windows on 150-base reads. The LDS saved buys workgroups per CU: two-word 2 -> 3 (extraction k = 63 7.67 ->
// 6.48 ms, k = 33 7.80 -> 7.14; 3072 keeps two: 7.86, 9.13), three-word 3 -> 5 (k = 77 11.54 -> 9.65 ms); four-word
// keys at 256 threads and four waves (kEWaves: 128 VGPRs) fit four workgroups: 10.04 ms, 9.63 with 768 records staged
// (five waves, 96 VGPRs, spill: 15.8 ms; six waves for three-word keys spill: 13.42 ms; 1792 records for two-word keys
// at four waves spill: 12.5 ms)
constexpr int E_CAP[5] = {0, 4096, 2560, 1024, 768};
template <int NL>
__host__ __device__ constexpr int kECap() {
  return E_CAP[NL] < kTile<NL>() ? E_CAP[NL] : kTile<NL>();
}
// Minimum waves per SIMD asked of the compiler for the extraction (caps its VGPRs; 1: no cap)
template <int NL>
constexpr int kEWaves() {
  return NL == 4 ? 4 : 1;
}

template <int NL, bool PACKED, bool CMP, int BPT = 8>
__global__ __launch_bounds__(kEThreads<NL>()) __attribute__((amdgpu_waves_per_eu(kEWaves<NL>()))) void k_extract_scatter(ExtractParams p) {
  constexpr int ET = kEThreads<NL>(), T = kTile<NL>(), W = T / ET;
  const int kk = p.k;
  extern __shared__ __align__(16) unsigned char smem0[];
  uint64_t *fwd;
  uint32_t *good, *start;
  unsigned char *smem = smem0, *area = smem0 + staged_cnt_bytes(p.n_bins);  // counters, then the tile aliased by
  carve_tile<NL>(area, fwd, good, start);                                   // the stage area
  scatter_clear<ET>((uint32_t *)smem, p.n_bins);
  const uint32_t tile = blockIdx.x;
  load_tile<NL>(p.reads, tile, p.tile_starts ? 0u : p.tile_first_read[tile], p.qual_cutoff, fwd, good, start, p.err,
                p.tile_starts);
  const int sh = 64 - p.coarse_bits;
  // stored hash bits, branch-free (hbits == 0: none)
  const int hsh = p.hbits ? 64 - p.hbits : 0;
  const uint64_t hmask = p.hbits ? ~0ull : 0ull;
  const uint32_t sub = p.bin_cap ? blockIdx.x % E_NSUB : 0;
  const BinLimit lim{(uint64_t)sub * p.bin_cap, (uint64_t)E_NSUB * p.bin_cap, p.bin_cap};
  if constexpr (RecKind<NL, CMP>::C32) {
    uint32_t lo[W], hi[W];
    // (the walk with k and the coarse bits as constants for MHM2's default k = 21: constant shifts and masks, measured
    // 1 % faster extraction; any other k takes the general walk)
    if (kk == 21 && p.coarse_bits == 8)
      walk_c32_lh<W, 21, 8>(fwd, good, start, tile, p.reads.n_bases, p.reads.head, kk, p.coarse_bits, lo, hi);
    else
      walk_c32_lh<W>(fwd, good, start, tile, p.reads.n_bases, p.reads.head, kk, p.coarse_bits, lo, hi);
    scatter_staged_c40<W, ET, true, BPT>(lo, hi, p.n_bins, smem, area, p.cursor + sub * p.n_bins, p.out, lim, p.ovf);
    return;
  }
  uint64_t rk[W][NL];
  uint32_t inf[W];
  if constexpr (RecKind<NL, CMP>::M2) {
    // (k as a constant for MHM2's default two-word k = 33, 55 and C4's 63: 2 % faster extraction at 63, the 64-bit
    // shifts by k split into constant 32-bit ones; any other k takes the general walk)
    if (p.coarse_bits == 8 && kk == 63)
      walk_m2<W, 63, 8>(fwd, good, start, tile, p.reads.n_bases, p.reads.head, kk, p.coarse_bits, rk, inf);
    else if (p.coarse_bits == 8 && kk == 55)
      walk_m2<W, 55, 8>(fwd, good, start, tile, p.reads.n_bases, p.reads.head, kk, p.coarse_bits, rk, inf);
    else if (p.coarse_bits == 8 && kk == 33)
      walk_m2<W, 33, 8>(fwd, good, start, tile, p.reads.n_bases, p.reads.head, kk, p.coarse_bits, rk, inf);
    else
      walk_m2<W>(fwd, good, start, tile, p.reads.n_bases, p.reads.head, kk, p.coarse_bits, rk, inf);
  } else {
    auto emit = [&](int i, const uint64_t *key, uint32_t e, bool valid) {
                       if constexpr (RecKind<NL, CMP>::MX) {  // (w0' below the coarse digit) << 6 | ext, r[1..]
                         uint64_t r[NL];
                         mx_mix<NL>(key, r);
                         const int xsh = 64 - p.coarse_bits;
                         rk[i][0] = ((r[0] & ((1ull << xsh) - 1)) << EXT_BITS) | e;
#pragma unroll
                         for (int w = 1; w < NL; w++) rk[i][w] = r[w];
                         inf[i] = valid ? (1u << 31) | (e << 16) | (uint32_t)(r[0] >> xsh) : 0u;
                       } else {  // the key words, the ext code and the stored hash bits packed into the last word
                         const uint64_t h = part_hash<NL>(key);
#pragma unroll
                         for (int w = 0; w < NL; w++) rk[i][w] = key[w];
                         if (PACKED) {
                           rk[i][NL - 1] |= e;
                           rk[i][NL - 1] |= (((h << p.coarse_bits) >> hsh) & hmask) << EXT_BITS;
                         }
                         inf[i] = valid ? (1u << 31) | (e << 16) | (uint32_t)(h >> sh) : 0u;
                       }
                       // materialise the record now: otherwise its inputs (key, e, h) are sunk into the
                       // scatter's conditional store and stay live across its barriers (~7 VGPRs/window)
#pragma unroll
                       for (int w = 0; w < NL; w++) asm volatile("" : "+v"(rk[i][w]));
                       asm volatile("" : "+v"(inf[i]));
                     };
    // (MHM2's default k = 77 and 99 with k as a constant: k = 99 extraction 1.5-3 % faster, k = 77 within noise; any
    // other k takes the general walk)
    if constexpr (RecKind<NL, CMP>::MX && NL == 3) {
      if (kk == 77)
        walk_windows<NL, 77>(fwd, good, start, tile, p.reads.n_bases, p.reads.head, kk, emit);
      else
        walk_windows<NL>(fwd, good, start, tile, p.reads.n_bases, p.reads.head, kk, emit);
    } else if constexpr (RecKind<NL, CMP>::MX && NL == 4) {
      if (kk == 99)
        walk_windows<NL, 99>(fwd, good, start, tile, p.reads.n_bases, p.reads.head, kk, emit);
      else
        walk_windows<NL>(fwd, good, start, tile, p.reads.n_bases, p.reads.head, kk, emit);
    } else {
      walk_windows<NL>(fwd, good, start, tile, p.reads.n_bases, p.reads.head, kk, emit);
    }
  }
  constexpr int SF = RecKind<NL, CMP>::M2 ? SF_AOS2 : SF_WORDS;
  scatter_staged<NL, PACKED, W, SF, ET, kECap<NL>(), BPT>(rk, inf, p.n_bins, smem, area, p.cursor + sub * p.n_bins, 1,
                                                     p.out, lim, p.ovf);
}

// ------------------------------------------------------------------------------------------------
// Supermer exchange (MHMKC_OWNER_MINIMIZER with several ranks and keys of two or more words).
// The reference ships a read's k-mers to their owners as supermers: runs of consecutive windows with the same
// get_kmer_target_rank, each run sent as its bases plus one flanking base on either side
// (SeqBlockInserter::process_seq, src/kcount/kcount_cpu.cpp:73-103 -> add_supermer, kmer_dht.cpp:222-224). Here:
//   k_smer_owner  per extraction tile: the canonical m-mer of every position (rolled along a strip per thread),
//                 the window minimizer as a sliding maximum over k - m + 1 of them (van Herk / Gil-Werman: block
//                 prefix and suffix maxima in LDS), owner = quick_hash(minimizer) % n_ranks for every counted
//                 window (one byte per position to global memory), and per destination the supermers and words
//                 the tile will send (runs are cut at tile edges);
//   k_smer_pack   the same runs again from the owner bytes; each supermer's L = n + k + 1 bases go to its
//                 destination's exact span (cursors from the counts) as whole 32-base words: 2-bit codes (u64,
//                 N -> G, MSB first like the staged tile) + "extension countable" bits (u32), and one u64
//                 descriptor (word offset << 16 | n windows);
//   k_smer_extract on the owner: every window of the received supermers, tile by tile over the window index
//                 (a thread's windows are consecutive, so its supermer is found once and then advanced), the key
//                 read straight from the code words, the record and its coarse bin as k_extract_scatter makes
//                 them, and the same staged scatter (or a bin histogram for the exact layout).
// A window's supermer holds both of its neighbours, so its record equals the one the read gives (interior windows
// of the pseudo-read, kcount_cpu.cpp:316-334).

template <int NL>
__host__ __device__ constexpr int smer_pmax() {  // m-mer positions of a tile: T + k - m + 1 <= T + 32 NL
  return kTile<NL>() + 32 * NL;
}
__host__ __device__ constexpr int smer_words(int n, int k) { return (n + k + 1 + 31) / 32; }

// The supermer starting at tile window i: its window count, 0 when no supermer starts there (not a counted window,
// or the previous window has the same owner). Runs are cut at the tile's last window.
template <int T>
__device__ __forceinline__ int smer_run(const uint8_t *own, int i) {
  const uint8_t d = own[i];
  if (d == 0xFF || (i > 0 && own[i - 1] == d)) return 0;
  int n = 1;
  while (i + n < T && own[i + n] == d) n++;
  return n;
}

template <int NL>
__host__ __device__ constexpr size_t smer_owner_lds(int n_ranks) {
  return tile_lds_bytes<NL>() + 2 * (size_t)smer_pmax<NL>() * 8 + (size_t)kTile<NL>() + (size_t)n_ranks * 8;
}

template <int NL>
__global__ __launch_bounds__(kEThreads<NL>()) void k_smer_owner(SmerParams p) {
  constexpr int ET = kEThreads<NL>(), T = kTile<NL>(), W = T / ET, PMX = smer_pmax<NL>();
  static_assert(T % 16 == 0 && (T + 32 * NL) / ET + 1 <= 32, "one funnel word of incoming bases per strip");
  extern __shared__ __align__(16) unsigned char smem[];
  uint64_t *fwd;
  uint32_t *good, *start;
  unsigned char *rest = carve_tile<NL>(smem, fwd, good, start);
  uint64_t *sm = (uint64_t *)rest, *pmx = sm + PMX;
  uint8_t *own = (uint8_t *)(pmx + PMX);
  uint32_t *dcnt = (uint32_t *)(own + T);  // [2 G]: words, supermers per destination
  const int G = p.n_ranks, k = p.k, m = p.m, w = k - m + 1;
  for (int i = threadIdx.x; i < 2 * G; i += ET) dcnt[i] = 0;
  const uint32_t tile = blockIdx.x;
  load_tile<NL>(p.reads, tile, p.tile_first_read[tile], p.qual_cutoff, fwd, good, start, p.err);
  // 1. canonical m-mer (right-aligned 2m bits, min of forward and reverse complement) of positions 32 + i
  const int pm = T + k - m + 1;
  {
    const int S = (pm + ET - 1) / ET, i0 = (int)threadIdx.x * S, i1 = min(i0 + S, pm);
    if (i0 < i1) {
      const uint64_t mm = (1ull << (2 * m)) - 1;
      const uint64_t x = WalkSpan<NL>::codes64(fwd, 32 + i0);
      uint64_t f = x >> (64 - 2 * m), r = rev2(~x) & mm;
      const uint64_t inc = WalkSpan<NL>::codes64(fwd, 32 + i0 + m);  // the base entering after position i0 + t
      for (int i = i0; i < i1; i++) {
        sm[i] = f < r ? f : r;
        const uint32_t c = (uint32_t)(inc >> (62 - 2 * (i - i0))) & 3u;
        f = ((f << 2) | c) & mm;
        r = (r >> 2) | ((uint64_t)(3u - c) << (2 * m - 2));
      }
    }
  }
  __syncthreads();
  // 2. blocks of w positions: prefix maxima into pmx, suffix maxima in place; the minimizer of the window at
  //    32 + i (its m-mers i .. i + w - 1) is max(sm[i], pmx[i + w - 1])
  for (int b = threadIdx.x; b * w < pm; b += ET) {
    const int lo = b * w, hi = min(lo + w, pm);
    uint64_t v = 0;
    for (int i = lo; i < hi; i++) {
      v = sm[i] > v ? sm[i] : v;
      pmx[i] = v;
    }
    v = 0;
    for (int i = hi - 1; i >= lo; i--) {
      v = sm[i] > v ? sm[i] : v;
      sm[i] = v;
    }
  }
  __syncthreads();
  // 3. the owner of every counted window, get_kmer_target_rank = minimizer_hash_fast % rank_n
  //    (kmer_dht.cpp:193-196; quick_hash of the minimizer left-aligned, src/kmer.cpp:454-463)
  {
    WalkSpan<NL> sp(fwd, good, start, tile, p.reads.n_bases, p.reads.head, k);
    uint64_t last_min = ~0ull;
    uint32_t last_own = 0;
#pragma unroll
    for (int j = 0; j < W; j++) {
      uint32_t cr, ef, er;
      const bool valid = sp.step(j, k, cr, ef, er);
      const int i = (int)threadIdx.x * W + j;
      const uint64_t a = sm[i], b2 = pmx[i + w - 1];
      const uint64_t mn = a > b2 ? a : b2;
      if (valid && mn != last_min) {
        last_min = mn;
        last_own = (uint32_t)(quick_hash(mn << (64 - 2 * m)) % (uint64_t)G);
      }
      own[i] = valid ? (uint8_t)last_own : (uint8_t)0xFF;
    }
  }
  __syncthreads();
  // 4. the supermers of the tile and what they will send, per destination
#pragma unroll
  for (int j = 0; j < W; j++) {
    const int i = (int)threadIdx.x * W + j;
    const int n = smer_run<T>(own, i);
    if (n) {
      const uint32_t d = own[i];
      atomicAdd(&dcnt[2 * d], (uint32_t)smer_words(n, k));
      atomicAdd(&dcnt[2 * d + 1], 1u);
    }
  }
  uint32_t *gown = (uint32_t *)(p.owners + (uint64_t)tile * T);
  for (int i = threadIdx.x; i < T / 4; i += ET) gown[i] = ((const uint32_t *)own)[i];
  __syncthreads();
  // counters per (destination, slice): consecutive tiles add to different words (with a handful of ranks one word
  // per destination took every workgroup's atomics: 16 ms for 2M reads)
  unsigned long long *h = p.hist + 2 * (uint64_t)(blockIdx.x % SMER_SLICES);
  for (int d = threadIdx.x; d < G; d += ET) {
    if (dcnt[2 * d + 1]) {
      atomicAdd(&h[2 * SMER_SLICES * d], (unsigned long long)dcnt[2 * d]);
      atomicAdd(&h[2 * SMER_SLICES * d + 1], (unsigned long long)dcnt[2 * d + 1]);
    }
  }
}

template <int NL>
__host__ __device__ constexpr size_t smer_pack_lds(int n_ranks) {
  return tile_lds_bytes<NL>() + (size_t)kTile<NL>() + (size_t)n_ranks * 8 + (size_t)n_ranks * 16;
}

template <int NL>
__global__ __launch_bounds__(kEThreads<NL>()) void k_smer_pack(SmerParams p) {
  constexpr int ET = kEThreads<NL>(), T = kTile<NL>(), W = T / ET, NG = kGroups<NL>();
  extern __shared__ __align__(16) unsigned char smem[];
  uint64_t *fwd;
  uint32_t *good, *start;
  unsigned char *rest = carve_tile<NL>(smem, fwd, good, start);
  uint8_t *own = rest;
  uint32_t *dcnt = (uint32_t *)(own + T);                                       // [2 G]
  unsigned long long *goff = (unsigned long long *)(dcnt + 2 * p.n_ranks);  // [2 G] (8-byte aligned: dcnt is 16)
  const int G = p.n_ranks, k = p.k;
  for (int i = threadIdx.x; i < 2 * G; i += ET) dcnt[i] = 0;
  const uint32_t tile = blockIdx.x;
  load_tile<NL>(p.reads, tile, p.tile_first_read[tile], p.qual_cutoff, fwd, good, start, p.err);
  const uint32_t *gown = (const uint32_t *)(p.owners + (uint64_t)tile * T);
  for (int i = threadIdx.x; i < T / 4; i += ET) ((uint32_t *)own)[i] = gown[i];
  __syncthreads();
  uint32_t wr[W], sr[W];
#pragma unroll
  for (int j = 0; j < W; j++) {
    const int i = (int)threadIdx.x * W + j;
    const int n = smer_run<T>(own, i);
    wr[j] = sr[j] = 0;
    if (n) {
      const uint32_t d = own[i];
      wr[j] = atomicAdd(&dcnt[2 * d], (uint32_t)smer_words(n, k));
      sr[j] = atomicAdd(&dcnt[2 * d + 1], 1u);
    }
  }
  __syncthreads();
  unsigned long long *cur = p.cursor + 2 * (uint64_t)(blockIdx.x % SMER_SLICES);  // this tile's slice (k_smer_owner)
  for (int d = threadIdx.x; d < G; d += ET) {
    const uint32_t nw = dcnt[2 * d], ns = dcnt[2 * d + 1];
    goff[2 * d] = ns ? atomicAdd(&cur[2 * SMER_SLICES * d], (unsigned long long)nw) : 0ull;
    goff[2 * d + 1] = ns ? atomicAdd(&cur[2 * SMER_SLICES * d + 1], (unsigned long long)ns) : 0ull;
  }
  __syncthreads();
  // the staged words past the tile read as zero (they only fill masked bits of a supermer's last word)
  auto code_at = [&](int g) { return g < NG ? fwd[g] : 0ull; };
  auto good_at = [&](int g) { return g < NG ? good[g] : 0u; };
#pragma unroll
  for (int j = 0; j < W; j++) {
    const int i = (int)threadIdx.x * W + j;
    const int n = smer_run<T>(own, i);
    if (!n) continue;
    const uint32_t d = own[i];
    const unsigned long long wo = goff[2 * d] + wr[j], so = goff[2 * d + 1] + sr[j];
    if (so >= p.n_smer || wo + smer_words(n, k) > p.n_words) {  // (counts of the two passes disagree: a bug)
      atomicOr(p.err, 8u);
      continue;
    }
    p.desc[so] = ((uint64_t)wo << 16) | (uint64_t)n;
    const int L = n + k + 1, q0 = 32 + i - 1;  // bases: the left flank, the n windows' bases, the right flank
    for (int g = 0; g < smer_words(n, k); g++) {
      const int q = q0 + 32 * g, gi = q >> 5, sh = q & 31;
      uint64_t cw = code_at(gi);
      uint32_t gw = good_at(gi);
      if (sh) {
        cw = (cw << (2 * sh)) | (code_at(gi + 1) >> (64 - 2 * sh));
        gw = (gw << sh) | (good_at(gi + 1) >> (32 - sh));
      }
      const int rem = L - 32 * g;
      if (rem < 32) {
        cw &= top_mask(rem);
        gw &= ~(~0u >> rem);
      }
      p.codes[wo + g] = cw;
      p.good[wo + g] = gw;
    }
  }
}

// The record of one window and its coarse bin, as k_extract_scatter's emit makes them (mixed two-word records,
// or the key words + packed ext code / stored hash bits).
template <int NL, bool PACKED, bool CMP>
__device__ __forceinline__ void window_record(const uint64_t *key, uint32_t e, bool valid, const ExtractParams &p,
                                              uint64_t (&rk)[NL], uint32_t &inf) {
  const int kk = p.k;
  if constexpr (RecKind<NL, CMP>::M2) {
    const int m2_csh = kk - p.coarse_bits;
    uint64_t L, R;
    m2_mix(key, kk, L, R);
    rk[0] = ((L & ((1ull << m2_csh) - 1)) << EXT_BITS) | e;
    rk[1] = R;
    inf = valid ? (1u << 31) | (e << 16) | (uint32_t)(L >> m2_csh) : 0u;
    return;
  }
  if constexpr (RecKind<NL, CMP>::MX) {
    const int xsh = 64 - p.coarse_bits;
    uint64_t r[NL];
    mx_mix<NL>(key, r);
    rk[0] = ((r[0] & ((1ull << xsh) - 1)) << EXT_BITS) | e;
#pragma unroll
    for (int w = 1; w < NL; w++) rk[w] = r[w];
    inf = valid ? (1u << 31) | (e << 16) | (uint32_t)(r[0] >> xsh) : 0u;
    return;
  }
  const uint64_t h = window_hash<NL, CMP>(key, kk);
#pragma unroll
  for (int w = 0; w < NL; w++) rk[w] = key[w];
  if (PACKED) {
    const int hsh = p.hbits ? 64 - p.hbits : 0;
    const uint64_t hmask = p.hbits ? ~0ull : 0ull;
    rk[NL - 1] |= e;
    rk[NL - 1] |= (((h << p.coarse_bits) >> hsh) & hmask) << EXT_BITS;
  }
  inf = valid ? (1u << 31) | (e << 16) | (uint32_t)(h >> (64 - p.coarse_bits)) : 0u;
}

// 32 codes from base q of a supermer code stream, first on top
__device__ __forceinline__ uint64_t smer_codes64(const uint64_t *c, uint64_t q) {
  const uint64_t g = q >> 5;
  const int sh = (int)(q & 31) * 2;
  return (gload(c + g) << sh) | ((gload(c + g + 1) >> 1) >> (63 - sh));
}

template <int NL, bool PACKED, bool CMP, bool HIST>
__global__ __launch_bounds__(kEThreads<NL>()) void k_smer_extract(ExtractParams p, SmerSource src) {
  constexpr int ET = kEThreads<NL>(), T = kTile<NL>(), W = T / ET;  // T windows per tile, W per thread
  extern __shared__ __align__(16) unsigned char smem[];
  const int k = p.k;
  const uint32_t tile = blockIdx.x;
  if (HIST)
    for (uint32_t b = threadIdx.x; b < p.n_bins; b += ET) ((uint32_t *)smem)[b] = 0;
  else
    scatter_clear<ET>((uint32_t *)smem, p.n_bins);
  const uint64_t J0 = (uint64_t)tile * T + (uint64_t)threadIdx.x * W;
  // the supermer holding window J0: the last s with wpre[s] <= J0, among the tile's supermers
  uint64_t s = src.tile_first[tile];
  {
    uint64_t hi = src.tile_first[tile + 1] + 1;
    if (hi > src.n_smer) hi = src.n_smer;
    while (hi - s > 1) {
      const uint64_t mid = (s + hi) >> 1;
      if (gload(src.wpre + mid) <= J0)
        s = mid;
      else
        hi = mid;
    }
  }
  uint64_t ws = gload(src.wpre + s), we = gload(src.wpre + s + 1), dsc = gload(src.desc + s);
  const uint64_t tmask = top_mask(k - 32 * (NL - 1));
  uint64_t rk[W][NL];
  uint32_t inf[W];
#pragma unroll
  for (int j = 0; j < W; j++) {
    const uint64_t J = J0 + (uint64_t)j;
    const bool valid = J < src.n_windows;
    if (valid)
      while (J >= we) {
        s++;
        ws = we;
        we = gload(src.wpre + s + 1);
        dsc = gload(src.desc + s);
      }
    // base of the window in the stream: its supermer's first word, the left flank, the window's offset
    uint64_t P = valid ? 32 * (dsc >> 16) + 1 + (J - ws) : 32;
    if ((P >> 5) + NL + 2 > src.n_words) {  // a descriptor past the stream (a bug): flag it, read nothing there
      if (valid) atomicOr(p.err, 8u);
      P = 32;
    }
    uint64_t fw[NL], rc[NL];
#pragma unroll
    for (int w = 0; w < NL; w++) fw[w] = smer_codes64(src.codes, P + 32 * (uint64_t)w);
    fw[NL - 1] &= tmask;
    const uint64_t ql = P - 1, qr = P + (uint64_t)k;
    const uint32_t cl = (uint32_t)(gload(src.codes + (ql >> 5)) >> (62 - 2 * (ql & 31))) & 3u;
    const uint32_t cr = (uint32_t)(gload(src.codes + (qr >> 5)) >> (62 - 2 * (qr & 31))) & 3u;
    const uint32_t gl = (gload(src.good + (ql >> 5)) >> (31 - (ql & 31))) & 1u;
    const uint32_t gr = (gload(src.good + (qr >> 5)) >> (31 - (qr & 31))) & 1u;
    revcomp<NL>(fw, rc, k);
    const bool use_rc = kmer_less<NL>(rc, fw);
    uint64_t key[NL];
#pragma unroll
    for (int w = 0; w < NL; w++) key[w] = use_rc ? rc[w] : fw[w];
    uint32_t l = gl ? cl : (uint32_t)EXT_NONE, r = gr ? cr : (uint32_t)EXT_NONE;
    if (use_rc) {
      const uint32_t nl_ = gr ? 3u - cr : (uint32_t)EXT_NONE, nr_ = gl ? 3u - cl : (uint32_t)EXT_NONE;
      l = nl_;
      r = nr_;
    }
    window_record<NL, PACKED, CMP>(key, (l << 3) | r, valid, p, rk[j], inf[j]);
    if (p.bin_hi && ((inf[j] & 0xffffu) < p.bin_lo || (inf[j] & 0xffffu) >= p.bin_hi)) inf[j] = 0u;  // other pass
#pragma unroll
    for (int w = 0; w < NL; w++) asm volatile("" : "+v"(rk[j][w]));
    asm volatile("" : "+v"(inf[j]));
  }
  if constexpr (HIST) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < W; j++)
      if (inf[j] >> 31) atomicAdd(&((uint32_t *)smem)[inf[j] & 0xffffu], 1u);
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < p.n_bins; b += ET) {
      const uint32_t c = ((uint32_t *)smem)[b];
      if (c) atomicAdd(&p.hist[b], (unsigned long long)c);
    }
  } else {
    __syncthreads();
    const uint32_t sub = p.bin_cap ? blockIdx.x % E_NSUB : 0;
    const BinLimit lim{(uint64_t)sub * p.bin_cap, (uint64_t)E_NSUB * p.bin_cap, p.bin_cap};
    constexpr int SF = RecKind<NL, CMP>::M2 ? SF_AOS2 : SF_WORDS;
    scatter_staged<NL, PACKED, W, SF, ET>(rk, inf, p.n_bins, smem, smem + staged_cnt_bytes(p.n_bins),
                                          p.cursor + sub * p.n_bins, 1, p.out, lim, p.ovf);
  }
}

// Descriptors of one received span: word offsets moved by delta (mod 2^64: the span's place in the concatenated
// stream minus its place in the sender's planes), window counts for the scan.
__global__ __launch_bounds__(256) void k_smer_rebase(uint64_t *desc, uint64_t n, uint64_t delta,
                                                     unsigned long long *nwin) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t d = desc[i] + (delta << 16);
    desc[i] = d;
    nwin[i] = d & 0xffffu;
  }
}

// Per window tile t (T windows): the supermer holding its first window (the last s with wpre[s] <= t T);
// tile_first[n_tiles] = n_smer - 1.
__global__ __launch_bounds__(256) void k_smer_tiles(const uint64_t *wpre, uint64_t n_smer, uint64_t *tile_first,
                                                    uint32_t n_tiles, int T) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t > n_tiles) return;
  if (t == n_tiles) {
    tile_first[t] = n_smer - 1;
    return;
  }
  const uint64_t J = (uint64_t)t * (uint64_t)T;
  uint64_t lo = 0, hi = n_smer;  // wpre[0] = 0 <= J
  while (hi - lo > 1) {
    const uint64_t mid = (lo + hi) >> 1;
    if (wpre[mid] <= J)
      lo = mid;
    else
      hi = mid;
  }
  tile_first[t] = lo;
}

// ------------------------------------------------------------------------------------------------
// partition coarse -> fine

// Fine digit of a record: from the hash bits stored next to the ext code when there are enough of them,
// otherwise by recomputing MurmurHash3 of the key. rk holds the raw record words.
template <int NL, bool PACKED, bool CMP>
__device__ __forceinline__ uint32_t fine_digit(const uint64_t *rk, const PartitionParams &p) {
  const uint64_t fmask = (1ull << p.fine_bits) - 1;
  if (CMP && NL == 1) return (uint32_t)((rk[0] >> (EXT_BITS + 2 * p.k - p.coarse_bits - p.fine_bits)) & fmask);
  if (CMP && NL == 2) return (uint32_t)((rk[0] >> (EXT_BITS + p.k - p.coarse_bits - p.fine_bits)) & fmask);
  if (CMP && NL >= 3) return (uint32_t)((rk[0] >> (EXT_BITS + 64 - p.coarse_bits - p.fine_bits)) & fmask);
  if (PACKED && p.hbits >= p.fine_bits) {
    const uint64_t stored = (rk[NL - 1] >> EXT_BITS) & ((1ull << p.hbits) - 1);
    return (uint32_t)((stored >> (p.hbits - p.fine_bits)) & fmask);
  }
  uint64_t key[NL];
#pragma unroll
  for (int w = 0; w < NL; w++) key[w] = rk[w];
  if (PACKED) key[NL - 1] &= ~((1ull << (EXT_BITS + p.hbits)) - 1);
  return (uint32_t)((part_hash<NL>(key) >> (64 - p.coarse_bits - p.fine_bits)) & fmask);
}

// Chunk of this workgroup: workgroups are dealt to the XCDs round-robin, so workgroup b runs on XCD b % 8
// and takes the (b / 8)-th chunk of XCD class b % 8. All chunks of a coarse bucket then write their fine
// buckets from one XCD, whose L2 merges the partial lines of consecutive chunks before they reach HBM.
__device__ __forceinline__ bool xcd_chunk(const PartitionParams &p, uint32_t &c) {
  const uint32_t x = blockIdx.x & 7u;
  c = p.xcd_start[x] + (blockIdx.x >> 3);
  return c < p.xcd_start[x + 1];
}

// The chunk a partition workgroup works on: one 24-byte load of the span k_chunk_runs expanded (the run index and
// then the run cost two dependent global round trips before the chunk's records could be loaded).
template <int T>
__device__ __forceinline__ SChunk chunk_of(const PartitionParams &p, uint32_t c) {
  return p.chunks[c];
}

// Every run's chunks (one workgroup per run): chunk i of a run is records [i T, min((i + 1) T, count)) of it.
__global__ __launch_bounds__(256) void k_chunk_runs(const SRun *runs, SChunk *chunks, int tile) {
  const SRun r = runs[blockIdx.x];
  const uint32_t n = (uint32_t)((r.count + tile - 1) / tile);
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
    const uint64_t o = (uint64_t)i * tile;
    SChunk ch;
    ch.start = r.start + o;
    ch.count = (uint32_t)(r.count - o < (uint64_t)tile ? r.count - o : (uint64_t)tile);
    ch.src = r.src;
    ch.coarse_local = r.coarse_local;
    ch.pad = 0;
    chunks[r.chunk0 + i] = ch;
  }
}

// All W records of a thread are loaded before any is processed (W * 8 B * NL in flight per lane). The
// loads are unconditional (lanes past the chunk end re-read its last record) so that no use of a loaded
// value sits inside a branch: a conditional load whose value is consumed in its own branch makes the
// compiler wait for it there, one load after the other. Callers check i < ch.count themselves.
template <int NL, bool PACKED, bool CMP, int W, int NT = kPThreads<NL>()>
__device__ __forceinline__ void load_chunk(const PlaneSet &src, const SChunk &ch, uint64_t (&rk)[W][NL],
                                           uint32_t (&re)[W]) {
  uint32_t rx[W];
#pragma unroll
  for (int j = 0; j < W; j++) {
    const uint32_t i = threadIdx.x + j * NT;
    const uint64_t idx = ch.start + (i < ch.count ? i : ch.count - 1);
    if (RecKind<NL, CMP>::C32) {  // coarse compact record: low 32 bits + high byte
      rk[j][0] = (uint64_t)gload((const uint32_t *)src.w[0] + idx);
      rx[j] = (uint32_t)gload(src.ext + idx);
      continue;
    }
    if (RecKind<NL, CMP>::M2) {  // one 16-byte record
      const u32x4 v = gload4((const uint32_t *)src.w[0] + 4 * idx);
      rk[j][0] = (uint64_t)v.x | ((uint64_t)v.y << 32);
      rk[j][NL - 1] = (uint64_t)v.z | ((uint64_t)v.w << 32);
      rx[j] = 0u;
      continue;
    }
#pragma unroll
    for (int w = 0; w < NL; w++) rk[j][w] = gload(src.w[w] + idx);
    rx[j] = PACKED ? 0u : (uint32_t)gload(src.ext + idx);
  }
  if (RecKind<NL, CMP>::C32) {
#pragma unroll
    for (int j = 0; j < W; j++) rk[j][0] |= (uint64_t)rx[j] << 32;
  }
#pragma unroll
  for (int j = 0; j < W; j++) re[j] = PACKED ? (uint32_t)(rk[j][RecKind<NL, CMP>::XW] & 63u) : rx[j];
}

template <int NL, bool PACKED, bool CMP>
__global__ __launch_bounds__(kPThreads<NL>()) void k_part_hist(PartitionParams p) {
  constexpr int NT = kPThreads<NL>(), T = kPTile<NL>(), W = T / NT;
  extern __shared__ __align__(16) uint32_t hist[];  // the only LDS object
  const uint32_t nf = 1u << p.fine_bits;
  for (uint32_t b = threadIdx.x; b < nf; b += NT) hist[b] = 0;
  uint32_t c;
  if (!xcd_chunk(p, c)) return;  // no chunk left in this workgroup's XCD class (uniform: before any barrier)
  const SChunk ch = chunk_of<T>(p, c);
  const PlaneSet src = p.srcs[ch.src];
  uint64_t rk[W][NL];
  uint32_t re[W];
  load_chunk<NL, PACKED, CMP, W>(src, ch, rk, re);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < W; j++) {
    if (threadIdx.x + j * NT < ch.count) atomicAdd(&hist[fine_digit<NL, PACKED, CMP>(rk[j], p)], 1u);
  }
  __syncthreads();
  unsigned long long *g = p.fine_hist + (uint64_t)ch.coarse_local * nf;
  for (uint32_t b = threadIdx.x; b < nf; b += NT) {
    const uint32_t c = hist[b];
    if (c) atomicAdd(&g[b], (unsigned long long)c);
  }
}

template <int NL, bool PACKED, bool CMP, int BPT = 8>
__global__ __launch_bounds__(kPThreads<NL>()) void k_part_scatter(PartitionParams p) {
  constexpr int NT = kPThreads<NL>(), T = kPTile<NL>(), W = T / NT;
  static_assert(T % NT == 0 && NT % 64 == 0, "whole records per thread, whole waves");
  extern __shared__ __align__(16) unsigned char smem[];
  const uint32_t nf = 1u << p.fine_bits;
  scatter_clear<NT>((uint32_t *)smem, nf);
  uint32_t c;
  if (!xcd_chunk(p, c)) return;  // no chunk left in this workgroup's XCD class (uniform: before any barrier)
  const SChunk ch = chunk_of<T>(p, c);
  const PlaneSet src = p.srcs[ch.src];
  if constexpr (RecKind<NL, CMP>::C32) {
    // Compact records as lo / hi registers (the extraction's scatter_staged_c40 with u32 records), loaded from the
    // chunk's planes through 32-bit offsets from its (uniform) start: 32 VGPRs of records instead of 64, and no
    // 64-bit address per load
    const uint32_t *b32 = (const uint32_t *)src.w[0] + ch.start;
    const uint8_t *b8 = src.ext + ch.start;
    uint32_t lo[W], hi[W];
#pragma unroll
    for (int j = 0; j < W; j++) {
      const uint32_t i = min((uint32_t)(threadIdx.x + j * NT), ch.count - 1u);
      lo[j] = gload(b32 + i);
      hi[j] = gload(b8 + i);
    }
    const uint64_t cmask = (1ull << (EXT_BITS + 2 * p.k - p.coarse_bits - p.fine_bits)) - 1;
#pragma unroll
    for (int j = 0; j < W; j++) {
      uint64_t r[1] = {(uint64_t)lo[j] | ((uint64_t)hi[j] << 32)};
      hi[j] = (threadIdx.x + j * NT < ch.count) ? (1u << 31) | fine_digit<NL, PACKED, CMP>(r, p) : 0u;
      lo[j] = (uint32_t)(r[0] & cmask);
    }
    BinLimit lim{0, 0, 0};
    if (p.coarse_fcap) {
      const uint64_t fc = p.coarse_fcap[ch.coarse_local];
      lim = BinLimit{p.coarse_base[ch.coarse_local], fc, fc};
    }
    __syncthreads();
    scatter_staged_c40<W, NT, false, BPT>(lo, hi, nf, smem, smem + staged_cnt_bytes(nf),
                                     p.fine_cursor + (uint64_t)ch.coarse_local * nf, p.out, lim, p.err);
    return;
  }
  uint64_t rk[W][NL];
  uint32_t re[W], inf[W];
  load_chunk<NL, PACKED, CMP, W>(src, ch, rk, re);
  // compact: the fine record keeps the bits below the fine digit (+ the ext code), <= 32 bits; mixed
  // two-word: w[0] keeps L' below the fine digit (+ the ext code)
  const uint64_t cmask =
      (1ull << (EXT_BITS + (NL == 1 ? 2 * p.k : RecKind<NL, CMP>::lw(p.k)) - p.coarse_bits - p.fine_bits)) - 1;
#pragma unroll
  for (int j = 0; j < W; j++) {
    inf[j] = (threadIdx.x + j * NT < ch.count)
                 ? ((1u << 31) | (re[j] << 16) | fine_digit<NL, PACKED, CMP>(rk[j], p))
                 : 0u;
    if (CMP) rk[j][0] &= cmask;
  }
  __syncthreads();
  BinLimit lim{0, 0, 0};
  if (p.coarse_fcap) {
    const uint64_t fc = p.coarse_fcap[ch.coarse_local];
    lim = BinLimit{p.coarse_base[ch.coarse_local], fc, fc};
  }
  unsigned long long *cur = p.fine_cursor + (uint64_t)ch.coarse_local * nf;
  constexpr int SF = RecKind<NL, CMP>::M2 ? SF_AOS2 : SF_WORDS;
  scatter_staged<NL, PACKED, W, SF, NT, W * NT, BPT>(rk, inf, nf, smem, smem + staged_cnt_bytes(nf), cur, 1, p.out, lim, p.err);
}

// Distinct-key sketch (HyperLogLog, SKETCH_M registers) over the records of one coarse bucket, from which
// the host sizes the fine partition (distinct keys per fine bucket vs the LDS table capacity). The key of
// a record is its words without the ext code and stored hash bits (compact: the stored bits, unique within
// the coarse bucket); the sketch hash is an fmix64 chain, independent of the partition hash.
// It also counts the extension adds of these records (the LDS op mix of k_count, reported in the stats as
// a sample of the whole).
template <int NL, bool PACKED, bool CMP>
__global__ __launch_bounds__(kPThreads<NL>()) void k_sketch(PartitionParams p, unsigned int *hll, unsigned int *fhist) {
  constexpr int NT = kPThreads<NL>(), T = kPTile<NL>(), W = T / NT;
  __shared__ unsigned int reg[SKETCH_M];
  __shared__ unsigned int fh[SKETCH_FH];
  __shared__ unsigned int s_ext;
  if (threadIdx.x == 0) s_ext = 0;
  for (int i = threadIdx.x; i < SKETCH_M; i += NT) reg[i] = 0;
  if (fhist)
    for (int i = threadIdx.x; i < SKETCH_FH; i += NT) fh[i] = 0;
  const SChunk ch = chunk_of<T>(p, blockIdx.x);
  const PlaneSet src = p.srcs[ch.src];
  uint64_t rk[W][NL];
  uint32_t re[W];
  load_chunk<NL, PACKED, CMP, W>(src, ch, rk, re);
  __syncthreads();
  const uint64_t low_mask = CMP ? 63ull : PACKED ? (1ull << (EXT_BITS + p.hbits)) - 1 : 0ull;
  uint32_t ext_adds = 0;
#pragma unroll
  for (int j = 0; j < W; j++) {
    if (threadIdx.x + j * NT >= ch.count) continue;
    ext_adds += (uint32_t)(((re[j] >> 3) & 7u) < 4u) + (uint32_t)((re[j] & 7u) < 4u);
    uint64_t h = 0x9E3779B97F4A7C15ull;
#pragma unroll
    for (int w = 0; w < NL; w++) h = fmix64(h ^ (w == RecKind<NL, CMP>::XW ? rk[j][w] & ~low_mask : rk[j][w]));
    const uint32_t rho = (uint32_t)__clzll(h | (uint64_t)(SKETCH_M - 1)) + 1;  // first 1 among the top bits
    atomicMax(&reg[h & (SKETCH_M - 1)], rho);
    if (fhist) atomicAdd(&fh[fine_digit<NL, PACKED, CMP>(rk[j], p)], 1u);
  }
  atomicAdd(&s_ext, ext_adds);
  __syncthreads();
  if (fhist)
    for (int i = threadIdx.x; i < SKETCH_FH; i += NT)
      if (fh[i]) atomicAdd(&fhist[i], fh[i]);
  for (int i = threadIdx.x; i < SKETCH_M; i += NT)
    if (reg[i]) {
      atomicMax(&hll[i], reg[i]);
      if (!(blockIdx.x & 1u)) atomicMax(&hll[SKETCH_M + 1 + i], reg[i]);  // the even chunks' sketch (about half)
    }
  if (threadIdx.x == 0 && s_ext) atomicAdd(&hll[SKETCH_M], s_ext);  // (one add per workgroup)
}

// capped fine layout
__global__ void k_init_fine(const unsigned long long *coarse_base, const unsigned long long *coarse_fcap, uint32_t n_coarse,
                            int fine_bits, unsigned long long *base, unsigned long long *cursor) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ((uint64_t)n_coarse << fine_bits)) return;
  const uint64_t c = i >> fine_bits, d = i & ((1ull << fine_bits) - 1);
  const unsigned long long b = coarse_base[c] + d * coarse_fcap[c];
  base[i] = b;
  cursor[i] = b;
}

// sum over reads of max(0, L - k - 1): the counted windows of a batch
// and the CSR checks of mhmkc_add_reads (offsets non-decreasing, reads <= 65535 bases: PackedRead's
// read_len is a uint16, src/packed_reads.hpp:60-80) for device-resident offsets
// (4 reads per lane per iteration, their loads issued together, and one global atomic per workgroup: the first
// version's two dependent loads per read took 0.11 ms at C2, and one atomic per wave over a 64k-workgroup grid 1.9 ms)
__global__ __launch_bounds__(256) void k_count_windows(ReadsView rv, int k, unsigned long long *out, unsigned int *err) {
  __shared__ unsigned long long s_acc[4];
  unsigned long long acc = 0;
  bool bad = false;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t r0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r0 < rv.n_reads; r0 += 4 * stride) {
    uint64_t a[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const uint64_t r = r0 + u * stride, rr = r < rv.n_reads ? r : rv.n_reads - 1;
      a[u] = rv.offs[rr];
      b[u] = rv.offs[rr + 1];
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      if (r0 + u * stride >= rv.n_reads) break;
      bad |= b[u] < a[u] || b[u] - a[u] > 65535;
      const uint64_t L = b[u] - a[u];
      acc += (b[u] >= a[u] && L > (uint64_t)k + 1) ? L - k - 1 : 0;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0)
    bad |= rv.offs[0] != rv.obase + rv.head || rv.offs[rv.n_reads] - rv.obase != rv.n_bases;
  if (bad) atomicOr(err, 4u);
  acc = wave_sum_u64(acc);
  if ((threadIdx.x & 63) == 0) s_acc[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long t = s_acc[0] + s_acc[1] + s_acc[2] + s_acc[3];
    if (t) atomicAdd(out, t);
  }
}

// The bases of one H2D chunk of a host batch, sent as nibbles (mhmkc_host.cpp nib_pack: code | (q >= qcut) << 3, two
// per byte, the first in the low half), written back into the arena as PackedRead bytes code | (q >= qcut ? 31 : 0) << 3:
// load_tile's only use of the quality is q >= qcut, which these bytes answer as the originals do for every qcut.
// Thread t writes the arena's 16-byte block t of [b0 & ~15, b0 + n) (bytes of that range outside [b0, b0 + n) belong to
// the neighbouring chunks and are left alone).
__global__ __launch_bounds__(256) void k_expand_nibbles(const uint8_t *nib, uint8_t *arena, uint64_t b0, uint64_t n) {
  const uint64_t a0 = b0 & ~15ull, end = b0 + n;
  const uint64_t p0 = a0 + ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16;
  if (p0 >= end) return;
  uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const uint64_t p = p0 + i;
    if (p >= b0 && p < end) {
      const uint64_t j = p - b0;
      const uint32_t v = (nib[j >> 1] >> (4 * (uint32_t)(j & 1))) & 15u;
      w[i >> 2] |= ((v & 7u) | ((v >> 3) * 0xf8u)) << (8 * (i & 3));
    }
  }
  if (p0 >= b0 && p0 + 16 <= end) {
    *(uint4 *)(arena + p0) = make_uint4(w[0], w[1], w[2], w[3]);
    return;
  }
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const uint64_t p = p0 + i;
    if (p >= b0 && p < end) arena[p] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
  }
}

// The chunk's offsets from the u32 distances to its first byte that the nibble H2D sends.
__global__ __launch_bounds__(256) void k_offs_from_deltas(const uint32_t *d, uint64_t *offs, uint64_t n, uint64_t b0) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) offs[i] = b0 + d[i];
}

__global__ __launch_bounds__(1024) void k_scan(const unsigned long long *in, unsigned long long *base,
                                               unsigned long long *cursor, uint32_t n) {
  __shared__ unsigned long long wsum[17];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const uint32_t per = (n + 1023) / 1024;
  const uint32_t lo = min((uint32_t)tid * per, n), hi = min(lo + per, n);
  // bucket bases are kept multiples of 4 records (k_count's compact rounds load 4 records per lane)
  unsigned long long s = 0;
  for (uint32_t i = lo; i < hi; i++) s += (in[i] + 3) & ~3ull;
  unsigned long long x = s;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    unsigned long long y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  if (tid == 0) {
    unsigned long long acc = 0;
    for (int w = 0; w < 16; w++) {
      unsigned long long t = wsum[w];
      wsum[w] = acc;
      acc += t;
    }
  }
  __syncthreads();
  unsigned long long run = wsum[wid] + x - s;
  for (uint32_t i = lo; i < hi; i++) {
    base[i] = run;
    cursor[i] = run;
    run += (in[i] + 3) & ~3ull;
  }
}

// ------------------------------------------------------------------------------------------------
// count: LDS open-addressing hash table per fine bucket

// Records per thread per round of k_count (register budget: 1024 threads -> <= 128 VGPRs): compact keys 4 (one
// 16-byte load of four records per lane); two-, three- and four-word keys 1 (round 4: fewer records in flight lose
// fewer claims to each other, phase-B records at k = 63 100M -> 71M; count k = 63 8.92 -> 8.81 ms, k = 33 8.56 ->
// 8.19 ms, k = 77 10.49 -> 10.25 ms, k = 99 11.02 -> 10.06 ms)
template <int NL>
constexpr int count_rpt() {
  return NL == 1 ? 4 : 1;
}

// LDS slot hash of k_count. All keys of a fine bucket share their top MurmurHash3 bits, so the slot
// uses an independent multiplicative mix of the key words (performance only; any function is correct).
template <int NL>
__device__ __forceinline__ uint32_t slot_hash(const uint64_t *key) {
  if (NL == 1) {  // 32-bit mix of the two halves (two quarter-rate multiplies instead of a 64-bit product)
    const uint32_t x = (uint32_t)(key[0] >> 32) * 0x9E3779B1u + (uint32_t)key[0] * 0x85EBCA77u;
    return x ^ (x >> 15);
  }
  uint64_t h = key[0] * 0x9E3779B97F4A7C15ull;
#pragma unroll
  for (int w = 1; w < NL; w++) h = (h ^ (h >> 31) ^ key[w]) * 0xC2B2AE3D27D4EB4Full;
  h ^= h >> 29;
  return (uint32_t)(h >> 32);
}

// Home group of a compact key. The stored bits of a compact record are bits of the bijectively mixed k-mer
// (kmer_ops.hpp cmix) below the bucket digits, already uniform: the group is their top 16 bits scaled to the
// group count with one full-rate 24-bit multiply (the generic slot_hash + fastrange cost three quarter-rate
// multiplies, in a kernel whose VALU issue is its limit). kshl = 26 - stored bits: the key word holds them in
// bits [6, 32 - kshl).
__device__ __forceinline__ int cmp_group(uint32_t key, int kshl, uint32_t ng) {
  return (int)(__umul24((key << kshl) >> 16, ng) >> 16);
}

template <typename K>  // key word type: uint64_t, or uint32_t for compact records
struct CountLds {
  K *keys;         // [NL][cap]
  uint32_t *cnt;   // [cap]
  uint32_t *ext;   // [4][cap]: (A|C<<16, G|T<<16) left, then right
  int cap;         // multiple of 4: slots are probed in groups of 4
};

// An LDS fetch-add whose result is used later (k_count's dynamic slot counter, read at the end of the round): the
// address goes through an opaque move, so the atomic optimizer does not expand the add for a uniform address (a
// reduction over the active lanes that waits for the result at once: an LDS round trip at the top of every round).
typedef __attribute__((address_space(3))) unsigned int lds_u32_t;
__device__ __forceinline__ uint32_t lds_add_late(unsigned int *p, uint32_t v) {
  lds_u32_t *q = (lds_u32_t *)p;
  asm volatile("" : "+v"(q));
  return __hip_atomic_fetch_add(q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Groups a key may probe before its record is deferred to the next sweep of its bucket.
constexpr int C_PROBE = 64;
// First-group reads a lane keeps in flight in phase A (two-word keys: one at a time, measured 11.39 -> 11.24 ms at
// k = 63; their group read is two ds_read_b128).
template <int NL>
constexpr int count_batch() {
  return NL == 2 ? 1 : 2;
}
// Slots per probe group of k_count's table: a lane's home lookup reads one group, 4 slots = one ds_read_b128 of
// 32-bit keys (two of 64-bit keys). Two-slot groups (one ds_read_b64 / b128) measured the same for compact keys and
// slower for two-, three- and four-word keys with one record per lane per round (§3.3, §4.2).
constexpr int GS_SLOTS = 4;

// The last key words of one group (4 x u64: two ds_read_b128, the group 32-byte aligned; 2 x u64: one)
template <int GS>
__device__ __forceinline__ void read_group(const uint64_t *last, int g, uint64_t (&v)[GS]) {
  const ulonglong2 *q = (const ulonglong2 *)(last + GS * g);
  const ulonglong2 a = q[0];
  v[0] = a.x, v[1] = a.y;
  if constexpr (GS == 4) {
    const ulonglong2 b = q[1];
    v[2] = b.x, v[3] = b.y;
  }
}
// 32-bit keys: one ds_read_b128 per 4-slot group, one ds_read_b64 per 2-slot group
template <int GS>
__device__ __forceinline__ void read_group(const uint32_t *last, int g, uint32_t (&v)[GS]) {
  if constexpr (GS == 4) {
    const uint4 a = *(const uint4 *)(last + 4 * g);
    v[0] = a.x, v[1] = a.y, v[2] = a.z, v[3] = a.w;
  } else {
    const uint2 a = *(const uint2 *)(last + 2 * g);
    v[0] = a.x, v[1] = a.y;
  }
}

template <int NL, typename K>
__device__ __forceinline__ bool rest_equal(const CountLds<K> &t, int slot, const uint64_t *key) {
  bool eq = true;
#pragma unroll
  for (int w = 0; w < NL - 1; w++) eq &= (t.keys[w * t.cap + slot] == key[w]);
  return eq;
}

// Result of looking at one group for key: >= 0 the slot holding it, -1 - i an empty slot i (and the key is
// not in the group), G_FULL no empty slot and no key, G_BUSY a multi-word key is being written.
constexpr int G_FULL = -8, G_BUSY = -9;
template <int NL, int GS, typename K>
__device__ __forceinline__ int examine_group(const CountLds<K> &t, const uint64_t *key, int g, const K (&v)[GS]) {
  const K kl = (K)key[NL - 1];
  if constexpr (NL == 1) {  // single-word keys: eight compares and selects, no branch (a key is never EMPTY)
    int r = G_FULL;
#pragma unroll
    for (int i = GS - 1; i >= 0; i--) r = v[i] == (K)KEY_EMPTY ? -1 - i : r;  // the first empty slot
#pragma unroll
    for (int i = GS - 1; i >= 0; i--) r = v[i] == kl ? GS * g + i : r;  // the key itself takes precedence
    return r;
  }
  if constexpr (NL >= 2) {  // the same on the last word, then one read of the other words
    int r = G_FULL;
#pragma unroll
    for (int i = GS - 1; i >= 0; i--) r = v[i] == (K)KEY_EMPTY ? -1 - i : r;
#pragma unroll
    for (int i = GS - 1; i >= 0; i--) r = v[i] == (K)KEY_BUSY ? G_BUSY : r;
#pragma unroll
    for (int i = GS - 1; i >= 0; i--) r = v[i] == kl ? GS * g + i : r;
    // a slot holding the last word: the key iff its other words match too (a second slot of the group with
    // the same last word is possible, so a mismatch falls back to the full examination below)
    if (r < 0 || rest_equal<NL>(t, r, key)) return r;
  }
  int found = -1, empty = -1;
  bool busy = false;
#pragma unroll
  for (int i = 0; i < GS; i++) {
    if (found < 0 && v[i] == kl && (NL == 1 || rest_equal<NL>(t, GS * g + i, key))) found = i;
    if (v[i] == (K)KEY_EMPTY && empty < 0) empty = i;
    if (NL > 1 && v[i] == (K)KEY_BUSY) busy = true;
  }
  if (found >= 0) return GS * g + found;
  if (busy) return G_BUSY;
  return empty >= 0 ? -1 - empty : G_FULL;
}

// Find-or-insert of key, starting at group g whose examination (examine_group) gave r: the caller reads
// the first group of all its records back to back and keeps only that verdict. Grouped linear probing
// over at most C_PROBE groups; slots are claimed by a CAS on the last key word (multi-word keys: CAS to
// BUSY, write the other words, publish the last word with a release store; readers re-read a BUSY group)
// and are never freed within a sweep.
// Returns the slot, -1 when the key is absent and all its C_PROBE groups are full (the record is deferred
// to the next sweep), -2 on an internal bound violation.
// Deferral is per key, never per occurrence: a key is deferred only when its C_PROBE groups held neither
// the key nor an empty slot; slots only fill, so the key can never be inserted later in the sweep, and had
// it been inserted earlier this lookup would have found it. Every occurrence of a key is therefore counted
// in the same sweep; no occupancy counter is needed.
template <int NL, int GS, typename K>
__device__ int lds_insert(const CountLds<K> &t, const uint64_t *key, int g, int r) {
  K *last = t.keys + (NL - 1) * t.cap;
  const int ng = t.cap / GS;
  const K kl = (K)key[NL - 1];
  int probed = 0;
  for (int iter = 0; iter < (1 << 20); iter++) {
    if (r >= 0) return r;
    if (r == G_FULL) {
      if (++probed == C_PROBE * 4 / GS) return -1;  // C_PROBE 4-slot groups' worth of slots
      g = (g + 1 == ng) ? 0 : g + 1;
    } else if (r != G_BUSY) {
      const int sl = GS * g + (-1 - r);
      const K want = (NL == 1) ? kl : (K)KEY_BUSY;
      K old;
      if constexpr (sizeof(K) == 4)
        old = atomicCAS((unsigned int *)&last[sl], 0xffffffffu, (unsigned int)want);
      else
        old = atomicCAS((unsigned long long *)&last[sl], (unsigned long long)KEY_EMPTY, (unsigned long long)want);
      if (old == (K)KEY_EMPTY) {
        if (NL > 1) {
#pragma unroll
          for (int w = 0; w < NL - 1; w++) t.keys[w * t.cap + sl] = (K)key[w];
          __hip_atomic_store(&last[sl], kl, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        return sl;
      }
      if (NL == 1 && old == kl) return sl;  // the winner inserted this very key
      // otherwise the slot was just taken: look at the group again
    }
    K v[GS];
    read_group<GS>(last, g, v);
    r = examine_group<NL, GS>(t, key, g, v);
  }
  return -2;
}

// Phase A claim of the home group's first empty slot for a key the group does not hold: one CAS
// instead of a trip through the miss list and phase B, for most new keys (a third of all records at k = 63).
// Returns the slot, or the verdict unchanged when the CAS lost (the record then goes to the miss list).
// Sound by lds_insert's argument: the home group had an empty slot, so the key is in no later group, and
// of the lanes that saw this slot empty exactly one claims it; a single-word key that lost to its own key
// is counted in the winner's slot, any other loser is resolved by phase B.
template <int NL, int GS, typename K>
__device__ __forceinline__ int claim_home(const CountLds<K> &t, const uint64_t *key, int g, int r) {
  K *last = t.keys + (NL - 1) * t.cap;
  const int sl = GS * g + (-1 - r);
  const K kl = (K)key[NL - 1];
  if constexpr (NL == 1) {
    K old;
    if constexpr (sizeof(K) == 4)
      old = atomicCAS((unsigned int *)&last[sl], 0xffffffffu, (unsigned int)kl);
    else
      old = atomicCAS((unsigned long long *)&last[sl], (unsigned long long)KEY_EMPTY, (unsigned long long)kl);
    return (old == (K)KEY_EMPTY || old == kl) ? sl : r;
  } else {
    const K old = atomicCAS((unsigned long long *)&last[sl], (unsigned long long)KEY_EMPTY, (unsigned long long)KEY_BUSY);
    if (old != (K)KEY_EMPTY) return r;
#pragma unroll
    for (int w = 0; w < NL - 1; w++) t.keys[w * t.cap + sl] = (K)key[w];
    __hip_atomic_store(&last[sl], kl, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    return sl;
  }
}

// insert_supermer_from_read's per-k-mer update (src/kcount/kcount_cpu.cpp:343-352): count + 1,
// left/right extension + 1 when they are A/C/G/T (ExtCounts::inc ignores the rest, :152-164).
// Extension counters are 16-bit halves of u32 LDS words, added without a return value; the old count
// is returned for the saturation check (lds_clamp).
template <typename K>
__device__ __forceinline__ uint32_t lds_add(const CountLds<K> &t, int slot, uint32_t e) {
  const uint32_t old = atomicAdd(&t.cnt[slot], 1u);
  const int l = (int)((e >> 3) & 7u), r = (int)(e & 7u);
  if (l < 4) atomicAdd(&t.ext[(l >> 1) * t.cap + slot], (l & 1) ? 0x10000u : 1u);
  if (r < 4) atomicAdd(&t.ext[(2 + (r >> 1)) * t.cap + slot], (r & 1) ? 0x10000u : 1u);
  return old;
}

// The update of a cold sweep (fewer than 0xC000 records: no counter can reach the clamp level, a counter
// never exceeds the sweep's records). Two non-returning adds and no branch: the count is not kept but
// derived at the end, count = left A + C + G + T + left-none, where left-none (a neighbour that is not a
// countable base) is counted in the count word (< 0xC000 there); a right-none add goes to a dummy word of
// the wave. slot_count() reads it back; ctg_apply stores an explicit count as 0x80000000 | count.
// (Three adds, count and both extensions: 8.24 -> 8.32 ms in round 1; branch-free adds of 0 by every lane
// that has nothing to count: 4.85 -> 5.04 ms in round 3.)
template <typename K>
__device__ __forceinline__ void lds_add_nr(const CountLds<K> &t, int slot, uint32_t e, uint32_t *dummy) {
  const uint32_t l = (e >> 3) & 7u, r = e & 7u;
  uint32_t *lw = l < 4u ? &t.ext[(l >> 1) * t.cap + slot] : &t.cnt[slot];
  atomicAdd(lw, (l & 1u) ? 0x10000u : 1u);
  uint32_t *rw = r < 4u ? &t.ext[(2 + (r >> 1)) * t.cap + slot] : dummy;
  atomicAdd(rw, (r & 1u) ? 0x10000u : 1u);
}

// The count of an occupied slot (see lds_add_nr for the cold-sweep encoding).
template <typename K>
__device__ __forceinline__ uint32_t slot_count(const CountLds<K> &t, int slot, bool cold) {
  const uint32_t c = t.cnt[slot];
  if (!cold) return c;
  if (c >> 31) return c & 0x7fffffffu;
  const uint32_t e0 = t.ext[slot], e1 = t.ext[t.cap + slot];
  return c + (e0 & 0xffffu) + (e0 >> 16) + (e1 & 0xffffu) + (e1 >> 16);
}

// Saturation at the decision level: a 16-bit half that reached 0xC000 is CAS-clamped back to 0x8000.
// Exact for the reference's get_ext, which only compares counters against thresholds
// <= max((int)(0.1 * 65535), dmin_thres) <= 32768, and whose top base is unique whenever it is chosen
// (DESIGN.md §3.4); the reference saturates the same counters at 65535 (kcount_cpu.cpp:148-164).
// When to check: a half never exceeds its k-mer's count, and between a lane's count add and its own
// extension add fewer than S = records per round other adds happen (the round barrier closes the
// round). So a lane whose count add returned old < 0xC000 - 2S cannot push a half to 0xC000, and every
// add that does is followed by its own lane's clamp before another S adds: a half stays below
// 0xC000 + S < 0x10000 and never carries into its neighbour.
__device__ __forceinline__ void ext_clamp(uint32_t *p, int half) {
  uint32_t cur = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  for (int iter = 0; iter < 4096; iter++) {
    const uint32_t f = half ? (cur >> 16) : (cur & 0xffffu);
    if (f < 0xC000u) break;
    const uint32_t nw = half ? ((cur & 0xffffu) | 0x80000000u) : ((cur & 0xffff0000u) | 0x8000u);
    const uint32_t prev = atomicCAS(p, cur, nw);
    if (prev == cur) break;
    cur = prev;
  }
}

template <typename K>
__device__ __forceinline__ void lds_clamp(const CountLds<K> &t, int slot, uint32_t e) {
  const int l = (int)((e >> 3) & 7u), r = (int)(e & 7u);
  if (l < 4) ext_clamp(&t.ext[(l >> 1) * t.cap + slot], l & 1);
  if (r < 4) ext_clamp(&t.ext[(2 + (r >> 1)) * t.cap + slot], r & 1);
}

// Diagnostic phase stamps of k_count (MHMKC_STAMP builds only): wave cycles per phase, summed into
// stats[8..15]: clear, load wait, insert/update, round barrier, overflow handling, finalize.
#ifndef MHMKC_STAMP
#define MHMKC_STAMP 0
#endif
#if MHMKC_STAMP
#define STAMP(var) const uint64_t var = __builtin_amdgcn_s_memtime()
#define STAMP_ADD(i, v) st_acc[i] += (v)
#else
#define STAMP(var)
#define STAMP_ADD(i, v)
#endif

// Final decision for one listed table slot (count >= 2): insert_into_local_hashtable
// (src/kcount/kcount_cpu.cpp:503-517): left/right = get_ext(count) (kcount_cpu.cpp:173-182, with the exact double
// expression of the dynamic threshold); both 'X' -> purged. The caller reads the slot's count word and its four
// extension words together (one LDS round trip: a listed slot always has count >= 2, so nothing waits for the count).
__device__ __forceinline__ bool slot_survives(uint32_t c32, uint32_t e0, uint32_t e1, uint32_t e2, uint32_t e3,
                                              const CountParams &p, uint16_t &c16, char &L, char &R) {
  const uint32_t c = c32 > 65535u ? 65535u : c32;
  c16 = (uint16_t)c;
  const int thr = dyn_threshold(c, p.dyn_mult, p.dmin_thres);
  L = ext_choice(e0 & 0xffffu, e0 >> 16, e1 & 0xffffu, e1 >> 16, thr);
  R = ext_choice(e2 & 0xffffu, e2 >> 16, e3 & 0xffffu, e3 >> 16, thr);
  return !(L == 'X' && R == 'X');
}

// Contig pass, applied in k_count once a sweep has inserted its reads (kcount_ctg.hip folds the contig
// occurrences of every k-mer; see there). For each folded contig k-mer of bucket b not yet applied: if the
// key is in this sweep's table its read entry is kept when it has count >= 2 and unique extensions on both
// sides (UU), otherwise it is replaced by the contig entry (insert_supermer_from_ctg,
// src/kcount/kcount_cpu.cpp:367-404); a key absent from the table is absent from the reads once the
// bucket's last sweep has run (deferred keys are counted in a later sweep), and is finalized here
// directly (insert_into_local_hashtable, kcount_cpu.cpp:503-522).
template <int NL, bool CMP, typename K>
__device__ void ctg_apply(const CountLds<K> &t, const CountParams &p, uint32_t b, bool last_sweep, bool cold,
                          unsigned long long *s_range) {
  const int tid = threadIdx.x;
  if (tid == 0) {
    auto lower = [&](uint32_t v) {
      uint64_t lo = 0, hi = p.ctg_n;
      while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (p.ctg_bucket[mid] < v)
          lo = mid + 1;
        else
          hi = mid;
      }
      return lo;
    };
    s_range[0] = lower(p.ctg_base + b);
    s_range[1] = lower(p.ctg_base + b + 1);
  }
  __syncthreads();
  const uint64_t q0 = s_range[0], q1 = s_range[1];
  constexpr int GS = GS_SLOTS;
  const int ng = t.cap / GS;
  const K *last = t.keys + (NL - 1) * t.cap;
  for (uint64_t q = q0 + tid; q < q1; q += C_THREADS) {
    if (p.ctg_done[q]) continue;
    uint64_t key[NL];
#pragma unroll
    for (int w = 0; w < NL; w++) key[w] = p.ctg_keys[w][q];
    const uint32_t st = p.ctg_state[q];
    const uint32_t c = st & 0xffffu, l = (st >> 16) & 7u, r = (st >> 19) & 7u;
    uint64_t tkey[NL];  // the key as the table holds it
#pragma unroll
    for (int w = 0; w < NL; w++) tkey[w] = key[w];
    if (RecKind<NL, CMP>::C32) {  // compact: the mixed key's bits below the bucket digits, above the ext code
      const int B = 2 * p.k, rb = B - p.coarse_bits - p.fine_bits;
      tkey[0] = (cmix(key[0] >> (64 - B), B) & ((1ull << rb) - 1)) << EXT_BITS;
    } else if (RecKind<NL, CMP>::M2) {  // mixed two-word: L' below the bucket digits << 6, R'
      uint64_t L, R;
      m2_mix(key, p.k, L, R);
      tkey[0] = (L & ((1ull << (p.k - p.coarse_bits - p.fine_bits)) - 1)) << EXT_BITS;
      tkey[NL - 1] = R;
    } else if (RecKind<NL, CMP>::MX) {  // mixed three- and four-word: w0' below the bucket digits << 6, r[1..]
      uint64_t r[NL];
      mx_mix<NL>(key, r);
      tkey[0] = (r[0] & ((1ull << (64 - p.coarse_bits - p.fine_bits)) - 1)) << EXT_BITS;
#pragma unroll
      for (int w = 1; w < NL; w++) tkey[w] = r[w];
    }
    int g = RecKind<NL, CMP>::C32 ? cmp_group((uint32_t)tkey[0], 26 - (2 * p.k - p.coarse_bits - p.fine_bits), (uint32_t)ng)
            : RecKind<NL, CMP>::MW ? cmp_group((uint32_t)tkey[NL - 1], 16, (uint32_t)ng)
                                   : (int)__umulhi(slot_hash<NL>(tkey), (uint32_t)ng);
    int slot = -1;
    for (int pr = 0; pr < C_PROBE * 4 / GS; pr++) {  // find only: a key in the table is within its probe window
      K v[GS];
      read_group<GS>(last, g, v);
      const int e = examine_group<NL, GS>(t, tkey, g, v);
      if (e >= 0) {
        slot = e;
        break;
      }
      if (e != G_FULL) break;  // an empty slot: absent
      g = (g + 1 == ng) ? 0 : g + 1;
    }
    if (slot >= 0) {
      const uint32_t c32 = slot_count(t, slot, cold);
      const uint32_t rc = c32 > 65535u ? 65535u : c32;
      bool keep = false;
      if (rc >= 2) {
        const int thr = dyn_threshold(rc, p.dyn_mult, p.dmin_thres);
        const uint32_t e0 = t.ext[slot], e1 = t.ext[t.cap + slot], e2 = t.ext[2 * t.cap + slot],
                       e3 = t.ext[3 * t.cap + slot];
        const char L = ext_choice(e0 & 0xffffu, e0 >> 16, e1 & 0xffffu, e1 >> 16, thr);
        const char R = ext_choice(e2 & 0xffffu, e2 >> 16, e3 & 0xffffu, e3 >> 16, thr);
        keep = L != 'X' && L != 'F' && R != 'X' && R != 'F';
      }
      if (!keep) {  // {count, left[l] = right[r] = count, from_ctg}; halves >= 0xC000 as 0x8000 (§3.4)
        const uint32_t h = c >= 0xC000u ? 0x8000u : c;
        uint32_t ew[4] = {0, 0, 0, 0};
        if (l < 4) ew[l >> 1] |= h << ((l & 1u) * 16);
        if (r < 4) ew[2 + (r >> 1)] |= h << ((r & 1u) * 16);
        t.cnt[slot] = cold ? 0x80000000u | c : c;  // an explicit count (slot_count)
#pragma unroll
        for (int i = 0; i < 4; i++) t.ext[i * t.cap + slot] = ew[i];
      }
      p.ctg_done[q] = 1;
    } else if (last_sweep) {
      const int thr = dyn_threshold(c, p.dyn_mult, p.dmin_thres);
      uint32_t cl[4] = {0, 0, 0, 0}, cr[4] = {0, 0, 0, 0};
      if (l < 4) cl[l] = c;
      if (r < 4) cr[r] = c;
      const char L = ext_choice(cl[0], cl[1], cl[2], cl[3], thr), R = ext_choice(cr[0], cr[1], cr[2], cr[3], thr);
      atomicAdd(&p.stats[STAT_DISTINCT], 1ull);
      atomicAdd(&p.stats[STAT_COUNTSUM], (unsigned long long)c);
      if (c >= 2 && !(L == 'X' && R == 'X')) {
        const unsigned long long o = atomicAdd(p.out_cursor, 1ull);
        atomicAdd(&p.stats[STAT_NOUT], 1ull);
        if (o >= p.out_cap) {  // the output is full: flag the launch (the host grows it and redoes the pass)
          atomicOr(p.err, 16u);
          p.ctg_done[q] = 1;
          continue;
        }
        uint64_t *ok = p.out_keys + o * (uint64_t)p.nlo;
#pragma unroll
        for (int w = 0; w < NL; w++) ok[w] = key[w];
        for (int w = NL; w < p.nlo; w++) ok[w] = 0;
        p.out_counts[o] = (uint16_t)c;
        p.out_left[o] = L;
        p.out_right[o] = R;
      } else {
        atomicAdd(&p.stats[STAT_PURGED], 1ull);
      }
      p.ctg_done[q] = 1;
    }
  }
  __syncthreads();
}

// A deferred record goes back unchanged: key | raw low bits (ext code, stored hash bits).
template <int NL, bool PACKED, bool CMP>
__device__ __forceinline__ void store_record(const PlaneSet &ps, uint64_t idx, const uint64_t *key, uint32_t e) {
  if (RecKind<NL, CMP>::C32) {
    ((uint32_t *)ps.w[0])[idx] = (uint32_t)(key[0] | e);
    return;
  }
  if (RecKind<NL, CMP>::M2) {
    ((ulonglong2 *)ps.w[0])[idx] = make_ulonglong2(key[0] | e, key[NL - 1]);
    return;
  }
#pragma unroll
  for (int w = 0; w < NL; w++) ps.w[w][idx] = (w == RecKind<NL, CMP>::XW && PACKED) ? (key[w] | e) : key[w];
  if (!PACKED) ps.ext[idx] = (uint8_t)e;
}


// k_count's thread index. For four-word keys it is recomputed through an opaque move at every use, so that nothing
// derived from it is hoisted out of the bucket loop to live in registers across it: that took 9 spilled VGPRs to
// none (127 -> 124) and the count at k = 99 11.79 -> 11.05 ms; at NL = 1-3 it measured 1-3 % slower (the recomputed
// addresses cost more than the registers they free).
__device__ __forceinline__ int count_opaque_tid() {
  int t;
  asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"((int)threadIdx.x));
  return t;
}
template <int NL>
__device__ __forceinline__ int count_tid() {
  if constexpr (NL >= 4)
    return count_opaque_tid();
  else
    return (int)threadIdx.x;
}

template <int NL, bool PACKED, bool CMP>
// (C_SPLIT workgroups per CU must fit its registers together: 4 waves per SIMD, 128 VGPRs each, as one 1024-thread
// workgroup has)
__global__ __launch_bounds__(C_THREADS, 4) void k_count(CountParams p) {
  // A capped fine bucket overflowed in k_part_scatter (same stream, earlier launch): its cursor, which is
  // this kernel's bucket end, ran past the bucket, so reading up to it would leave the layout. The host
  // discards this launch and redoes the partition with exact bucket sizes. (Uniform: every lane reads the
  // same word before any barrier.)
  if (p.err && (__hip_atomic_load(p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 2u)) return;
  extern __shared__ __align__(16) unsigned char smem[];
  using RK = RecKind<NL, CMP>;
  using K = typename std::conditional<RK::C32, uint32_t, uint64_t>::type;
  CountLds<K> t;
  t.cap = p.cap & 0xffff;  // (< 2^16: the compiler then multiplies plane indices by it with v_mul_u32_u24)
  t.keys = (K *)smem;
  t.cnt = (uint32_t *)(t.keys + NL * t.cap);
  t.ext = t.cnt + t.cap;
  // scalars live after the table in the same dynamic region (count_table_bytes adds 256 bytes)
  unsigned long long *s_u64 = (unsigned long long *)(t.ext + 4 * t.cap);
  unsigned long long &s_gbase = s_u64[0];
  unsigned long long *s_red = s_u64 + 1;  // [3]
  unsigned int &s_ovf = *(unsigned int *)(s_u64 + 5);
  unsigned int &s_err = *((unsigned int *)(s_u64 + 5) + 1);
  unsigned int *s_wave = (unsigned int *)(s_u64 + 6);  // [16] per-wave survivor counts, then offsets
  unsigned int *s_wdef = (unsigned int *)(s_u64 + 16);  // [16] per-wave deferred records of the sweep
  unsigned int &s_next = *(unsigned int *)(s_u64 + 24);   // dynamic sweeps: the next record slot to hand out
  // miss space after the largest table this NL can have: keys [NL][MC] | ext [MC], cut into one miss queue per wave
  // (MW entries; a shared list worked off by the lowest threads held the other waves at the round barrier, §3.3),
  // worked off by its own wave once it holds WQ_THR entries, and emptied after the sweep's last round
  constexpr int MC = miss_cap(NL, RK::C32);
  constexpr int MW = MC / (C_THREADS / 64);
  // (round 4, with one record per lane per round: a two-word key's queue is worked off when its slice is full, not
  // half full: k = 63 count 8.27 -> 8.00 ms; three-word keys measured 10.28 -> 11.48 ms that way, four-word the same;
  // a quarter of the slice: 5.42 -> 5.62 ms at k = 21)
  constexpr int WQ_THR = NL == 2 ? (MW < 64 ? MW : 64) : (MW / 2 < 64 ? MW / 2 : 64);
  const uint32_t wq_base = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * (uint32_t)MW;
  K *s_mkey = (K *)(smem + count_table_bytes(NL, RK::C32));
  uint32_t *s_me = (uint32_t *)(s_mkey + NL * MC);
  constexpr int SPT = (count_cap(NL, RK::C32) + C_THREADS - 1) / C_THREADS;  // table slots per thread (finalize)
  // The finalize keeps its survivors' key words in registers (one- to three-word keys; four key words would
  // hold SPT x NL x 2 more VGPRs) when the slots it lists fit KJ per thread, so that it clears the table while the
  // output reservation is in flight; a bucket with more listed slots writes its output from the table first.
#ifndef MHMKC_KREG_NL
#define MHMKC_KREG_NL 3
#endif
#ifndef MHMKC_KJ
#define MHMKC_KJ 2
#endif
  constexpr bool KREG = NL <= MHMKC_KREG_NL;
  constexpr int KJ = KREG ? (MHMKC_KJ < SPT ? MHMKC_KJ : SPT) : 1;

#define tid (count_tid<NL>())  // (see count_tid; #undef after the kernel)
#define lane (count_tid<NL>() & 63)
// the wave index as a scalar (readfirstlane): per-wave queue / deferral / scan-slot addresses in SGPRs
// (k = 21 count 4.83 -> 4.78 ms, k = 63 9.05 -> 8.95, k = 99 11.08 -> 11.03)
#define wid (__builtin_amdgcn_readfirstlane(count_tid<NL>() >> 6))
  const uint64_t low_mask = (1ull << (EXT_BITS + p.hbits)) - 1;

  constexpr int R = count_rpt<NL>();
  constexpr uint32_t NONE = 0xffffffffu;
  constexpr uint32_t RND = (uint32_t)R * C_THREADS;
  // see ext_clamp: between two barriers a round's records and at most the miss space's queued records are added
  constexpr uint32_t HOT = 0xC000u - 2u * (RND + (uint32_t)miss_cap(NL, RecKind<NL, CMP>::C32));
  static_assert(HOT > 0x8000u, "round too large for the extension-counter clamp");
  constexpr int C_BATCH = count_batch<NL>() < R ? count_batch<NL>() : R;
  static_assert(R % C_BATCH == 0, "batch must divide the records per round");
  constexpr int GS = GS_SLOTS;  // slots per probe group
  const int ng = t.cap / GS;
  const K *last = t.keys + (NL - 1) * t.cap;
  // cmp_group: compact keys from their top stored bits; mixed two-word keys from the low 16 bits of R' (the
  // table's last word)
  const int kshl = RK::C32 ? 26 - (2 * p.k - p.coarse_bits - p.fine_bits) : 16;

  // Persistent workgroups: workgroup w counts buckets w, w + G, w + 2G, ... (G = grid size). The first
  // round of the next bucket is loaded while the current one is finalized, so no bucket starts with an
  // exposed HBM round trip.
  // Raw records of the next round, loaded unconditionally (lanes past the end re-read the last record)
  // and split into key / ext only when the round starts, so the loads stay in flight (see load_chunk).
  uint64_t nk[R][NL];
  uint32_t nx[R];
  // Compact records: a lane takes 4 consecutive records of the round with one 16-byte load (bucket bases are
  // multiples of 4 records: capped fine buckets are multiples of 16, the exact scan rounds them up), so one
  // address per 4 records; lanes past the end re-read the last aligned quad (inside the bucket's region).
  static_assert(!RK::C32 || R == 4, "compact rounds take one 16-byte load of 4 records per lane");
  // nwv: NONE for a dense sweep of cnt records, else this wave's records of a re-sweep (wave-owned positions,
  // see defer_pos; lanes past them read the bucket's first record or quad)
  // A record source: the fine records (p.recs) or this workgroup's spill area (p.spill), from record `off` on. Kept
  // as (offset, which) and turned into plane pointers where used: full plane sets for the bucket, the next bucket and
  // the spill area held across the sweep loop spilled registers at three and four key words.
  struct Src {
    uint64_t off;
    uint32_t spl;
  };
  auto planes_of = [&](const Src &sr) -> PlaneSet {
    PlaneSet q = sr.spl ? p.spill : p.recs;
    const uint64_t o = sr.off;
    if (RK::C32) {
      q.w[0] = (uint64_t *)((uint32_t *)q.w[0] + o);
    } else if (RK::M2) {
      q.w[0] += 2 * o;
    } else {
#pragma unroll
      for (int w = 0; w < NL; w++) q.w[w] += o;
    }
    if (!PACKED) q.ext += o;
    return q;
  };
  // (vt: the thread slot whose records to load, tid except in dynamic sweeps)
  auto prefetch = [&](const Src &sr, uint32_t cnt, uint32_t first, uint32_t nwv, uint32_t vt) {
    const PlaneSet src = planes_of(sr);
    const uint32_t dbase = first / RND * (uint32_t)(64 * R);
    if constexpr (RK::C32) {
      const uint32_t q = first + 4u * vt, qmax = (cnt - 1) & ~3u;
      const uint32_t qq = nwv == NONE ? (q < qmax ? q : qmax) : (dbase + 4u * (uint32_t)lane < nwv ? q : 0u);
      const u32x4 v = gload4((const uint32_t *)src.w[0] + qq);
      nk[0][0] = v.x;
      nk[1][0] = v.y;
      nk[2][0] = v.z;
      nk[3][0] = v.w;
#pragma unroll
      for (int j = 0; j < R; j++) nx[j] = 0;
      return;
    }
#pragma unroll
    for (int j = 0; j < R; j++) {
      const uint32_t i = first + vt + (uint32_t)j * C_THREADS;
      const uint32_t idx = nwv == NONE ? (i < cnt ? i : cnt - 1) : (dbase + (uint32_t)(64 * j + lane) < nwv ? i : 0u);
      if (RK::C32) {
        nk[j][0] = ((const uint32_t *)src.w[0])[idx];
      } else if (RK::M2) {  // one 16-byte record
        const u32x4 v = gload4((const uint32_t *)src.w[0] + 4 * (uint64_t)idx);
        nk[j][0] = (uint64_t)v.x | ((uint64_t)v.y << 32);
        nk[j][NL - 1] = (uint64_t)v.z | ((uint64_t)v.w << 32);
      } else {
#pragma unroll
        for (int w = 0; w < NL; w++) nk[j][w] = src.w[w][idx];
      }
      nx[j] = PACKED ? 0u : (uint32_t)src.ext[idx];
    }
  };
  // a bucket's records from its extent [base, end) (< 2^32 records per bucket: host check)
  auto bucket_at = [&](uint64_t base, uint64_t end, Src &src, uint32_t &cnt) {
    cnt = (uint32_t)(end - base);
    src = Src{base, 0u};
  };
  auto bucket = [&](uint32_t bb, Src &src, uint32_t &cnt) { bucket_at(p.bucket_base[bb], p.bucket_end[bb], src, cnt); };

  // Position of a record deferred to the next sweep. With per-wave queues a wave defers only records it loaded
  // itself, so its d-th deferral goes to its own d-th record position of the sweep (wave-owned positions in round
  // order: lanes 64 apart for one record per lane, 4 consecutive records per lane for compact quads), which it
  // has already consumed: no other wave reads it, and the waves need no barrier between rounds. The next sweep
  // reads the first s_wdef[w] positions of every wave w.
  auto defer_pos = [&]() -> uint32_t {
    (void)atomicAdd(&s_ovf, 1u);
    const uint32_t d = atomicAdd(&s_wdef[wid], 1u), rr = d / (uint32_t)(64 * R), rem = d % (uint32_t)(64 * R);
    return rr * RND + (RK::C32 ? (uint32_t)wid * 256u + rem : rem / 64u * C_THREADS + (uint32_t)wid * 64u + rem % 64u);
  };
  unsigned long long my_occ = 0, my_purged = 0, my_sum = 0, my_out = 0, my_sweeps = 0, my_maxb = 0;
  unsigned long long &s_missacc = s_u64[4];  // phase-B records of this workgroup (the LDS op mix, stats)
#if MHMKC_STAMP
  uint64_t st_acc[6] = {0, 0, 0, 0, 0, 0};
  const uint64_t st_wg0 = __builtin_amdgcn_s_memtime();
#endif
  // clear the table with 16-byte stores: last-word plane = EMPTY, counters = 0
  auto clear_table = [&]() {
    uint4 *ones = (uint4 *)(t.keys + (NL - 1) * t.cap);
    const int n_ones = t.cap * (int)sizeof(K) / 16;
    for (int i = tid; i < n_ones; i += C_THREADS) ones[i] = make_uint4(~0u, ~0u, ~0u, ~0u);
    uint4 *zeros = (uint4 *)t.cnt;
    const int n_zeros = t.cap * 20 / 16;
    for (int i = tid; i < n_zeros; i += C_THREADS) zeros[i] = make_uint4(0, 0, 0, 0);
  };
  // a sweep's scalars: deferral counters, dynamic slot counter, error flag
  auto reset_sweep = [&]() {
    if (tid == 0) {
      s_ovf = 0;
      s_err = 0;
      s_next = 2 * (C_THREADS / 64);  // (slots s and 16 + s are wave s's own: already prefetched / next)
    }
    if (tid < C_THREADS / 64) s_wdef[tid] = 0;
  };
  if (tid == 0) {
    s_missacc = 0;
    s_u64[3] = 0;  // finalize's counters
  }
  // the first sweep's table; every later sweep's is cleared by the finalize before it
  clear_table();
  reset_sweep();
  __syncthreads();
  // this workgroup's spill area (dynamic sweeps: their deferred records; the sweep after reads them from there)
  const Src spill{(uint64_t)blockIdx.x * SPILL_RECORDS, 1u};
  const bool has_spill = p.spill.w[0] != nullptr;
  uint32_t b = blockIdx.x;
  Src ps;
  uint32_t n;
  bucket(b, ps, n);
  if (n) prefetch(ps, n, 0, NONE, (uint32_t)tid);
  while (true) {  // buckets
  my_maxb = my_maxb > n ? my_maxb : n;
  bool first_sweep = true;
  // records of this wave in a re-sweep (NONE: the first sweep, dense over [0, n)) and the sweep's round bound
  uint32_t nw = NONE, lim = n;
  // Dynamic sweeps (cold, with a spill area): the rounds' record slots of 64 lanes (a round's wave slot: lane l of
  // slot s of round r takes what thread 64 s + l would) are handed to the waves in order as they ask, so a wave that
  // runs ahead takes more of them and the waves reach the sweep's barrier together (statically, each wave's share
  // of a cold sweep ran without barriers and the waves drifted apart: the barrier held 17-25 % of k_count's wave
  // cycles, MHMKC_STAMP). Their deferred records go densely to the other of (bucket region, spill area), which the
  // next sweep (dynamic too: fewer records) reads.
  bool dyn_sweep = false;
  Src pd = spill;  // where a dynamic sweep defers to
  uint32_t nb_next = 0;
  Src ps_next;
  const uint32_t b_next = b + gridDim.x;
  // the next bucket's extent, loaded now so that its first records can be fetched at this bucket's finalize without
  // a dependent round trip there (unconditional: without a next bucket it re-reads this bucket's, never used)
  const uint32_t b_ext = b_next < p.n_buckets ? b_next : b;
  const uint64_t nx_base = p.bucket_base[b_ext], nx_end = p.bucket_end[b_ext];
  while (true) {  // sweeps of bucket b (the table is clear and the sweep's scalars reset)
    // R records per thread per round, the next round prefetched into registers, so that every CU keeps
    // R * 8 KB of record loads in flight. A round has two phases:
    //   A. every lane looks its records up in their home group; found keys are counted at once, a new key with an
    //      empty slot in its home group claims it, the others (lost claims, keys displaced by a full group) are
    //      appended to the wave's miss queue in LDS;
    //   B. the wave works its queue off densely, one record per lane (probing, CAS insert, counting), once it
    //      holds WQ_THR entries, so the slow path does not hold every wave in a divergent loop.
    if (!first_sweep && n) prefetch(ps, n, 0, nw, (uint32_t)tid);  // a re-sweep reads the deferred records
    first_sweep = false;
    // a sweep of fewer than 0xC000 records cannot bring a counter to the clamp level: its rounds count
    // with non-returning adds and carry no clamp check (COLD instantiation of the round loop)
    auto rounds = [&](auto cold_tag, auto dyn_tag) {
      constexpr bool COLD = decltype(cold_tag)::value;
      constexpr bool DYN = decltype(dyn_tag)::value;  // dynamic slots (cold sweeps only)
      constexpr uint32_t NWV = C_THREADS / 64;
      int rnd = 0;
      uint32_t wq_n = 0;  // entries in this wave's miss queue (wave-uniform)
      // DYN: this wave's slot (round cc / NWV, wave slot cc % NWV) and its next one; wave s starts with slots s and
      // NWV + s, every later one comes from s_next (asked for one slot ahead, so the answer is never waited for)
      uint32_t cc = (uint32_t)wid, cn = (uint32_t)wid + NWV;
      auto slot_first = [&](uint32_t c) { return c / NWV * RND + c % NWV * (RK::C32 ? 256u : 64u); };
      for (uint32_t r0 = 0; DYN ? slot_first(cc) < n : r0 < lim; r0 += RND, rnd++) {
        STAMP(t_r0);
        uint64_t ck[R][NL];
        uint32_t ce[R];
        uint32_t ca = 0;  // DYN: the slot after cn (lane 0 asks now, the answer is read at the end of the round)
        if (DYN && lane == 0) ca = lds_add_late(&s_next, 1u);
        const uint32_t cr0 = DYN ? cc / NWV * RND : r0;                              // the slot's round
        const uint32_t vt = DYN ? cc % NWV * 64u + (uint32_t)lane : (uint32_t)tid;  // its thread slot
        // record j of this lane is valid iff j * vstep < vrem: the records left from this lane's first one (a dense
        // sweep: [r0, n) in thread order; a re-sweep: this wave's own nw positions), saturated at 0
        const uint32_t vfirst = nw == NONE ? cr0 + (RK::C32 ? 4u * vt : vt)
                                           : (uint32_t)rnd * (uint32_t)(64 * R) + (RK::C32 ? 4u * (uint32_t)lane : (uint32_t)lane);
        const uint32_t vend = nw == NONE ? n : nw;
        const uint32_t vrem = (vend > vfirst ? vend : vfirst) - vfirst;
        const uint32_t vstep = RK::C32 ? 1u : nw == NONE ? (uint32_t)C_THREADS : 64u;
#pragma unroll
        for (int j = 0; j < R; j++) {
          const bool valid = (uint32_t)j * vstep < vrem;
#pragma unroll
          for (int w = 0; w < NL; w++) ck[j][w] = nk[j][w];
          if (PACKED) {
            ce[j] = valid ? (uint32_t)(ck[j][RK::XW] & low_mask) : NONE;
            ck[j][RK::XW] &= ~low_mask;
          } else {
            ce[j] = valid ? nx[j] : NONE;
          }
        }
#if MHMKC_STAMP
#pragma unroll
        for (int j = 0; j < R; j++) asm volatile("" ::"v"(ck[j][0]), "v"(ce[j]));
#endif
        STAMP(t_r1);
        STAMP_ADD(1, t_r1 - t_r0);
        // (unconditional: in the last round it re-reads this round's records, never used. A load under a branch
        // left its registers to a phi whose copies made hipcc wait for the load right there, vmcnt(0), so the next
        // round's records were fetched with the whole HBM latency exposed every round)
        if (DYN)  // (unconditional too: past the records it re-reads the last quad / record)
          prefetch(ps, n, cn / NWV * RND, NONE, cn % NWV * 64u + (uint32_t)lane);
        else
          prefetch(ps, n, r0 + RND < lim ? r0 + RND : r0, nw, (uint32_t)tid);
        // A. home-group lookups: the first groups of all R records are read in batches of C_BATCH (the
        //    reads of a batch in flight together), then found records are counted, missed ones listed.
        uint32_t old[R], defer = 0, okm = 0, missm = 0;
        int slot[R], g[R];
        if constexpr (RK::C32 && COLD) {
          // compact keys in a cold sweep: the R home groups read back to back and examined, every claim CAS
          // issued before the first one is waited for (the general path below waits for each in turn), then the
          // non-returning adds; misses join the wave queue below. Same verdicts as the general path.
          K gv[R][GS];
          uint32_t res[R];
#pragma unroll
          for (int j = 0; j < R; j++) {
            g[j] = cmp_group((uint32_t)ck[j][0], kshl, (uint32_t)ng);
            read_group<GS>(last, g[j], gv[j]);
          }
#pragma unroll
          for (int j = 0; j < R; j++) slot[j] = examine_group<NL, GS>(t, ck[j], g[j], gv[j]);
#pragma unroll
          for (int j = 0; j < R; j++) {
            res[j] = 0u;
            if (ce[j] != NONE && slot[j] < 0 && slot[j] > G_FULL)  // slot -1 - r of the home group was empty: claim it
              res[j] = atomicCAS((unsigned int *)&last[GS * g[j] - 1 - slot[j]], 0xffffffffu, (uint32_t)ck[j][0]);
          }
#pragma unroll
          for (int j = 0; j < R; j++) {
            old[j] = 0;
            int r = slot[j];
            if (r < 0 && r > G_FULL && (res[j] == 0xffffffffu || res[j] == (uint32_t)ck[j][0])) r = GS * g[j] - 1 - r;
            if (ce[j] == NONE) {
              slot[j] = -3;
            } else if (r >= 0) {
              slot[j] = r;
              lds_add_nr(t, r, ce[j], &s_wave[wid]);
              okm |= 1u << j;
            } else {  // a full home group, or a lost claim (lds_insert re-examines the group)
              missm |= 1u << j;
            }
          }
        } else {
#pragma unroll
        for (int j0 = 0; j0 < R; j0 += C_BATCH) {
          K v[C_BATCH][GS];
#pragma unroll
          for (int j = j0; j < j0 + C_BATCH; j++) {
            g[j] = CMP ? cmp_group((uint32_t)ck[j][NL - 1], kshl, (uint32_t)ng)
                       : (int)__umulhi(slot_hash<NL>(ck[j]), (uint32_t)ng);
            read_group<GS>(last, g[j], v[j - j0]);  // also for an invalid lane: harmless, keeps the batch uniform
          }
#pragma unroll
          for (int j = j0; j < j0 + C_BATCH; j++) slot[j] = examine_group<NL, GS>(t, ck[j], g[j], v[j - j0]);
        }
#pragma unroll
        for (int j = 0; j < R; j++) {
          old[j] = 0;
          if (ce[j] == NONE) {
            slot[j] = -3;
            continue;
          }
          int r = slot[j];
          if (r < 0 && r > G_FULL) {  // -1 - i: slot i of the home group was empty
            const int sl = GS * g[j] + (-1 - r);
            r = claim_home<NL, GS>(t, ck[j], g[j], r);
            if (NL > 1 && r < 0) {  // lost: the winner may have claimed it for this very key (a lane of this
                                    // wave has published it by now; another wave's is left to phase B)
              const K v = __hip_atomic_load(&last[sl], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
              if (v == (K)ck[j][NL - 1] && rest_equal<NL>(t, sl, ck[j])) r = sl;
            }
            slot[j] = r;
          }
          if (r < 0) {  // a full home group, or a lost claim: listed below, in wave-uniform code
            missm |= 1u << j;
            slot[j] = r;
            continue;
          }
          if (COLD)
            lds_add_nr(t, r, ce[j], &s_wave[wid]);
          else
            old[j] = lds_add(t, r, ce[j]);
          okm |= 1u << j;
        }
        }  // general phase A
        {
          // this wave's misses join its own queue (ballot + prefix: no LDS atomic); a queue without room for
          // them inserts in place
#pragma unroll
          for (int j = 0; j < R; j++) {
            const bool mj = (missm >> j) & 1u;
            const uint64_t bal = __ballot(mj);
            const uint32_t tot = (uint32_t)__popcll(bal);
            if (wq_n + tot <= (uint32_t)MW) {
              if (mj) {
                const uint32_t q = wq_base + wq_n +
                                   __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
#pragma unroll
                for (int w = 0; w < NL; w++) s_mkey[w * MC + q] = (K)ck[j][w];
                s_me[q] = ce[j];
                slot[j] = -3;
              }
              wq_n += tot;
            } else if (mj) {
              const int r = lds_insert<NL, GS>(t, ck[j], g[j], slot[j]);
              if (r == -1) defer |= 1u << j;
              if (r == -2) s_err = 1;
              slot[j] = r;
              if (r >= 0) {
                if (COLD)
                  lds_add_nr(t, r, ce[j], &s_wave[wid]);
                else
                  old[j] = lds_add(t, r, ce[j]);
                okm |= 1u << j;
              }
            }
          }
        }
#pragma unroll
        for (int j = 0; j < R; j++)
          if (!COLD && ((okm >> j) & 1u) && old[j] >= HOT) lds_clamp(t, slot[j], ce[j]);
        STAMP(t_r2);
        STAMP_ADD(2, t_r2 - t_r1);
        // The round barrier. A cold sweep needs none: no clamp bound to keep (§3.4), every wave works off its own
        // queue, and deferred records go to positions their own wave has consumed (defer_pos), so the waves drift
        // apart freely until the sweep's barrier (k = 63 count 10.9 -> 9.2 ms).
        if (!COLD) __syncthreads();
        STAMP(t_r3);
        STAMP_ADD(3, t_r3 - t_r2);
        // deferred records go back into the bucket for the next sweep, to positions already consumed (defer_pos)
        if (defer) {
#pragma unroll
          for (int j = 0; j < R; j++) {
            if ((defer >> j) & 1u) {
              if (DYN)
                store_record<NL, PACKED, CMP>(planes_of(pd), atomicAdd(&s_ovf, 1u), ck[j], ce[j]);
              else
                store_record<NL, PACKED, CMP>(planes_of(ps), defer_pos(), ck[j], ce[j]);
            }
          }
        }
        {
          // B. this wave's queue, 64 entries at a time once it holds WQ_THR (all of it after the sweep's last
          // round): whole-wave batches, and every wave takes its own share of the slow path, so no wave holds
          // the next barrier with the misses of all the others. The sweep's rounds run while r0 < lim (lim = n
          // in a first sweep; in a re-sweep lim >= n covers the largest wave share of deferred records), so the
          // queue is drained in the round the loop ends with.
          const bool last_round = DYN ? slot_first(cn) >= n : r0 + RND >= lim;
          while (wq_n >= (uint32_t)WQ_THR || (last_round && wq_n > 0)) {
            const uint32_t take = wq_n < 64u ? wq_n : 64u;
            const uint32_t qb = wq_n - take;
            if ((uint32_t)lane < take) {
              const uint32_t q = wq_base + qb + (uint32_t)lane;
              uint64_t key[NL];
#pragma unroll
              for (int w = 0; w < NL; w++) key[w] = s_mkey[w * MC + q];
              const uint32_t e = s_me[q];
              const int g = CMP ? cmp_group((uint32_t)key[NL - 1], kshl, (uint32_t)ng)
                                : (int)__umulhi(slot_hash<NL>(key), (uint32_t)ng);
              K v[GS];
              read_group<GS>(last, g, v);
              const int r = lds_insert<NL, GS>(t, key, g, examine_group<NL, GS>(t, key, g, v));
              if (r >= 0) {
                if (COLD)
                  lds_add_nr(t, r, e, &s_wave[wid]);
                else if (lds_add(t, r, e) >= HOT)
                  lds_clamp(t, r, e);
              } else if (r == -1) {
                if (DYN)
                  store_record<NL, PACKED, CMP>(planes_of(pd), atomicAdd(&s_ovf, 1u), key, e);
                else
                  store_record<NL, PACKED, CMP>(planes_of(ps), defer_pos(), key, e);
              } else {
                s_err = 1;
              }
            }
            if (lane == 0) atomicAdd(&s_missacc, (unsigned long long)take);
            wq_n = qb;
          }
          if (DYN) {
            cc = cn;
            cn = __builtin_amdgcn_readfirstlane(ca);
          }
#if MHMKC_STAMP
          const uint64_t t_r4w = __builtin_amdgcn_s_memtime();
          STAMP_ADD(4, t_r4w - t_r3);
#endif
        }
      }
    };
    // (s_wave holds the dummy words of the cold adds until finalize overwrites it after a barrier)
    // dynamic: a cold first sweep, or a sweep after a dynamic one (fewer records: cold too). A cold sweep after a hot
    // (static) one, whose deferred records sit in wave-owned positions, or one without a spill area runs the hot
    // instantiation (only two instantiations of the round loop: a third spilled registers at every key width).
    // `cold` is the table's counter encoding (lds_add_nr / slot_count) of the instantiation that ran.
    // (one- and two-word keys only: with three and four key words the dynamic instantiation spilled 20-40 VGPRs
    // and made k_count 10-22 % slower, against 2 % faster at k = 21 and 63)
    constexpr bool DYNS = NL <= DYN_SWEEP_MAX_NL;
    dyn_sweep = DYNS && has_spill && n < 0xC000u && (dyn_sweep || nw == NONE);
    const bool cold = DYNS ? dyn_sweep : n < 0xC000u;
    if constexpr (DYNS) {
      if (dyn_sweep)
        rounds(std::true_type{}, std::true_type{});
      else
        rounds(std::false_type{}, std::false_type{});
    } else {
      if (cold)
        rounds(std::true_type{}, std::false_type{});
      else
        rounds(std::false_type{}, std::false_type{});
    }
    STAMP(t_b0);
    __syncthreads();
    STAMP(t_f0);
    STAMP_ADD(3, t_f0 - t_b0);  // (the sweep's end barrier: the waves' imbalance; cold sweeps have no round barrier)
    // no deferred records: this is the bucket's last sweep, so start loading the next bucket now
    const bool last_sweep = s_ovf == 0;
    // what a next sweep of this bucket needs, read before the finalize resets the sweep's scalars
    const uint32_t n_def = s_ovf;
    const bool err_sw = s_err != 0;
    uint32_t nw_def = 0, mx_def = 0;
    if (!last_sweep) {
      nw_def = s_wdef[wid];
#pragma unroll
      for (int w = 0; w < C_THREADS / 64; w++) mx_def = mx_def > s_wdef[w] ? mx_def : s_wdef[w];
      // this wave's deferred records (global stores of the rounds) are released before the finalize's barriers; the
      // next sweep's loads acquire them after the last one
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
    }
    // (a skipped coarse bucket's fine buckets are empty, k_inc_fixup, and its contig k-mers wait for the launch
    // that counts it)
    if (p.ctg_n && !(p.coarse_skip && p.coarse_skip[b >> p.fine_bits])) ctg_apply<NL, CMP>(t, p, b, last_sweep, cold, s_red);
    {
      // the next bucket's first round, loaded while this one is finalized; unconditional (as the round prefetch:
      // a load under a branch was waited for at once): without a next bucket, or before a re-sweep (which loads
      // its own first round), it re-reads this bucket's first records, never used (cnt >= 1 keeps the read at
      // or next to the bucket's base, inside the records' allocation)
      const bool nxt = last_sweep && b_next < p.n_buckets;
      if (nxt) bucket_at(nx_base, nx_end, ps_next, nb_next);
      const bool use_next = nxt && nb_next;
      prefetch(use_next ? ps_next : ps, use_next ? nb_next : (n ? n : 1u), 0, NONE, (uint32_t)tid);
    }

    // finalize in two passes. 1: occupancy and count of every slot; the slots with count >= 2 (the only ones
    // that can survive) are listed in the miss-list space (free: phase B of the last round ended before the
    // barrier above). 2: the listed slots, dense over the lanes, get get_ext and the X/X purge. (One pass
    // took every lane through the whole decision for each of its 6 slots whether or not it was occupied.)
    uint16_t *flist = (uint16_t *)s_mkey;
    unsigned int *s_fin = (unsigned int *)(s_u64 + 3);  // [0] listed slots, [1] survivors (zeroed between buckets)
    uint32_t occ = 0;
    unsigned long long sum = 0;
    // pass 1 over quads of slots: an occupied slot has count >= 1 (every claim is followed by its add; a contig
    // entry's depth is >= 1) and a free one count 0, so the counters alone decide, read four slots at a time
    // (one ds_read_b128 per counter plane, consecutive lanes on consecutive quads: no bank conflicts)
    constexpr int QPT = (count_cap(NL, RK::C32) / 4 + C_THREADS - 1) / C_THREADS;
#pragma unroll
    for (int j = 0; j < QPT; j++) {
      const int qd = tid + j * C_THREADS;
      uint32_t c[4] = {0, 0, 0, 0};
      if (4 * qd < t.cap) {
        const uint4 c4 = *(const uint4 *)(t.cnt + 4 * qd);
        c[0] = c4.x, c[1] = c4.y, c[2] = c4.z, c[3] = c4.w;
        if (cold) {  // slot_count's cold encoding, four at a time
          const uint4 a4 = *(const uint4 *)(t.ext + 4 * qd), b4 = *(const uint4 *)(t.ext + t.cap + 4 * qd);
          const uint32_t a[4] = {a4.x, a4.y, a4.z, a4.w}, bb[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
          for (int i = 0; i < 4; i++)
            c[i] = (c[i] >> 31) ? c[i] & 0x7fffffffu
                                : c[i] + (a[i] & 0xffffu) + (a[i] >> 16) + (bb[i] & 0xffffu) + (bb[i] >> 16);
        }
      }
      // the wave's listed slots take one reservation (ballots + lane prefixes), not one LDS atomic each on the
      // same word
      uint64_t bal[4];
      uint32_t pre[4], tot = 0;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        occ += c[i] != 0u;
        sum += c[i];
        bal[i] = __ballot(c[i] >= 2);
        pre[i] = tot;
        tot += (uint32_t)__popcll(bal[i]);
      }
      if (tot) {
        uint32_t fb = 0;
        if (lane == 0) fb = atomicAdd(&s_fin[0], tot);
        fb = __builtin_amdgcn_readfirstlane(fb);
#pragma unroll
        for (int i = 0; i < 4; i++)
          if (c[i] >= 2)
            flist[fb + pre[i] + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal[i] >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)bal[i], 0u))] =
                (uint16_t)(4 * qd + i);
      }
    }
    __syncthreads();
    const uint32_t n_list = s_fin[0];
    // per listed slot of this thread: sp = slot | output position << 16 (both < 2^16), row = count | L << 16 | R << 24
    uint32_t surv_mask = 0, sp[SPT], row[SPT];
    // (uniform) the survivors' key words go to registers: the table may be cleared before the output is written
    const bool kfast = KREG && n_list <= (uint32_t)(KJ * C_THREADS);
    K kreg[KJ][NL];
#pragma unroll
    for (int j = 0; j < SPT; j++) {
      const uint32_t i = (uint32_t)tid + (uint32_t)j * C_THREADS;
      sp[j] = 0;
      row[j] = 0;
      bool sv = false;
      if (i < n_list) {
        const int slot = flist[i];
        sp[j] = (uint32_t)slot;
        uint16_t c16;
        char L, R_;
        const uint32_t cw = t.cnt[slot], e0 = t.ext[slot], e1 = t.ext[t.cap + slot], e2 = t.ext[2 * t.cap + slot],
                       e3 = t.ext[3 * t.cap + slot];
        if (KREG && j < KJ) {  // (with the counters: the same round trip)
#pragma unroll
          for (int w = 0; w < NL; w++) kreg[j < KJ ? j : 0][w] = t.keys[w * t.cap + slot];
        }
        // slot_count's cold encoding from the words already read
        const uint32_t c32 = !cold ? cw
                             : (cw >> 31) ? cw & 0x7fffffffu
                                          : cw + (e0 & 0xffffu) + (e0 >> 16) + (e1 & 0xffffu) + (e1 >> 16);
        sv = slot_survives(c32, e0, e1, e2, e3, p, c16, L, R_);
        row[j] = (uint32_t)c16 | (uint32_t)(uint8_t)L << 16 | (uint32_t)(uint8_t)R_ << 24;
      }
      // one reservation per wave for its survivors (ballot + lane prefix)
      const uint64_t bal = __ballot(sv);
      if (bal) {
        uint32_t sb = 0;
        if (lane == 0) sb = atomicAdd(&s_fin[1], (uint32_t)__popcll(bal));
        sb = __builtin_amdgcn_readfirstlane(sb);
        if (sv) {
          surv_mask |= 1u << j;
          sp[j] |= (sb + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u))) << 16;
        }
      }
    }
    const uint32_t mine = __popc(surv_mask);
    __syncthreads();
    // The survivors take one global reservation. With their key words in registers (kfast) the table is cleared for
    // the next sweep while it is in flight, and the output rows are written after one barrier with the next sweep's
    // rounds right behind them (two barriers fewer per bucket than clearing at the sweep's start).
    unsigned long long gret = 0;
    uint32_t acc = 0;
    if (tid == 0) {
      acc = s_fin[1];
      if (acc) gret = atomicAdd(p.out_cursor, (unsigned long long)acc);
    }
    STAMP(t_c0);
    if (kfast) clear_table();
    STAMP(t_c1);
    reset_sweep();  // (every thread read what it needs of the sweep's scalars above)
    if (tid == 0) {
      unsigned long long gb = gret;
      if (acc && gb + acc > p.out_cap) {  // the output is full: write nothing, flag the launch (the cursor still
        atomicOr(p.err, 16u);             // counts: the host grows the output to it and redoes the pass)
        gb = ~0ull;
      }
      s_gbase = gb;
      my_out += acc;
      s_fin[0] = 0;
      s_fin[1] = 0;
    }
    __syncthreads();
    if (s_gbase == ~0ull) surv_mask = 0;
#pragma unroll
    for (int j = 0; j < SPT; j++) {
      if ((surv_mask >> j) & 1u) {
        const int slot = (int)(sp[j] & 0xffffu);
        // the key words: from registers (kfast: every listed slot is one of a thread's first KJ) or from the table
        auto kw_of = [&](int w) -> K { return (KREG && j < KJ && kfast) ? kreg[j < KJ ? j : 0][w] : t.keys[w * t.cap + slot]; };
        const unsigned long long g = s_gbase + (sp[j] >> 16);
        uint64_t *ok = p.out_keys + g * (uint64_t)p.nlo;
        if (RK::C32) {  // key = cunmix(global fine bucket digits | stored bits)
          const int B = 2 * p.k, rb = B - p.coarse_bits - p.fine_bits;
          const uint64_t y = ((uint64_t)(p.bucket0 + b) << rb) | (kw_of(0) >> EXT_BITS);
          ok[0] = cunmix(y, B) << (64 - B);
        } else if (RK::M2) {  // key = m2_unmix(global fine bucket digits | stored L' bits, R')
          const int rb = p.k - p.coarse_bits - p.fine_bits;
          const uint64_t L = ((uint64_t)(p.bucket0 + b) << rb) | (kw_of(0) >> EXT_BITS);
          uint64_t kw[2];
          m2_unmix(L, kw_of(1), p.k, kw);
          ok[0] = kw[0];
          ok[1] = kw[1];
        } else if (RK::MX) {  // key = mx_unmix(global fine bucket digits | stored w0' bits, r[1..])
          const int rb = 64 - p.coarse_bits - p.fine_bits;
          uint64_t r[NL], kw[NL];
          r[0] = ((uint64_t)(p.bucket0 + b) << rb) | (kw_of(0) >> EXT_BITS);
#pragma unroll
          for (int w = 1; w < NL; w++) r[w] = kw_of(w);
          mx_unmix<NL>(r, kw);
#pragma unroll
          for (int w = 0; w < NL; w++) ok[w] = kw[w];
        } else {
#pragma unroll
          for (int w = 0; w < NL; w++) ok[w] = kw_of(w);
        }
        for (int w = NL; w < p.nlo; w++) ok[w] = 0;
        p.out_counts[g] = (uint16_t)row[j];
        p.out_left[g] = (char)(row[j] >> 16);
        p.out_right[g] = (char)(row[j] >> 24);
      }
    }
    my_occ += occ;
    my_purged += occ;  // minus the survivors, in 64 bits: with two passes a lane's survivors are not its slots
    my_purged -= mine;
    my_sum += sum;
    if (!kfast) {  // the output read the table: clear it after
      __syncthreads();
      clear_table();
      __syncthreads();
    }
    STAMP(t_f1);
    STAMP_ADD(0, t_c1 - t_c0);
    STAMP_ADD(5, t_f1 - t_f0 - (t_c1 - t_c0));
    if (err_sw && tid == 0) atomicAdd(&p.stats[STAT_N - 1], 1ull);
    if (last_sweep) break;
    n = n_def;
    lim = n;
    if (dyn_sweep) {  // the deferred records, dense in pd, are the next sweep's; the region it read takes its deferrals
      const Src t_ = ps;
      ps = pd;
      pd = t_;
      nw = NONE;
    } else {  // each wave re-reads its own deferred records; the rounds cover the largest share
      nw = nw_def;
      lim = (mx_def + (uint32_t)(64 * R) - 1) / (uint32_t)(64 * R) * RND;
    }
    my_sweeps++;
    // the deferred records of every wave (released before the finalize's barriers) are visible to this wave's loads
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
  }  // sweeps
  if (b_next >= p.n_buckets) break;
  b = b_next;  // (the finalize cleared the table for the next bucket)
  ps = ps_next;
  n = nb_next;
  pd = spill;
  dyn_sweep = false;
  }  // buckets

#if MHMKC_STAMP
  if (lane == 0)
    for (int i = 0; i < 6; i++) atomicAdd(&p.stats[8 + i], (unsigned long long)st_acc[i]);
  if (tid == 0) {  // the workgroup's cycles: sum and largest (the launch's tail)
    const uint64_t el = __builtin_amdgcn_s_memtime() - st_wg0;
    atomicAdd(&p.stats[14], (unsigned long long)el);
    atomicMax(&p.stats[15], (unsigned long long)el);
  }
#endif
  // block reduction of the statistics
  my_occ = wave_sum_u64(my_occ);
  my_purged = wave_sum_u64(my_purged);
  my_sum = wave_sum_u64(my_sum);
  if (tid == 0 && s_missacc) atomicAdd(&p.stats[STAT_MISSES], s_missacc);
  if (tid == 0) {
    s_red[0] = 0;
    s_red[1] = 0;
    s_red[2] = 0;
  }
  __syncthreads();
  if (lane == 0) {
    atomicAdd(&s_red[0], my_occ);
    atomicAdd(&s_red[1], my_purged);
    atomicAdd(&s_red[2], my_sum);
  }
  __syncthreads();
  if (tid == 0) {
    atomicAdd(&p.stats[STAT_DISTINCT], s_red[0]);
    atomicAdd(&p.stats[STAT_PURGED], s_red[1]);
    atomicAdd(&p.stats[STAT_COUNTSUM], s_red[2]);
    atomicAdd(&p.stats[STAT_NOUT], my_out);
    // sweep count and largest bucket are the same in every wave of the workgroup
    if (my_sweeps) atomicAdd(&p.stats[STAT_SWEEPS], my_sweeps);
    atomicMax(&p.stats[STAT_MAXBUCKET], my_maxb);
  }
}
#undef tid
#undef lane
#undef wid

// ------------------------------------------------------------------------------------------------
// launchers

#define MHM_DISPATCH(nl, packed, FN, ARGS)   \
  switch ((nl) * 2 + ((packed) ? 1 : 0)) {   \
    case 2: return FN<1, false> ARGS;        \
    case 3: return FN<1, true> ARGS;         \
    case 4: return FN<2, false> ARGS;        \
    case 5: return FN<2, true> ARGS;         \
    case 6: return FN<3, false> ARGS;        \
    case 7: return FN<3, true> ARGS;         \
    case 8: return FN<4, false> ARGS;        \
    case 9: return FN<4, true> ARGS;         \
    default: return hipErrorInvalidValue;    \
  }
// mixed records (compact, two-, three- and four-word): <NL, packed, mixed>
#define MHM_DISPATCH_MIXED(nl, FN, ARGS)                                                                \
  ((nl) == 1 ? FN<1, true, true> ARGS : (nl) == 2 ? FN<2, true, true> ARGS : (nl) == 3 ? FN<3, true, true> ARGS \
             : (nl) == 4 ? FN<4, true, true> ARGS : hipErrorInvalidValue)

template <typename K>
static hipError_t allow_lds(K kernel, size_t lds) {
  if (lds <= 65536) return hipSuccess;
  return hipFuncSetAttribute((const void *)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}

// CMP: compact records (NL = 1, packed), selected by the params' compact flag
template <int NL, bool PK, bool CMP = false>
static hipError_t do_extract_hist(const ExtractParams &p, hipStream_t s) {
  const size_t lds = tile_lds_bytes<NL>() + (size_t)p.n_bins * 4;
  hipError_t e = allow_lds(k_extract_hist<NL, PK, CMP>, lds);
  if (e != hipSuccess) return e;
  k_extract_hist<NL, PK, CMP><<<dim3(p.n_tiles), dim3(kEThreads<NL>()), lds, s>>>(p);
  return hipGetLastError();
}

template <int NL, bool PK, bool CMP = false>
static hipError_t do_extract_scatter(const ExtractParams &p, hipStream_t s) {
  const size_t lds = staged_cnt_bytes(p.n_bins) +
                     std::max(tile_lds_bytes<NL>(),
                              staged_area_bytes(NL, kECap<NL>(), PK, RecKind<NL, CMP>::C32 ? SF_C40 : SF_WORDS));
  if (p.n_bins <= (uint32_t)kEThreads<NL>()) {  // one coarse bin per thread (one rank: 256 bins), see do_part_scatter
    hipError_t e = allow_lds(k_extract_scatter<NL, PK, CMP, 1>, lds);
    if (e != hipSuccess) return e;
    k_extract_scatter<NL, PK, CMP, 1><<<dim3(p.n_tiles), dim3(kEThreads<NL>()), lds, s>>>(p);
    return hipGetLastError();
  }
  hipError_t e = allow_lds(k_extract_scatter<NL, PK, CMP>, lds);
  if (e != hipSuccess) return e;
  k_extract_scatter<NL, PK, CMP><<<dim3(p.n_tiles), dim3(kEThreads<NL>()), lds, s>>>(p);
  return hipGetLastError();
}

template <int NL, bool PK, bool CMP = false>
static hipError_t do_part_hist(const PartitionParams &p, hipStream_t s) {
  const size_t lds = ((size_t)1 << p.fine_bits) * 4;
  hipError_t e = allow_lds(k_part_hist<NL, PK, CMP>, lds);
  if (e != hipSuccess) return e;
  k_part_hist<NL, PK, CMP><<<dim3(p.grid), dim3(kPThreads<NL>()), lds, s>>>(p);
  return hipGetLastError();
}

template <int NL, bool PK, bool CMP = false>
static hipError_t do_part_scatter(const PartitionParams &p, hipStream_t s) {
  const uint32_t nf = 1u << p.fine_bits;
  const size_t lds = staged_cnt_bytes(nf) + staged_area_bytes(NL, kPTile<NL>(), PK, RecKind<NL, CMP>::C32 ? SF_C32 : SF_WORDS);
  // one fine bin per thread when the launch has no more, not the eight of the most (the bin registers: five
  // workgroups per CU at k = 21, part_scatter 2.64 -> 2.45 ms; two bins per thread at k = 63 measured 5.46 -> 5.55)
  if (nf <= (uint32_t)kPThreads<NL>()) {
    hipError_t e = allow_lds(k_part_scatter<NL, PK, CMP, 1>, lds);
    if (e != hipSuccess) return e;
    k_part_scatter<NL, PK, CMP, 1><<<dim3(p.grid), dim3(kPThreads<NL>()), lds, s>>>(p);
    return hipGetLastError();
  }
  hipError_t e = allow_lds(k_part_scatter<NL, PK, CMP>, lds);
  if (e != hipSuccess) return e;
  k_part_scatter<NL, PK, CMP><<<dim3(p.grid), dim3(kPThreads<NL>()), lds, s>>>(p);
  return hipGetLastError();
}

template <int NL, bool PK, bool CMP = false>
static hipError_t do_count(const CountParams &p, hipStream_t s) {
  const size_t lds = count_lds_bytes(NL, RecKind<NL, CMP>::C32);
  hipError_t e = allow_lds(k_count<NL, PK, CMP>, lds);
  if (e != hipSuccess) return e;
  const uint32_t grid = p.grid && p.grid < p.n_buckets ? p.grid : p.n_buckets;
  k_count<NL, PK, CMP><<<dim3(grid), dim3(C_THREADS), lds, s>>>(p);
  return hipGetLastError();
}

hipError_t launch_tile_first_read(const ReadsView &r, uint32_t *out, uint32_t n_tiles, int tile, hipStream_t s) {
  if (!n_tiles) return hipSuccess;
  k_tile_first_read<<<dim3((n_tiles + 255) / 256), dim3(256), 0, s>>>(r, out, n_tiles, tile);
  return hipGetLastError();
}

uint64_t read_start_words(uint64_t n_tiles, int nl) {
  const uint64_t T = nl == 1 ? kTile<1>() : nl == 2 ? kTile<2>() : nl == 3 ? kTile<3>() : kTile<4>();
  const uint64_t NG = nl == 1 ? kGroups<1>() : nl == 2 ? kGroups<2>() : nl == 3 ? kGroups<3>() : kGroups<4>();
  return n_tiles * (T / 32) + NG + 2;
}

hipError_t launch_read_start_bits(const ReadsView &r, uint32_t *bits, uint64_t n_words, hipStream_t s) {
  const uint64_t blocks = std::min<uint64_t>(8192, (r.n_reads + 1 + 255) / 256);
  k_read_start_bits<<<dim3((unsigned)blocks), dim3(256), 0, s>>>(r, bits, n_words);
  return hipGetLastError();
}

hipError_t launch_count_windows(const ReadsView &r, int k, unsigned long long *out, unsigned int *err, hipStream_t s) {
  if (!r.n_reads) return hipSuccess;
  const uint64_t blocks = std::min<uint64_t>(2048, (r.n_reads + 1023) / 1024);
  k_count_windows<<<dim3((unsigned)blocks), dim3(256), 0, s>>>(r, k, out, err);
  return hipGetLastError();
}

hipError_t launch_offs_from_deltas(const uint32_t *d, uint64_t *offs, uint64_t n, uint64_t b0, hipStream_t s) {
  if (!n) return hipSuccess;
  k_offs_from_deltas<<<dim3((unsigned)std::min<uint64_t>(4096, (n + 255) / 256)), dim3(256), 0, s>>>(d, offs, n, b0);
  return hipGetLastError();
}

hipError_t launch_expand_nibbles(const uint8_t *nib, uint8_t *arena, uint64_t b0, uint64_t n, hipStream_t s) {
  if (!n) return hipSuccess;
  const uint64_t blocks16 = (b0 + n - (b0 & ~15ull) + 15) / 16;
  k_expand_nibbles<<<dim3((unsigned)((blocks16 + 255) / 256)), dim3(256), 0, s>>>(nib, arena, b0, n);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_inc_fixup(const unsigned long long *coarse_base,
                                                  const unsigned long long *coarse_fcap, int fine_bits,
                                                  unsigned long long *cursor, uint8_t *skip, unsigned int *err) {
  const uint32_t c = blockIdx.x, nf = 1u << fine_bits;
  const unsigned long long b0 = coarse_base[c], fcap = coarse_fcap[c];
  unsigned long long *cur = cursor + ((uint64_t)c << fine_bits);
  int over = 0;
  for (uint32_t f = threadIdx.x; f < nf; f += 256) over |= cur[f] > b0 + (f + 1) * fcap;
  over = __syncthreads_or(over);
  if (over)
    for (uint32_t f = threadIdx.x; f < nf; f += 256) cur[f] = b0 + f * fcap;
  if (threadIdx.x == 0) {
    skip[c] = (uint8_t)over;
    if (c == 0) atomicAnd(err, ~2u);
  }
}

hipError_t launch_inc_fixup(const unsigned long long *coarse_base, const unsigned long long *coarse_fcap,
                            uint32_t n_coarse, int fine_bits, unsigned long long *cursor, uint8_t *skip,
                            unsigned int *err, hipStream_t s) {
  if (!n_coarse) return hipSuccess;
  k_inc_fixup<<<dim3(n_coarse), dim3(256), 0, s>>>(coarse_base, coarse_fcap, fine_bits, cursor, skip, err);
  return hipGetLastError();
}

hipError_t launch_init_fine(const unsigned long long *coarse_base, const unsigned long long *coarse_fcap,
                            uint32_t n_coarse, int fine_bits, unsigned long long *base, unsigned long long *cursor,
                            hipStream_t s) {
  const uint64_t n = (uint64_t)n_coarse << fine_bits;
  if (!n) return hipSuccess;
  k_init_fine<<<dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s>>>(coarse_base, coarse_fcap, n_coarse, fine_bits,
                                                                      base, cursor);
  return hipGetLastError();
}

hipError_t launch_extract_hist(const ExtractParams &p, int nl, bool packed, hipStream_t s) {
  if (!p.n_tiles) return hipSuccess;
  if (p.compact) return MHM_DISPATCH_MIXED(nl, do_extract_hist, (p, s));
  MHM_DISPATCH(nl, packed, do_extract_hist, (p, s));
}

hipError_t launch_extract_scatter(const ExtractParams &p, int nl, bool packed, hipStream_t s) {
  if (!p.n_tiles) return hipSuccess;
  if (p.compact) return MHM_DISPATCH_MIXED(nl, do_extract_scatter, (p, s));
  MHM_DISPATCH(nl, packed, do_extract_scatter, (p, s));
}

hipError_t launch_part_hist(const PartitionParams &p, int nl, bool packed, hipStream_t s) {
  if (!p.n_chunks) return hipSuccess;
  if (p.compact) return MHM_DISPATCH_MIXED(nl, do_part_hist, (p, s));
  MHM_DISPATCH(nl, packed, do_part_hist, (p, s));
}

hipError_t launch_part_scatter(const PartitionParams &p, int nl, bool packed, hipStream_t s) {
  if (!p.n_chunks) return hipSuccess;
  if (p.compact) return MHM_DISPATCH_MIXED(nl, do_part_scatter, (p, s));
  MHM_DISPATCH(nl, packed, do_part_scatter, (p, s));
}

hipError_t launch_chunk_runs(const SRun *runs, uint32_t n_runs, SChunk *chunks, int tile, hipStream_t s) {
  if (!n_runs) return hipSuccess;
  k_chunk_runs<<<dim3(n_runs), dim3(256), 0, s>>>(runs, chunks, tile);
  return hipGetLastError();
}

template <int NL, bool PK, bool CMP = false>
static hipError_t do_sketch(const PartitionParams &p, uint32_t n, unsigned int *hll, bool fh, hipStream_t s) {
  k_sketch<NL, PK, CMP><<<dim3(n), dim3(kPThreads<NL>()), 0, s>>>(p, hll, fh ? hll + SKETCH_WORDS : nullptr);
  return hipGetLastError();
}

hipError_t launch_sketch(const PartitionParams &p, uint32_t n_chunks, unsigned int *hll, int nl, bool packed,
                         hipStream_t s, bool fine_hist) {
  if (!n_chunks) return hipSuccess;
  if (fine_hist && p.fine_bits != SKETCH_FB) return hipErrorInvalidValue;
  if (p.compact) return MHM_DISPATCH_MIXED(nl, do_sketch, (p, n_chunks, hll, fine_hist, s));
  MHM_DISPATCH(nl, packed, do_sketch, (p, n_chunks, hll, fine_hist, s));
}

hipError_t launch_scan(const unsigned long long *in, unsigned long long *base, unsigned long long *cursor, uint32_t n,
                       hipStream_t s) {
  k_scan<<<dim3(1), dim3(1024), 0, s>>>(in, base, cursor, n);
  return hipGetLastError();
}

hipError_t launch_count(const CountParams &p, int nl, bool packed, hipStream_t s) {
  if (!p.n_buckets) return hipSuccess;
  if (p.compact) return MHM_DISPATCH_MIXED(nl, do_count, (p, s));
  MHM_DISPATCH(nl, packed, do_count, (p, s));
}

// ------------------------------------------------------------------------------------------------
// exchange: dense send planes (one workgroup per filled segment; consecutive lanes copy consecutive elements)

template <typename V>
__global__ __launch_bounds__(256) void k_seg_gather(const SegCopy *segs, const V *src, V *dst) {
  const SegCopy sc = segs[blockIdx.x];
  const V *s = src + sc.src;
  V *d = dst + sc.dst;
  for (uint64_t i = threadIdx.x; i < sc.n; i += 256) d[i] = s[i];
}

hipError_t launch_seg_gather(const SegCopy *segs, uint32_t n_segs, const void *src, void *dst, int elem_bytes,
                             hipStream_t s) {
  if (!n_segs) return hipSuccess;
  const dim3 grid(n_segs), block(256);
  switch (elem_bytes) {
    case 1: k_seg_gather<uint8_t><<<grid, block, 0, s>>>(segs, (const uint8_t *)src, (uint8_t *)dst); break;
    case 4: k_seg_gather<uint32_t><<<grid, block, 0, s>>>(segs, (const uint32_t *)src, (uint32_t *)dst); break;
    case 8: k_seg_gather<uint2><<<grid, block, 0, s>>>(segs, (const uint2 *)src, (uint2 *)dst); break;
    case 16: k_seg_gather<uint4><<<grid, block, 0, s>>>(segs, (const uint4 *)src, (uint4 *)dst); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// supermer exchange launchers (NL >= 2)

template <int NL>
static hipError_t do_smer_owner(const SmerParams &p, hipStream_t s) {
  const size_t lds = smer_owner_lds<NL>(p.n_ranks);
  hipError_t e = allow_lds(k_smer_owner<NL>, lds);
  if (e != hipSuccess) return e;
  k_smer_owner<NL><<<dim3(p.n_tiles), dim3(kEThreads<NL>()), lds, s>>>(p);
  return hipGetLastError();
}

template <int NL>
static hipError_t do_smer_pack(const SmerParams &p, hipStream_t s) {
  const size_t lds = smer_pack_lds<NL>(p.n_ranks);
  hipError_t e = allow_lds(k_smer_pack<NL>, lds);
  if (e != hipSuccess) return e;
  k_smer_pack<NL><<<dim3(p.n_tiles), dim3(kEThreads<NL>()), lds, s>>>(p);
  return hipGetLastError();
}

hipError_t launch_smer_owner(const SmerParams &p, int nl, hipStream_t s) {
  if (!p.n_tiles) return hipSuccess;
  if (p.n_ranks < 2 || p.n_ranks > 255 || p.m < 1 || p.m > 28 || p.m > p.k) return hipErrorInvalidValue;
  switch (nl) {
    case 2: return do_smer_owner<2>(p, s);
    case 3: return do_smer_owner<3>(p, s);
    case 4: return do_smer_owner<4>(p, s);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_smer_pack(const SmerParams &p, int nl, hipStream_t s) {
  if (!p.n_tiles) return hipSuccess;
  if (p.n_ranks < 2 || p.n_ranks > 255) return hipErrorInvalidValue;
  switch (nl) {
    case 2: return do_smer_pack<2>(p, s);
    case 3: return do_smer_pack<3>(p, s);
    case 4: return do_smer_pack<4>(p, s);
  }
  return hipErrorInvalidValue;
}

template <int NL, bool PK, bool CMP, bool HIST>
static hipError_t do_smer_extract(const ExtractParams &p, const SmerSource &src, hipStream_t s) {
  constexpr int T = kTile<NL>();
  constexpr int SF = RecKind<NL, CMP>::M2 ? SF_AOS2 : SF_WORDS;
  const size_t lds = HIST ? (size_t)p.n_bins * 4 : staged_cnt_bytes(p.n_bins) + staged_area_bytes(NL, T, PK, SF);
  hipError_t e = allow_lds(k_smer_extract<NL, PK, CMP, HIST>, lds);
  if (e != hipSuccess) return e;
  k_smer_extract<NL, PK, CMP, HIST><<<dim3(p.n_tiles), dim3(kEThreads<NL>()), lds, s>>>(p, src);
  return hipGetLastError();
}

template <bool HIST>
static hipError_t smer_extract_nl(const ExtractParams &p, const SmerSource &src, int nl, bool packed, hipStream_t s) {
  if (p.compact)
    return nl == 2 ? do_smer_extract<2, true, true, HIST>(p, src, s) : nl == 3 ? do_smer_extract<3, true, true, HIST>(p, src, s)
         : nl == 4 ? do_smer_extract<4, true, true, HIST>(p, src, s) : hipErrorInvalidValue;
  switch (nl * 2 + (packed ? 1 : 0)) {
    case 4: return do_smer_extract<2, false, false, HIST>(p, src, s);
    case 5: return do_smer_extract<2, true, false, HIST>(p, src, s);
    case 6: return do_smer_extract<3, false, false, HIST>(p, src, s);
    case 7: return do_smer_extract<3, true, false, HIST>(p, src, s);
    case 8: return do_smer_extract<4, false, false, HIST>(p, src, s);
    case 9: return do_smer_extract<4, true, false, HIST>(p, src, s);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_smer_extract(const ExtractParams &p, const SmerSource &src, int nl, bool packed, bool hist,
                               hipStream_t s) {
  if (!p.n_tiles) return hipSuccess;
  return hist ? smer_extract_nl<true>(p, src, nl, packed, s) : smer_extract_nl<false>(p, src, nl, packed, s);
}

hipError_t launch_smer_rebase(uint64_t *desc, uint64_t n, uint64_t delta, unsigned long long *nwin, hipStream_t s) {
  if (!n) return hipSuccess;
  k_smer_rebase<<<dim3((unsigned)std::min<uint64_t>(4096, (n + 255) / 256)), dim3(256), 0, s>>>(desc, n, delta, nwin);
  return hipGetLastError();
}

hipError_t launch_smer_tiles(const uint64_t *wpre, uint64_t n_smer, uint64_t *tile_first, uint32_t n_tiles, int tile,
                             hipStream_t s) {
  if (!n_smer) return hipSuccess;
  k_smer_tiles<<<dim3((n_tiles + 1 + 255) / 256), dim3(256), 0, s>>>(wpre, n_smer, tile_first, n_tiles, tile);
  return hipGetLastError();
}

}  // namespace mhm
