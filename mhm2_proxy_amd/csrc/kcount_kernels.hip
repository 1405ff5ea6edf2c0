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

#include "kcount_launch.hpp"
#include "kmer_ops.hpp"

namespace mhm {

template <int NL>
constexpr int kTile() {
  return NL <= 2 ? 4096 : 2048;
}
template <int NL>
constexpr int kGroups() {
  return kTile<NL>() / 32 + NL + 2;
}

constexpr size_t WSUM_BYTES = 64;  // block-scan scratch at the start of the scatter region

constexpr size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

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
                          uint32_t *good, uint32_t *start, unsigned int *err) {
  constexpr int T = kTile<NL>(), NG = kGroups<NL>();
  const int64_t gA = (int64_t)tile * (T / 32) - 1;
  for (int g = threadIdx.x; g < NG; g += blockDim.x) {
    const int64_t gi = gA + g;
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
      uint32_t bad = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) {
#pragma unroll
        for (int bj = 0; bj < 4; bj++) {
          const int j = 4 * i + bj;
          const uint32_t byte = (wv[i] >> (8 * bj)) & 0xffu;
          const uint32_t c = byte & 7u, q = byte >> 3;
          const uint32_t code = (c == 4u) ? 2u : (c & 3u);
          bad |= (c > 4u) & ((uint64_t)j < rem);
          f |= (uint64_t)code << (62 - 2 * j);
          gd |= (uint32_t)((q >= (uint32_t)qcut) & (c < 4u)) << (31 - j);
        }
      }
      if (bad) atomicOr(err, 1u);
    }
    fwd[g] = f;
    good[g] = gd;
    start[g] = 0;
  }
  __syncthreads();
  const int64_t lo = gA * 32, hi = (gA + NG) * 32;
  for (uint64_t r = (uint64_t)first_read + threadIdx.x; r <= rv.n_reads; r += blockDim.x) {
    const int64_t s = (int64_t)rv.offs[r];
    if (s >= hi) break;
    if (s >= lo) {
      const int64_t d = s - lo;
      atomicOr(&start[d >> 5], 1u << (31 - (d & 31)));
    }
  }
  __syncthreads();
}

// Build the record of the window starting at global base p (tile-local position lp).
// Valid iff the window and both neighbours lie in one read: the interior windows i in [1, L-k-1]
// of get_kmers_and_exts (src/kcount/kcount_cpu.cpp:316-334); at one rank the supermer is the read
// (kcount_cpu.cpp:84-101). Canonical = min(fwd, revcomp) (kcount_cpu.cpp:326-332);
// extensions are the neighbour bases, '0' (none) when low quality, complemented and swapped when the
// reverse complement is used (comp_nucleotide, src/utils.cpp:121-143).
template <int NL>
__device__ __forceinline__ bool make_record(const uint64_t *fwd, const uint32_t *good, const uint32_t *start,
                                            int lp, uint64_t p, uint64_t n_bases, int k, uint64_t *key,
                                            uint32_t &e) {
  if (p + (uint64_t)k >= n_bases) return false;
  {
    const int a = lp, b = lp + k;
    const int ga = a >> 5, gb = b >> 5;
    for (int g = ga; g <= gb; g++) {
      uint32_t m = ~0u;
      if (g == ga) m &= ~0u >> (a & 31);
      if (g == gb) m &= ~0u << (31 - (b & 31));
      if (start[g] & m) return false;
    }
  }
  uint64_t fw[NL];
#pragma unroll
  for (int m = 0; m < NL; m++) {
    const int pos = lp + 32 * m;
    const int g = pos >> 5, s = (pos & 31) * 2;
    uint64_t v = fwd[g];
    if (s) v = (v << s) | (fwd[g + 1] >> (64 - s));
    fw[m] = v;
  }
  fw[NL - 1] &= top_mask(k - 32 * (NL - 1));
  uint64_t rc[NL];
  revcomp<NL>(fw, rc, k);
  int l, r;
  {
    const int q = lp - 1, g = q >> 5, j = q & 31;
    const int code = (int)((fwd[g] >> (62 - 2 * j)) & 3u);
    l = ((good[g] >> (31 - j)) & 1u) ? code : EXT_NONE;
  }
  {
    const int q = lp + k, g = q >> 5, j = q & 31;
    const int code = (int)((fwd[g] >> (62 - 2 * j)) & 3u);
    r = ((good[g] >> (31 - j)) & 1u) ? code : EXT_NONE;
  }
  if (kmer_less<NL>(rc, fw)) {
#pragma unroll
    for (int m = 0; m < NL; m++) key[m] = rc[m];
    const int nl_ = (r == EXT_NONE) ? EXT_NONE : 3 - r;
    const int nr_ = (l == EXT_NONE) ? EXT_NONE : 3 - l;
    l = nl_;
    r = nr_;
  } else {
#pragma unroll
    for (int m = 0; m < NL; m++) key[m] = fw[m];
  }
  e = (uint32_t)((l << 3) | r);
  return true;
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
    if (rv.offs[m] < lo)
      a = m + 1;
    else
      b = m;
  }
  out[t] = (uint32_t)a;
}

// ------------------------------------------------------------------------------------------------
// extract: histogram

template <int NL, bool PACKED>
__global__ __launch_bounds__(E_THREADS) void k_extract_hist(ExtractParams p) {
  constexpr int T = kTile<NL>(), W = T / E_THREADS;
  extern __shared__ __align__(16) unsigned char smem[];
  uint64_t *fwd;
  uint32_t *good, *start;
  unsigned char *rest = carve_tile<NL>(smem, fwd, good, start);
  uint32_t *hist = (uint32_t *)rest;
  for (uint32_t b = threadIdx.x; b < p.n_bins; b += E_THREADS) hist[b] = 0;
  const uint32_t tile = blockIdx.x;
  load_tile<NL>(p.reads, tile, p.tile_first_read[tile], p.qual_cutoff, fwd, good, start, p.err);
  const uint64_t p0 = (uint64_t)tile * T;
  const int sh = 64 - p.coarse_bits;
#pragma unroll 2
  for (int j = 0; j < W; j++) {
    const int lt = threadIdx.x + j * E_THREADS;
    uint64_t key[NL];
    uint32_t e;
    if (make_record<NL>(fwd, good, start, lt + 32, p0 + lt, p.reads.n_bases, p.k, key, e)) {
      const uint64_t h = murmur3_h1<NL>(key);
      atomicAdd(&hist[(uint32_t)(h >> sh)], 1u);
    }
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < p.n_bins; b += E_THREADS) {
    const uint32_t c = hist[b];
    if (c) atomicAdd(&p.hist[b], (unsigned long long)c);
  }
}

// ------------------------------------------------------------------------------------------------
// LDS-staged scatter shared by extract_scatter and part_scatter.
// Records are first staged in arrival order (raw[w][i], inf[i] = valid<<31 | e<<16 | digit), then
// ranked per bin through a permutation so that each bin's run is written with consecutive lanes.
// Dynamic LDS layout of the scatter region (all offsets multiples of 16):
//   wsum[16] u32 | lcnt[nb] u32 | lpre[nb] u32 | goff[nb] u64 | raw[NL][T] u64 | inf[T] u32 | perm[T] u16
template <int NL>
struct ScatterLds {
  uint32_t *wsum, *lcnt, *lpre;
  unsigned long long *goff;
  uint64_t *raw;
  uint32_t *inf;
  uint16_t *perm;
};

template <int NL>
__device__ __forceinline__ ScatterLds<NL> carve_scatter(unsigned char *smem, uint32_t nb) {
  constexpr int T = kTile<NL>();
  ScatterLds<NL> s;
  s.wsum = (uint32_t *)smem;
  s.lcnt = (uint32_t *)(smem + WSUM_BYTES);
  s.lpre = s.lcnt + nb;
  s.goff = (unsigned long long *)(s.lpre + nb);
  s.raw = (uint64_t *)(s.goff + nb);
  s.inf = (uint32_t *)(s.raw + NL * T);
  s.perm = (uint16_t *)(s.inf + T);
  return s;
}

// bins are powers of two >= 256, so every carve offset stays a multiple of 16
template <int NL>
__host__ __device__ constexpr size_t scatter_lds_bytes(uint32_t nb) {
  return WSUM_BYTES + (size_t)nb * 4 * 2 + (size_t)nb * 8 + (size_t)NL * kTile<NL>() * 8 + (size_t)kTile<NL>() * 4 +
         (size_t)kTile<NL>() * 2;
}

template <int NL>
__device__ __forceinline__ void scatter_clear(const ScatterLds<NL> &s, uint32_t nb) {
  for (uint32_t b = threadIdx.x; b < nb; b += E_THREADS) s.lcnt[b] = 0;
}

// Called after every thread has written its raw/inf entries and counted them into lcnt.
template <int NL, bool PACKED>
__device__ void scatter_from_raw(const ScatterLds<NL> &s, uint32_t nb, unsigned long long *cursor, const PlaneSet &out) {
  constexpr int T = kTile<NL>(), W = T / E_THREADS;
  const int tid = threadIdx.x;
  __syncthreads();
  for (uint32_t b = tid; b < nb; b += E_THREADS) {
    const uint32_t c = s.lcnt[b];
    s.goff[b] = c ? atomicAdd(&cursor[b], (unsigned long long)c) : 0ull;
    s.lpre[b] = c;
  }
  __syncthreads();
  const uint32_t total = block_excl_scan<E_THREADS>(s.lpre, (int)nb, s.wsum);
  for (uint32_t b = tid; b < nb; b += E_THREADS) s.lcnt[b] = 0;
  __syncthreads();
  for (int j = 0; j < W; j++) {
    const int i = tid + j * E_THREADS;
    const uint32_t inf = s.inf[i];
    if (inf >> 31) {
      const uint32_t d = inf & 0xffffu;
      s.perm[s.lpre[d] + atomicAdd(&s.lcnt[d], 1u)] = (uint16_t)i;
    }
  }
  __syncthreads();
  for (uint32_t i = tid; i < total; i += E_THREADS) {
    const uint32_t src = s.perm[i];
    const uint32_t inf = s.inf[src];
    const uint32_t d = inf & 0xffffu;
    const unsigned long long dst = s.goff[d] + (i - s.lpre[d]);
#pragma unroll
    for (int w = 0; w < NL; w++) out.w[w][dst] = s.raw[w * T + src];
    if (!PACKED) out.ext[dst] = (uint8_t)((inf >> 16) & 63u);
  }
}

// ------------------------------------------------------------------------------------------------
// extract: scatter into coarse buckets

template <int NL, bool PACKED>
__global__ __launch_bounds__(E_THREADS) void k_extract_scatter(ExtractParams p) {
  constexpr int T = kTile<NL>(), W = T / E_THREADS;
  extern __shared__ __align__(16) unsigned char smem0[];
  uint64_t *fwd;
  uint32_t *good, *start;
  const ScatterLds<NL> s = carve_scatter<NL>(carve_tile<NL>(smem0, fwd, good, start), p.n_bins);
  scatter_clear<NL>(s, p.n_bins);
  const uint32_t tile = blockIdx.x;
  load_tile<NL>(p.reads, tile, p.tile_first_read[tile], p.qual_cutoff, fwd, good, start, p.err);
  const uint64_t p0 = (uint64_t)tile * T;
  const int sh = 64 - p.coarse_bits;
  for (int j = 0; j < W; j++) {
    const int lt = threadIdx.x + j * E_THREADS;
    uint64_t key[NL];
    uint32_t e = 0, inf = 0;
    if (make_record<NL>(fwd, good, start, lt + 32, p0 + lt, p.reads.n_bases, p.k, key, e)) {
      const uint32_t d = (uint32_t)(murmur3_h1<NL>(key) >> sh);
      if (PACKED) key[NL - 1] |= e;
#pragma unroll
      for (int w = 0; w < NL; w++) s.raw[w * T + lt] = key[w];
      inf = (1u << 31) | (e << 16) | d;
      atomicAdd(&s.lcnt[d], 1u);
    }
    s.inf[lt] = inf;
  }
  scatter_from_raw<NL, PACKED>(s, p.n_bins, p.cursor, p.out);
}

// ------------------------------------------------------------------------------------------------
// partition coarse -> fine

// Load one record of a chunk and compute its fine digit (hash recomputed from the key).
template <int NL, bool PACKED>
__device__ __forceinline__ uint32_t chunk_record(const PlaneSet &src, uint64_t idx, int shf, uint64_t fmask,
                                                 uint64_t *rk, uint32_t &e) {
#pragma unroll
  for (int w = 0; w < NL; w++) rk[w] = src.w[w][idx];
  uint64_t key[NL];
#pragma unroll
  for (int w = 0; w < NL; w++) key[w] = rk[w];
  if (PACKED) {
    e = (uint32_t)(key[NL - 1] & 63u);
    key[NL - 1] &= ~63ull;
  } else {
    e = src.ext[idx];
  }
  return (uint32_t)((murmur3_h1<NL>(key) >> shf) & fmask);
}

template <int NL, bool PACKED>
__global__ __launch_bounds__(E_THREADS) void k_part_hist(PartitionParams p) {
  constexpr int T = kTile<NL>(), W = T / E_THREADS;
  extern __shared__ __align__(16) uint32_t hist[];  // the only LDS object
  const uint32_t nf = 1u << p.fine_bits;
  for (uint32_t b = threadIdx.x; b < nf; b += E_THREADS) hist[b] = 0;
  const SChunk ch = p.chunks[blockIdx.x];
  const PlaneSet src = p.srcs[ch.src];
  const int shf = 64 - p.coarse_bits - p.fine_bits;
  const uint64_t fmask = nf - 1;
  __syncthreads();
#pragma unroll 4
  for (int j = 0; j < W; j++) {
    const uint32_t i = threadIdx.x + j * E_THREADS;
    if (i < ch.count) {
      uint64_t rk[NL];
      uint32_t e;
      atomicAdd(&hist[chunk_record<NL, PACKED>(src, ch.start + i, shf, fmask, rk, e)], 1u);
    }
  }
  __syncthreads();
  unsigned long long *g = p.fine_hist + (uint64_t)ch.coarse_local * nf;
  for (uint32_t b = threadIdx.x; b < nf; b += E_THREADS) {
    const uint32_t c = hist[b];
    if (c) atomicAdd(&g[b], (unsigned long long)c);
  }
}

template <int NL, bool PACKED>
__global__ __launch_bounds__(E_THREADS) void k_part_scatter(PartitionParams p) {
  constexpr int T = kTile<NL>(), W = T / E_THREADS;
  extern __shared__ __align__(16) unsigned char smem[];
  const uint32_t nf = 1u << p.fine_bits;
  const ScatterLds<NL> s = carve_scatter<NL>(smem, nf);
  scatter_clear<NL>(s, nf);
  const SChunk ch = p.chunks[blockIdx.x];
  const PlaneSet src = p.srcs[ch.src];
  const int shf = 64 - p.coarse_bits - p.fine_bits;
  const uint64_t fmask = nf - 1;
  __syncthreads();
#pragma unroll 4
  for (int j = 0; j < W; j++) {
    const uint32_t i = threadIdx.x + j * E_THREADS;
    uint32_t inf = 0;
    if (i < ch.count) {
      uint64_t rk[NL];
      uint32_t e;
      const uint32_t d = chunk_record<NL, PACKED>(src, ch.start + i, shf, fmask, rk, e);
#pragma unroll
      for (int w = 0; w < NL; w++) s.raw[w * T + i] = rk[w];
      inf = (1u << 31) | (e << 16) | d;
      atomicAdd(&s.lcnt[d], 1u);
    }
    s.inf[i] = inf;
  }
  scatter_from_raw<NL, PACKED>(s, nf, p.fine_cursor + (uint64_t)ch.coarse_local * nf, p.out);
}

// ------------------------------------------------------------------------------------------------
// exclusive scan of bucket counts (one workgroup)

__global__ __launch_bounds__(1024) void k_scan(const unsigned long long *in, unsigned long long *base,
                                               unsigned long long *cursor, uint32_t n) {
  __shared__ unsigned long long wsum[17];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const uint32_t per = (n + 1023) / 1024;
  const uint32_t lo = min((uint32_t)tid * per, n), hi = min(lo + per, n);
  unsigned long long s = 0;
  for (uint32_t i = lo; i < hi; i++) s += in[i];
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
    run += in[i];
  }
}

// ------------------------------------------------------------------------------------------------
// count: LDS open-addressing hash table per fine bucket

struct CountLds {
  uint64_t *keys;  // [NL][cap]
  uint32_t *cnt;   // [cap]
  uint32_t *ext;   // [4][cap]: (A|C<<16, G|T<<16) left, then right
  int cap;
};

__device__ __forceinline__ bool reserve_slot(int *s_res, int *s_closed, int limit) {
  if (__hip_atomic_load(s_closed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return false;
  const int old = atomicAdd(s_res, 1);
  if (old >= limit) {
    __hip_atomic_store(s_closed, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return false;
  }
  return true;
}

// Returns the slot holding key (inserting it if allowed), -1 when the table is closed and the key
// is absent, -2 on an internal bound violation.
template <int NL>
__device__ int lds_insert_or_find(const CountLds &t, const uint64_t *key, int slot, int *s_res, int *s_closed,
                                  int limit) {
  uint64_t *last = t.keys + (NL - 1) * t.cap;
  for (int iter = 0; iter < (1 << 22); iter++) {
    const uint64_t cur = __hip_atomic_load(&last[slot], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (cur == KEY_EMPTY) {
      if (!reserve_slot(s_res, s_closed, limit)) return -1;
      const uint64_t want = (NL == 1) ? key[0] : KEY_BUSY;
      const uint64_t old = atomicCAS((unsigned long long *)&last[slot], (unsigned long long)KEY_EMPTY,
                                     (unsigned long long)want);
      if (old == KEY_EMPTY) {
        if (NL > 1) {
#pragma unroll
          for (int w = 0; w < NL - 1; w++) t.keys[w * t.cap + slot] = key[w];
          __hip_atomic_store(&last[slot], key[NL - 1], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        return slot;
      }
      atomicSub(s_res, 1);
      continue;  // re-examine the slot that was just taken
    }
    if (NL > 1 && cur == KEY_BUSY) continue;  // writer publishes within its own iteration
    if (cur == key[NL - 1]) {
      bool eq = true;
#pragma unroll
      for (int w = 0; w < NL - 1; w++) eq &= (t.keys[w * t.cap + slot] == key[w]);
      if (eq) return slot;
    }
    slot = (slot + 1 == t.cap) ? 0 : slot + 1;
  }
  return -2;
}

template <int NL>
__device__ int lds_find(const CountLds &t, const uint64_t *key, int slot) {
  const uint64_t *last = t.keys + (NL - 1) * t.cap;
  for (int iter = 0; iter < t.cap + 1; iter++) {
    const uint64_t cur = __hip_atomic_load(&last[slot], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (cur == KEY_EMPTY) return -1;
    if (cur == key[NL - 1]) {
      bool eq = true;
#pragma unroll
      for (int w = 0; w < NL - 1; w++) eq &= (t.keys[w * t.cap + slot] == key[w]);
      if (eq) return slot;
    }
    slot = (slot + 1 == t.cap) ? 0 : slot + 1;
  }
  return -1;
}

// Saturating-at-the-decision-level extension counter: 16-bit halves of a u32, incremented with one
// LDS atomic. A half that reaches 0xC000 is clamped back to 0x8000 by CAS. Exact for the reference's
// get_ext, which only compares counters against thresholds <= max(6553, dmin_thres) <= 32768
// (DESIGN.md §3.4); the reference saturates the same counters at 65535 (kcount_cpu.cpp:148-164).
__device__ __forceinline__ void ext_inc(uint32_t *p, int half) {
  const uint32_t inc = half ? 0x10000u : 1u;
  const uint32_t old = atomicAdd(p, inc);
  const uint32_t v = half ? (old >> 16) : (old & 0xffffu);
  if (v >= 0xC000u) {
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
}

// insert_supermer_from_read's per-k-mer update (src/kcount/kcount_cpu.cpp:343-352): count + 1,
// left/right extension + 1 when they are A/C/G/T.
__device__ __forceinline__ void lds_update(const CountLds &t, int slot, uint32_t e) {
  atomicAdd(&t.cnt[slot], 1u);
  const int l = (int)(e >> 3), r = (int)(e & 7u);
  if (l < 4) ext_inc(&t.ext[(l >> 1) * t.cap + slot], l & 1);
  if (r < 4) ext_inc(&t.ext[(2 + (r >> 1)) * t.cap + slot], r & 1);
}

// Final decision for one table slot: insert_into_local_hashtable (src/kcount/kcount_cpu.cpp:503-517):
// count < 2 -> purged; left/right = get_ext(count) (kcount_cpu.cpp:173-182, with the exact double
// expression of the dynamic threshold); both 'X' -> purged.
__device__ __forceinline__ bool slot_survives(const CountLds &t, int slot, const CountParams &p, uint16_t &c16,
                                              char &L, char &R) {
  const uint32_t c32 = t.cnt[slot];
  const uint32_t c = c32 > 65535u ? 65535u : c32;
  c16 = (uint16_t)c;
  if (c < 2) return false;
  const int thr = dyn_threshold(c, p.dyn_mult, p.dmin_thres);
  const uint32_t e0 = t.ext[slot], e1 = t.ext[t.cap + slot];
  const uint32_t e2 = t.ext[2 * t.cap + slot], e3 = t.ext[3 * t.cap + slot];
  L = ext_choice(e0 & 0xffffu, e0 >> 16, e1 & 0xffffu, e1 >> 16, thr);
  R = ext_choice(e2 & 0xffffu, e2 >> 16, e3 & 0xffffu, e3 >> 16, thr);
  return !(L == 'X' && R == 'X');
}

template <int NL, bool PACKED>
__device__ __forceinline__ void load_record(const PlaneSet &ps, uint64_t idx, uint64_t *key, uint32_t &e) {
#pragma unroll
  for (int w = 0; w < NL; w++) key[w] = ps.w[w][idx];
  if (PACKED) {
    e = (uint32_t)(key[NL - 1] & 63u);
    key[NL - 1] &= ~63ull;
  } else {
    e = ps.ext[idx];
  }
}

template <int NL, bool PACKED>
__device__ __forceinline__ void store_record(const PlaneSet &ps, uint64_t idx, const uint64_t *key, uint32_t e) {
#pragma unroll
  for (int w = 0; w < NL; w++) ps.w[w][idx] = (w == NL - 1 && PACKED) ? (key[w] | e) : key[w];
  if (!PACKED) ps.ext[idx] = (uint8_t)e;
}

template <int NL, bool PACKED>
__global__ __launch_bounds__(C_THREADS) void k_count(CountParams p) {
  extern __shared__ __align__(16) unsigned char smem[];
  CountLds t;
  t.cap = p.cap;
  t.keys = (uint64_t *)smem;
  t.cnt = (uint32_t *)(t.keys + NL * t.cap);
  t.ext = t.cnt + t.cap;
  // scalars live after the table in the same dynamic region (count_lds_bytes adds 64 bytes)
  unsigned long long *s_u64 = (unsigned long long *)(t.ext + 4 * t.cap);
  unsigned long long &s_gbase = s_u64[0];
  unsigned long long *s_red = s_u64 + 1;  // [3]
  int &s_res = *(int *)(s_u64 + 4);
  int &s_closed = *((int *)(s_u64 + 4) + 1);
  unsigned int &s_ovf = *(unsigned int *)(s_u64 + 5);
  unsigned int &s_nsurv = *((unsigned int *)(s_u64 + 5) + 1);
  unsigned int &s_wr = *(unsigned int *)(s_u64 + 6);
  unsigned int &s_err = *((unsigned int *)(s_u64 + 6) + 1);

  const int tid = threadIdx.x;
  const uint32_t b = blockIdx.x;
  uint64_t n = p.bucket_n[b];
  const uint64_t n0 = n;
  const uint64_t base = p.bucket_base[b];
  PlaneSet ps = p.recs;
#pragma unroll
  for (int w = 0; w < NL; w++) ps.w[w] += base;
  if (!PACKED) ps.ext += base;

  uint32_t sweeps = 0;
  unsigned long long my_occ = 0, my_purged = 0, my_sum = 0, my_out = 0;
  while (true) {
    for (int i = tid; i < t.cap; i += C_THREADS) {
      t.keys[(NL - 1) * t.cap + i] = KEY_EMPTY;
      t.cnt[i] = 0;
      t.ext[i] = 0;
      t.ext[t.cap + i] = 0;
      t.ext[2 * t.cap + i] = 0;
      t.ext[3 * t.cap + i] = 0;
    }
    if (tid == 0) {
      s_res = 0;
      s_closed = 0;
      s_ovf = 0;
      s_nsurv = 0;
      s_wr = 0;
      s_err = 0;
    }
    __syncthreads();

    uint64_t nk[NL];
    uint32_t ne = 0;
    bool nh = (uint64_t)tid < n;
    if (nh) load_record<NL, PACKED>(ps, tid, nk, ne);
    for (uint64_t r0 = 0; r0 < n; r0 += C_THREADS) {
      uint64_t key[NL];
#pragma unroll
      for (int w = 0; w < NL; w++) key[w] = nk[w];
      const uint32_t e = ne;
      const bool have = nh;
      const uint64_t nxt = r0 + C_THREADS + tid;
      nh = nxt < n;
      if (nh) load_record<NL, PACKED>(ps, nxt, nk, ne);
      int s0 = 0;
      bool tent = false;
      if (have) {
        const uint64_t h = murmur3_h1<NL>(key);
        s0 = (int)(((uint64_t)(uint32_t)h * (uint64_t)t.cap) >> 32);
        const int slot = lds_insert_or_find<NL>(t, key, s0, &s_res, &s_closed, p.limit);
        if (slot >= 0)
          lds_update(t, slot, e);
        else if (slot == -1)
          tent = true;
        else
          s_err = 1;
      }
      __syncthreads();
      if (tent) {
        // The table closed this round: keys inserted concurrently are visible now; a key still absent
        // is never inserted in this sweep, so all its occurrences go to the next sweep together.
        const int slot = lds_find<NL>(t, key, s0);
        if (slot >= 0) {
          lds_update(t, slot, e);
        } else {
          const unsigned int pos = atomicAdd(&s_ovf, 1u);
          store_record<NL, PACKED>(ps, pos, key, e);  // pos < r0 + C_THREADS: already consumed
        }
      }
    }
    __syncthreads();

    // finalize: survivors of this sweep -> output table
    uint32_t occ = 0, purged = 0, surv = 0;
    unsigned long long sum = 0;
    for (int slot = tid; slot < t.cap; slot += C_THREADS) {
      if (t.keys[(NL - 1) * t.cap + slot] != KEY_EMPTY) {
        occ++;
        sum += t.cnt[slot];
        uint16_t c16;
        char L, R;
        if (slot_survives(t, slot, p, c16, L, R))
          surv++;
        else
          purged++;
      }
    }
    surv = wave_sum_u32(surv);
    if ((tid & 63) == 0 && surv) atomicAdd(&s_nsurv, surv);
    __syncthreads();
    if (tid == 0) s_gbase = s_nsurv ? atomicAdd(p.out_cursor, (unsigned long long)s_nsurv) : 0ull;
    __syncthreads();
    for (int slot = tid; slot < t.cap; slot += C_THREADS) {
      if (t.keys[(NL - 1) * t.cap + slot] != KEY_EMPTY) {
        uint16_t c16;
        char L, R;
        if (slot_survives(t, slot, p, c16, L, R)) {
          const unsigned long long g = s_gbase + atomicAdd(&s_wr, 1u);
          uint64_t *ok = p.out_keys + g * (uint64_t)p.nlo;
#pragma unroll
          for (int w = 0; w < NL; w++) ok[w] = t.keys[w * t.cap + slot];
          for (int w = NL; w < p.nlo; w++) ok[w] = 0;
          p.out_counts[g] = c16;
          p.out_left[g] = L;
          p.out_right[g] = R;
        }
      }
    }
    my_occ += occ;
    my_purged += purged;
    my_sum += sum;
    if (tid == 0) my_out += s_nsurv;
    __syncthreads();
    if (s_err && tid == 0) atomicAdd(&p.stats[STAT_N - 1], 1ull);
    if (s_ovf == 0) break;
    n = s_ovf;
    sweeps++;
    // overflow records were written by this workgroup: make them visible to its own loads
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
    __syncthreads();
  }

  // block reduction of the statistics
  my_occ = wave_sum_u64(my_occ);
  my_purged = wave_sum_u64(my_purged);
  my_sum = wave_sum_u64(my_sum);
  if (tid == 0) {
    s_red[0] = 0;
    s_red[1] = 0;
    s_red[2] = 0;
  }
  __syncthreads();
  if ((tid & 63) == 0) {
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
    if (sweeps) atomicAdd(&p.stats[STAT_SWEEPS], (unsigned long long)sweeps);
    atomicMax(&p.stats[STAT_MAXBUCKET], (unsigned long long)n0);
  }
}

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

template <typename K>
static hipError_t allow_lds(K kernel, size_t lds) {
  if (lds <= 65536) return hipSuccess;
  return hipFuncSetAttribute((const void *)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}

template <int NL, bool PK>
static hipError_t do_extract_hist(const ExtractParams &p, hipStream_t s) {
  const size_t lds = tile_lds_bytes<NL>() + (size_t)p.n_bins * 4;
  hipError_t e = allow_lds(k_extract_hist<NL, PK>, lds);
  if (e != hipSuccess) return e;
  k_extract_hist<NL, PK><<<dim3(p.n_tiles), dim3(E_THREADS), lds, s>>>(p);
  return hipGetLastError();
}

template <int NL, bool PK>
static hipError_t do_extract_scatter(const ExtractParams &p, hipStream_t s) {
  const size_t lds = tile_lds_bytes<NL>() + scatter_lds_bytes<NL>(p.n_bins);
  hipError_t e = allow_lds(k_extract_scatter<NL, PK>, lds);
  if (e != hipSuccess) return e;
  k_extract_scatter<NL, PK><<<dim3(p.n_tiles), dim3(E_THREADS), lds, s>>>(p);
  return hipGetLastError();
}

template <int NL, bool PK>
static hipError_t do_part_hist(const PartitionParams &p, hipStream_t s) {
  const size_t lds = ((size_t)1 << p.fine_bits) * 4;
  hipError_t e = allow_lds(k_part_hist<NL, PK>, lds);
  if (e != hipSuccess) return e;
  k_part_hist<NL, PK><<<dim3(p.n_chunks), dim3(E_THREADS), lds, s>>>(p);
  return hipGetLastError();
}

template <int NL, bool PK>
static hipError_t do_part_scatter(const PartitionParams &p, hipStream_t s) {
  const size_t lds = scatter_lds_bytes<NL>(1u << p.fine_bits);
  hipError_t e = allow_lds(k_part_scatter<NL, PK>, lds);
  if (e != hipSuccess) return e;
  k_part_scatter<NL, PK><<<dim3(p.n_chunks), dim3(E_THREADS), lds, s>>>(p);
  return hipGetLastError();
}

template <int NL, bool PK>
static hipError_t do_count(const CountParams &p, hipStream_t s) {
  const size_t lds = count_lds_bytes(NL);
  hipError_t e = allow_lds(k_count<NL, PK>, lds);
  if (e != hipSuccess) return e;
  k_count<NL, PK><<<dim3(p.n_buckets), dim3(C_THREADS), lds, s>>>(p);
  return hipGetLastError();
}

hipError_t launch_tile_first_read(const ReadsView &r, uint32_t *out, uint32_t n_tiles, int tile, hipStream_t s) {
  if (!n_tiles) return hipSuccess;
  k_tile_first_read<<<dim3((n_tiles + 255) / 256), dim3(256), 0, s>>>(r, out, n_tiles, tile);
  return hipGetLastError();
}

hipError_t launch_extract_hist(const ExtractParams &p, int nl, bool packed, hipStream_t s) {
  if (!p.n_tiles) return hipSuccess;
  MHM_DISPATCH(nl, packed, do_extract_hist, (p, s));
}

hipError_t launch_extract_scatter(const ExtractParams &p, int nl, bool packed, hipStream_t s) {
  if (!p.n_tiles) return hipSuccess;
  MHM_DISPATCH(nl, packed, do_extract_scatter, (p, s));
}

hipError_t launch_part_hist(const PartitionParams &p, int nl, bool packed, hipStream_t s) {
  if (!p.n_chunks) return hipSuccess;
  MHM_DISPATCH(nl, packed, do_part_hist, (p, s));
}

hipError_t launch_part_scatter(const PartitionParams &p, int nl, bool packed, hipStream_t s) {
  if (!p.n_chunks) return hipSuccess;
  MHM_DISPATCH(nl, packed, do_part_scatter, (p, s));
}

hipError_t launch_scan(const unsigned long long *in, unsigned long long *base, unsigned long long *cursor, uint32_t n,
                       hipStream_t s) {
  k_scan<<<dim3(1), dim3(1024), 0, s>>>(in, base, cursor, n);
  return hipGetLastError();
}

hipError_t launch_count(const CountParams &p, int nl, bool packed, hipStream_t s) {
  if (!p.n_buckets) return hipSuccess;
  MHM_DISPATCH(nl, packed, do_count, (p, s));
}

}  // namespace mhm
