// Output hand-off to the reference's owner rank on gfx950.
//
// dbjg looks a k-mer up on rank get_kmer_target_rank(kmer) = minimizer_hash_fast(minimizer_len) % rank_n
// (src/kcount/kmer_dht.cpp:193-196; callers src/dbjg_traversal.cpp:232-234,264-274). The count itself is
// partitioned by hash range (kcount_kernels.hip); after finalize, mhmkc_finish moves every surviving k-mer to
// that owner when the handle asks for it (mhmkc_config.output_owner). These kernels compute the owner of
// each output row and group the rows by owner for the exchange.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>

#include "../../include/mhmkc.h"

#include "kcount_launch.hpp"
#include "kmer_ops.hpp"

namespace mhm {

namespace {

constexpr int O_THREADS = 256;

inline unsigned grid_for(uint64_t n) { return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(8192, (n + 255) / 256)); }

__global__ __launch_bounds__(O_THREADS) void k_minimizer_hash(const uint64_t *keys, uint64_t n, int nlo, int k, int m,
                                                              uint64_t *out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = quick_hash(minimizer_fast(keys + i * (uint64_t)nlo, k, m));
}

__global__ __launch_bounds__(O_THREADS) void k_owner_hist(const uint64_t *keys, uint64_t n, int nlo, int k, int m, int G,
                                                          uint8_t *dest, unsigned long long *hist) {
  __shared__ unsigned int lh[256];
  for (int i = threadIdx.x; i < G; i += blockDim.x) lh[i] = 0;
  __syncthreads();
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t d = (uint32_t)(quick_hash(minimizer_fast(keys + i * (uint64_t)nlo, k, m)) % (uint64_t)G);
    dest[i] = (uint8_t)d;
    atomicAdd(&lh[d], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < G; i += blockDim.x)
    if (lh[i]) atomicAdd(&hist[i], (unsigned long long)lh[i]);
}

// Rows grouped by owner. The order inside an owner's group is free (the reference's KmerMap order is
// unspecified): each workgroup reserves one run per owner with one atomic and ranks its rows in LDS.
__global__ __launch_bounds__(O_THREADS) void k_owner_scatter(OutRows in, uint64_t n, int nlo, const uint8_t *dest, int G,
                                                             unsigned long long *cursor, OutRows out) {
  __shared__ unsigned int lc[256];
  __shared__ unsigned long long lb[256];
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x; i0 < n; i0 += stride) {
    for (int i = threadIdx.x; i < G; i += blockDim.x) lc[i] = 0;
    __syncthreads();
    const uint64_t i = i0 + threadIdx.x;
    uint32_t d = 0, rk = 0;
    if (i < n) {
      d = dest[i];
      rk = atomicAdd(&lc[d], 1u);
    }
    __syncthreads();
    for (int j = threadIdx.x; j < G; j += blockDim.x) lb[j] = lc[j] ? atomicAdd(&cursor[j], (unsigned long long)lc[j]) : 0ull;
    __syncthreads();
    if (i < n) {
      const uint64_t o = lb[d] + rk;
      for (int w = 0; w < nlo; w++) out.keys[o * nlo + w] = in.keys[i * nlo + w];
      out.counts[o] = in.counts[i];
      out.left[o] = in.left[i];
      out.right[o] = in.right[i];
    }
    __syncthreads();
  }
}

// mhmkc_fetch_ordered: the top 32 bits of the KmerMap hash of every output row (mhmkc_map_hash, include/mhmkc.h) as
// the sort key, the row index as the value
__global__ __launch_bounds__(O_THREADS) void k_map_hash(const uint64_t *keys, uint64_t n, int nlo, uint32_t *hkey,
                                                        uint32_t *idx) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    hkey[i] = (uint32_t)(mhmkc_map_hash(keys + i * (uint64_t)nlo, nlo) >> 32);
    idx[i] = (uint32_t)i;
  }
}

__global__ __launch_bounds__(O_THREADS) void k_gather_rows(OutRows in, const uint32_t *idx, uint64_t n, int nlo, OutRows out) {
  for (uint64_t o = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; o < n; o += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = idx[o];
    for (int w = 0; w < nlo; w++) out.keys[o * nlo + w] = in.keys[i * nlo + w];
    out.counts[o] = in.counts[i];
    out.left[o] = in.left[i];
    out.right[o] = in.right[i];
  }
}

// mhmkc_fetch_ordered for keys of up to four words: every row packed into one record (key words, then count | left << 16
// | right << 24), sorted with its hash key, then unpacked: all streaming. (A sort of row indices followed by a gather
// from the four output planes fetched >= 21x the rows' bytes: four narrow random reads per row.)
template <int NLO>
struct PackedRow {
  uint64_t key[NLO];
  uint32_t meta, pad;
};

template <int NLO>
__global__ __launch_bounds__(O_THREADS) void k_pack_rows(OutRows in, uint64_t n, uint32_t *hkey, PackedRow<NLO> *rows) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    PackedRow<NLO> r;
#pragma unroll
    for (int w = 0; w < NLO; w++) r.key[w] = in.keys[i * NLO + w];
    r.meta = (uint32_t)in.counts[i] | (uint32_t)(uint8_t)in.left[i] << 16 | (uint32_t)(uint8_t)in.right[i] << 24;
    r.pad = 0;
    hkey[i] = (uint32_t)(mhmkc_map_hash(r.key, NLO) >> 32);
    rows[i] = r;
  }
}

template <int NLO>
__global__ __launch_bounds__(O_THREADS) void k_unpack_rows(const PackedRow<NLO> *rows, uint64_t n, OutRows out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const PackedRow<NLO> r = rows[i];
#pragma unroll
    for (int w = 0; w < NLO; w++) out.keys[i * NLO + w] = r.key[w];
    out.counts[i] = (uint16_t)r.meta;
    out.left[i] = (char)(r.meta >> 16);
    out.right[i] = (char)(r.meta >> 24);
  }
}

template <int NLO>
size_t packed_order_bytes(uint64_t n) {
  size_t t = 0;
  (void)rocprim::radix_sort_pairs(nullptr, t, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                  (const PackedRow<NLO> *)nullptr, (PackedRow<NLO> *)nullptr, (size_t)n);
  const size_t a = (n + 63) / 64 * 64;
  return 2 * a * 4 + 2 * a * sizeof(PackedRow<NLO>) + t + 512;
}

template <int NLO>
hipError_t packed_order(const OutRows &in, uint64_t n, void *scratch, size_t scratch_bytes, const OutRows &out,
                        hipStream_t s) {
  const size_t a = (n + 63) / 64 * 64;
  uint32_t *hk = (uint32_t *)scratch, *hk2 = hk + a;
  PackedRow<NLO> *rw = (PackedRow<NLO> *)(hk2 + a), *rw2 = rw + a;
  void *tmp = rw2 + a;
  size_t tb = scratch_bytes - (2 * a * 4 + 2 * a * sizeof(PackedRow<NLO>));
  k_pack_rows<NLO><<<grid_for(n), O_THREADS, 0, s>>>(in, n, hk, rw);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if ((e = rocprim::radix_sort_pairs(tmp, tb, hk, hk2, rw, rw2, (size_t)n, 0, 32, s)) != hipSuccess) return e;
  k_unpack_rows<NLO><<<grid_for(n), O_THREADS, 0, s>>>(rw2, n, out);
  return hipGetLastError();
}

// mhmkc_fetch_map_range: every ordered row's home slot in a KmerMap of 2^(64 - shift) slots, minus its row index.
// Linear probing that inserts rows in home order into an empty map puts row i at pos_i = max(home_i, pos_{i-1} + 1),
// that is pos_i = i + max_{j <= i}(home_j - j) (a prefix maximum: include/mhmkc_kcount.hpp chunk_ordered).
__global__ __launch_bounds__(O_THREADS) void k_map_home(const uint64_t *keys, uint64_t n, int nlo, int shift,
                                                        long long *v) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    v[i] = (long long)(mhmkc_map_hash(keys + i * (uint64_t)nlo, nlo) >> shift) - (long long)i;
}

// The slot (0xFFFFFFFF past the last one: the map places that row itself) and the tag byte (0x80 | 7 hash bits) of
// every ordered row.
__global__ __launch_bounds__(O_THREADS) void k_map_slots(const uint64_t *keys, const long long *m, uint64_t n, int nlo,
                                                         uint64_t cap, uint32_t *slot, uint8_t *tag) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t pos = i + (uint64_t)m[i];
    slot[i] = pos < cap && pos < 0xffffffffull ? (uint32_t)pos : 0xffffffffu;
    tag[i] = (uint8_t)(0x80u | (mhmkc_map_hash(keys + i * (uint64_t)nlo, nlo) & 0x7fu));
  }
}

}  // namespace

size_t map_slots_scratch_bytes(uint64_t n) {
  size_t t = 0;
  (void)rocprim::inclusive_scan(nullptr, t, (const long long *)nullptr, (long long *)nullptr, (size_t)n,
                                rocprim::maximum<long long>());
  return 2 * ((n + 63) / 64 * 64) * 8 + t + 512;
}

hipError_t launch_map_slots(const uint64_t *keys, uint64_t n, int nlo, uint64_t cap, void *scratch, size_t scratch_bytes,
                            uint32_t *slot, uint8_t *tag, hipStream_t s) {
  if (!n) return hipSuccess;
  if (cap < 2 || (cap & (cap - 1)) || scratch_bytes < map_slots_scratch_bytes(n)) return hipErrorInvalidValue;
  const size_t a = (n + 63) / 64 * 64;
  long long *v = (long long *)scratch, *m = v + a;
  void *tmp = m + a;
  size_t tb = scratch_bytes - 2 * a * 8;
  k_map_home<<<grid_for(n), O_THREADS, 0, s>>>(keys, n, nlo, __builtin_clzll(cap) + 1, v);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if ((e = rocprim::inclusive_scan(tmp, tb, v, m, (size_t)n, rocprim::maximum<long long>(), s)) != hipSuccess) return e;
  k_map_slots<<<grid_for(n), O_THREADS, 0, s>>>(keys, m, n, nlo, cap, slot, tag);
  return hipGetLastError();
}

// The code object of this file (the hand-off kernels and their rocPRIM sorts) is loaded at its first kernel use; a
// handle asks for it at create, so that the first ordered fetch of a process does not pay the load (~40 ms).
hipError_t preload_owner_kernels() {
  hipFuncAttributes a;
  return hipFuncGetAttributes(&a, (const void *)k_map_hash);
}

size_t map_order_scratch_bytes(uint64_t n, int nlo) {
  switch (nlo) {
    case 1: return packed_order_bytes<1>(n);
    case 2: return packed_order_bytes<2>(n);
    case 3: return packed_order_bytes<3>(n);
    case 4: return packed_order_bytes<4>(n);
    default: break;
  }
  size_t t = 0;  // wider output keys (n_longs 5..8): sort row indices, then gather
  (void)rocprim::radix_sort_pairs(nullptr, t, (const uint32_t *)nullptr, (uint32_t *)nullptr, (const uint32_t *)nullptr,
                                  (uint32_t *)nullptr, (size_t)n);
  return 4 * ((n + 63) / 64 * 64) * 4 + t + 256;
}

hipError_t launch_map_order(const OutRows &in, uint64_t n, int nlo, void *scratch, size_t scratch_bytes, const OutRows &out,
                            hipStream_t s) {
  if (!n) return hipSuccess;
  if (n >= 0xffffffffull || scratch_bytes < map_order_scratch_bytes(n, nlo)) return hipErrorInvalidValue;
  switch (nlo) {
    case 1: return packed_order<1>(in, n, scratch, scratch_bytes, out, s);
    case 2: return packed_order<2>(in, n, scratch, scratch_bytes, out, s);
    case 3: return packed_order<3>(in, n, scratch, scratch_bytes, out, s);
    case 4: return packed_order<4>(in, n, scratch, scratch_bytes, out, s);
    default: break;
  }
  const size_t a = (n + 63) / 64 * 64;
  uint32_t *hk = (uint32_t *)scratch, *hk2 = hk + a, *ix = hk2 + a, *ix2 = ix + a;
  void *tmp = ix2 + a;
  size_t tb = scratch_bytes - 4 * a * 4;
  k_map_hash<<<grid_for(n), O_THREADS, 0, s>>>(in.keys, n, nlo, hk, ix);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if ((e = rocprim::radix_sort_pairs(tmp, tb, hk, hk2, ix, ix2, (size_t)n, 0, 32, s)) != hipSuccess) return e;
  k_gather_rows<<<grid_for(n), O_THREADS, 0, s>>>(in, ix2, n, nlo, out);
  return hipGetLastError();
}

hipError_t launch_minimizer_hash(const uint64_t *keys, uint64_t n, int nlo, int k, int m, uint64_t *out, hipStream_t s) {
  if (!n) return hipSuccess;
  if (m < 1 || m > 28 || m > k) return hipErrorInvalidValue;
  k_minimizer_hash<<<grid_for(n), O_THREADS, 0, s>>>(keys, n, nlo, k, m, out);
  return hipGetLastError();
}

hipError_t launch_owner_hist(const uint64_t *keys, uint64_t n, int nlo, int k, int m, int n_ranks, uint8_t *dest,
                             unsigned long long *hist, hipStream_t s) {
  if (!n) return hipSuccess;
  if (m < 1 || m > 28 || m > k || n_ranks < 1 || n_ranks > 256) return hipErrorInvalidValue;
  k_owner_hist<<<grid_for(n), O_THREADS, 0, s>>>(keys, n, nlo, k, m, n_ranks, dest, hist);
  return hipGetLastError();
}

hipError_t launch_owner_scatter(const OutRows &in, uint64_t n, int nlo, const uint8_t *dest, int n_ranks,
                                unsigned long long *cursor, const OutRows &out, hipStream_t s) {
  if (!n) return hipSuccess;
  if (n_ranks < 1 || n_ranks > 256) return hipErrorInvalidValue;
  k_owner_scatter<<<grid_for(n), O_THREADS, 0, s>>>(in, n, nlo, dest, n_ranks, cursor, out);
  return hipGetLastError();
}

}  // namespace mhm
