// KmerMap materialisation timing for bench.py (D2H + KmerMap fill reported beside the GPU
// step). Reads a fetched table (mhmkc_fetch layout) from raw files and fills the adapter's KmerMap<MAX_K>
// (include/mhmkc_kcount.hpp, the reference's insert loop of insert_into_local_hashtable,
// src/kcount/kcount_cpu.cpp:503-517) with KmerMap::fill, as HashTableInserter::insert_into_local_hashtable does.
//   kmermap_fill <k> <n_rows> <prefix> [threads] [--sort] [--chunks C]
//     prefix.keys u64 [n * N_LONGS], .counts u16, .left, .right
//     threads: fill threads (0 or absent: KmerMap::fill_threads())
//     --sort: order the rows by the top 32 bits of mhmkc_map_hash first (what mhmkc_fetch_ordered gives), untimed
//     --chunks C: the threaded fill in C chunks (fill_begin / fill_chunk / fill_end, as load_ordered streams them)
//     --slots: (implies --sort; repeated keys dropped) each row's slot and tag computed as mhmkc_fetch_map_range's
//              device kernel computes them, the rows placed by KmerMap::fill_chunk_slots (load_ordered's path into an
//              empty map)
// prints one JSON line: {"rows": n, "ms": fill time, "ms_one_thread": the one-thread fill, ...}. Every row is looked up
// in both maps afterwards; the exit code is 1 if any is missing or differs.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <climits>
#include <cstdlib>
#include <numeric>
#include <string>
#include <vector>

#include "mhmkc_kcount.hpp"

template <typename T>
static std::vector<T> slurp(const std::string &path, size_t n) {
  std::vector<T> v(n);
  FILE *f = fopen(path.c_str(), "rb");
  if (!f || fread(v.data(), sizeof(T), n, f) != n) {
    fprintf(stderr, "cannot read %s\n", path.c_str());
    exit(2);
  }
  fclose(f);
  return v;
}

template <int MAX_K>
static int run(int k, size_t n, const std::string &pre, int threads, bool sort_rows, uint64_t chunks, bool slots_mode) {
  mhm2::Kmer<MAX_K>::set_k(k);
  const int nl = mhm2::Kmer<MAX_K>::N_LONGS;
  auto keys = slurp<uint64_t>(pre + ".keys", n * nl);
  auto counts = slurp<uint16_t>(pre + ".counts", n);
  auto left = slurp<char>(pre + ".left", n), right = slurp<char>(pre + ".right", n);
  if (sort_rows) {
    std::vector<uint64_t> ix(n);
    std::iota(ix.begin(), ix.end(), 0);
    std::stable_sort(ix.begin(), ix.end(), [&](uint64_t a, uint64_t b) {
      return (mhmkc_map_hash(&keys[a * nl], nl) >> 32) < (mhmkc_map_hash(&keys[b * nl], nl) >> 32);
    });
    std::vector<uint64_t> k2(n * nl);
    std::vector<uint16_t> c2(n);
    std::vector<char> l2(n), r2(n);
    for (size_t i = 0; i < n; i++) {
      std::copy(&keys[ix[i] * nl], &keys[ix[i] * nl] + nl, &k2[i * nl]);
      c2[i] = counts[ix[i]], l2[i] = left[ix[i]], r2[i] = right[ix[i]];
    }
    keys.swap(k2), counts.swap(c2), left.swap(l2), right.swap(r2);
  }
  if (threads <= 0) threads = mhm2::KmerMap<MAX_K>::fill_threads();
  if (slots_mode) {  // the rows' unique keys only (the device's slots assume a finished table's unique keys)
    std::vector<uint64_t> k2;
    std::vector<uint16_t> c2;
    std::vector<char> l2, r2;
    mhm2::KmerMap<MAX_K> seen;
    for (size_t i = 0; i < n; i++) {
      if (!seen.emplace(mhm2::Kmer<MAX_K>(&keys[i * nl]), mhm2::KmerCounts()).second) continue;
      k2.insert(k2.end(), &keys[i * nl], &keys[i * nl] + nl);
      c2.push_back(counts[i]), l2.push_back(left[i]), r2.push_back(right[i]);
    }
    n = c2.size();
    keys.swap(k2), counts.swap(c2), left.swap(l2), right.swap(r2);
  }
  mhm2::KmerMap<MAX_K> map;
  const auto t0 = std::chrono::steady_clock::now();
  if (slots_mode) {  // mhmkc_fetch_map_range's slots and tags, computed here as the device does (k_map_slots)
    map.fill_begin(n, threads);
    if (!map.fill_by_slots()) {
      fprintf(stderr, "fill_by_slots is false\n");
      return 2;
    }
    const uint64_t cap = map.bucket_count();
    const int shift = 64 - __builtin_ctzll(cap);
    std::vector<uint32_t> slot(n);
    std::vector<uint8_t> tag(n);
    int64_t mx = INT64_MIN;
    for (size_t i = 0; i < n; i++) {
      const uint64_t h = mhmkc_map_hash(&keys[i * nl], nl);
      mx = std::max<int64_t>(mx, (int64_t)(h >> shift) - (int64_t)i);
      const uint64_t pos = i + (uint64_t)mx;
      slot[i] = pos < cap && pos < 0xffffffffull ? (uint32_t)pos : 0xffffffffu;
      tag[i] = (uint8_t)(0x80u | (h & 0x7fu));
    }
    const auto t2 = std::chrono::steady_clock::now();  // (the fill alone, as load_ordered runs it)
    for (uint64_t c = 0; c < std::max<uint64_t>(1, chunks); c++) {
      const uint64_t a = n * c / std::max<uint64_t>(1, chunks), b = n * (c + 1) / std::max<uint64_t>(1, chunks);
      map.fill_chunk_slots(&keys[a * nl], &counts[a], &left[a], &right[a], &slot[a], &tag[a], b - a);
    }
    map.fill_end();
    (void)t2;
  } else if (chunks <= 1) {
    map.fill(keys.data(), counts.data(), left.data(), right.data(), n, threads);
  } else {
    map.fill_begin(n, threads);
    for (uint64_t c = 0; c < chunks; c++) {
      const uint64_t a = n * c / chunks, b = n * (c + 1) / chunks;
      map.fill_chunk(&keys[a * nl], &counts[a], &left[a], &right[a], b - a);
    }
    map.fill_end();
  }
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  // the same rows through the one-thread prefetched loop
  mhm2::KmerMap<MAX_K> map1;
  const auto t1 = std::chrono::steady_clock::now();
  map1.fill(keys.data(), counts.data(), left.data(), right.data(), n, 1);
  const double ms1 = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
  // every row is found again in both maps with its first occurrence's counts (fill keeps a present entry)
  size_t bad = 0;
  for (size_t i = 0; i < n; i++) {
    const mhm2::Kmer<MAX_K> km(&keys[i * nl]);
    auto it = map.find(km);
    auto it1 = map1.find(km);
    if (it == map.end() || it1 == map1.end()) {
      bad++;
      continue;
    }
    if (it->second.count != it1->second.count || it->second.left != it1->second.left ||
        it->second.right != it1->second.right)
      bad++;
  }
  printf("{\"rows\": %zu, \"ms\": %.3f, \"threads\": %d, \"ms_one_thread\": %.3f, \"size\": %zu, \"size_one_thread\": "
         "%zu, \"buckets\": %zu, \"bad\": %zu}\n",
         n, ms, threads, ms1, map.size(), map1.size(), map.bucket_count(), bad);
  return map.size() == map1.size() && bad == 0 ? 0 : 1;
}

int main(int argc, char **argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: kmermap_fill <k> <n_rows> <prefix> [threads] [--sort]\n");
    return 2;
  }
  const int k = atoi(argv[1]);
  const size_t n = strtoull(argv[2], nullptr, 10);
  const std::string pre = argv[3];
  int threads = 0;
  bool sort_rows = false, slots_mode = false;
  uint64_t chunks = 1;
  for (int a = 4; a < argc; a++) {
    if (std::string(argv[a]) == "--sort")
      sort_rows = true;
    else if (std::string(argv[a]) == "--slots")
      slots_mode = sort_rows = true;
    else if (std::string(argv[a]) == "--chunks" && a + 1 < argc)
      chunks = strtoull(argv[++a], nullptr, 10);
    else
      threads = atoi(argv[a]);
  }
  switch (k / 32 + 1) {
    case 1: return run<32>(k, n, pre, threads, sort_rows, chunks, slots_mode);
    case 2: return run<64>(k, n, pre, threads, sort_rows, chunks, slots_mode);
    case 3: return run<96>(k, n, pre, threads, sort_rows, chunks, slots_mode);
    case 4: return run<128>(k, n, pre, threads, sort_rows, chunks, slots_mode);
  }
  return 2;
}
