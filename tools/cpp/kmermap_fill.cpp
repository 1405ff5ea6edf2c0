// KmerMap materialisation timing for bench.py (D2H + KmerMap fill reported beside the GPU
// step). Reads a fetched table (mhmkc_fetch layout) from raw files and fills the adapter's KmerMap<MAX_K>
// (include/mhmkc_kcount.hpp, the reference's insert loop of insert_into_local_hashtable,
// src/kcount/kcount_cpu.cpp:503-517) with the same emplace loop as KmerDHT::load_table.
//   kmermap_fill <k> <n_rows> <prefix>   (prefix.keys u64 [n * N_LONGS], .counts u16, .left, .right)
// prints one JSON line: {"rows": n, "ms": fill time, "buckets": ...}
#include <chrono>
#include <cstdio>
#include <cstdlib>
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
static int run(int k, size_t n, const std::string &pre) {
  mhm2::Kmer<MAX_K>::set_k(k);
  const int nl = mhm2::Kmer<MAX_K>::N_LONGS;
  auto keys = slurp<uint64_t>(pre + ".keys", n * nl);
  auto counts = slurp<uint16_t>(pre + ".counts", n);
  auto left = slurp<char>(pre + ".left", n), right = slurp<char>(pre + ".right", n);
  mhm2::KmerMap<MAX_K> map;
  const auto t0 = std::chrono::steady_clock::now();
  map.fill(keys.data(), counts.data(), left.data(), right.data(), n);  // KmerDHT::load_table's loop
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  // the same rows through the per-row emplace (no prefetch): what a caller's own loop costs
  mhm2::KmerMap<MAX_K> map2;
  const auto t1 = std::chrono::steady_clock::now();
  map2.reserve(n);
  for (size_t i = 0; i < n; i++) {
    mhm2::KmerCounts kc;
    kc.count = counts[i];
    kc.left = left[i];
    kc.right = right[i];
    map2.emplace(mhm2::Kmer<MAX_K>(&keys[i * nl]), kc);
  }
  const double ms2 = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
  // every row is found again with its counts
  size_t bad = 0;
  for (size_t i = 0; i < n; i += 97) {
    auto it = map.find(mhm2::Kmer<MAX_K>(&keys[i * nl]));
    if (it == map.end() || it->second.count != counts[i] || it->second.left != left[i] || it->second.right != right[i]) bad++;
  }
  printf("{\"rows\": %zu, \"ms\": %.3f, \"ms_emplace_loop\": %.3f, \"size\": %zu, \"bad\": %zu}\n", n, ms, ms2,
         map.size(), bad);
  return map.size() == n && map2.size() == n && bad == 0 ? 0 : 1;
}

int main(int argc, char **argv) {
  if (argc != 4) {
    fprintf(stderr, "usage: kmermap_fill <k> <n_rows> <prefix>\n");
    return 2;
  }
  const int k = atoi(argv[1]);
  const size_t n = strtoull(argv[2], nullptr, 10);
  const std::string pre = argv[3];
  switch (k / 32 + 1) {
    case 1: return run<32>(k, n, pre);
    case 2: return run<64>(k, n, pre);
    case 3: return run<96>(k, n, pre);
    case 4: return run<128>(k, n, pre);
  }
  return 2;
}
