// TEST INFRASTRUCTURE. The restated de Bruijn traversal (include/mhmkc_dbjg.hpp, src/dbjg_traversal.cpp:569-596) over
// a count table given as arrays, for the multi-rank multi-k chain of tests/test_c5_scale.py: rank 0 traverses the
// union of the ranks' tables and the uutigs become the next k's contigs (src/contigging.cpp:93-158).
//   int64_t mhmkc_dbjg_traverse(int k, const uint64_t *keys, const uint16_t *counts, const char *left,
//                               const char *right, uint64_t n, const char *path)
// keys: n rows of k / 32 + 1 words; writes "<seq> <Contig::get_uint16_t_depth()>" lines to path in the traversal's
// order (walks start in Kmer order, so equal tables give equal files whatever their row order); returns the number of
// uutigs, -1 if k is out of range or the file cannot be written.
#include <cstdio>

#include "mhmkc_dbjg.hpp"

using namespace mhm2;

template <int MAX_K>
static int64_t run(int k, const uint64_t *keys, const uint16_t *counts, const char *left, const char *right, uint64_t n,
                   const char *path) {
  Kmer<MAX_K>::set_k(k);
  RankInfo ri;
  ri.table_only = true;
  KmerDHT<MAX_K> dht(1000, 1 << 20, 100, false, true, ri);
  dht.load_table(keys, counts, left, right, n);
  Contigs out;
  traverse_debruijn_graph<MAX_K>((unsigned)k, dht, out);
  FILE *f = std::fopen(path, "w");
  if (!f) return -1;
  for (auto &c : out) std::fprintf(f, "%s %u\n", c.seq.c_str(), (unsigned)c.get_uint16_t_depth());
  if (std::fclose(f) != 0) return -1;
  return (int64_t)out.size();
}

extern "C" int64_t mhmkc_dbjg_traverse(int k, const uint64_t *keys, const uint16_t *counts, const char *left,
                                       const char *right, uint64_t n, const char *path) {
  if (k < 2 || k > 127 || k % 32 == 0) return -1;
  switch (k / 32) {
    case 0: return run<32>(k, keys, counts, left, right, n, path);
    case 1: return run<64>(k, keys, counts, left, right, n, path);
    case 2: return run<96>(k, keys, counts, left, right, n, path);
    default: return run<128>(k, keys, counts, left, right, n, path);
  }
}
