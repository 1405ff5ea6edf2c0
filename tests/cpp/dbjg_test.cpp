// Multi-k contigging end to end at one rank (src/contigging.cpp:93-158, src/main.cpp:167-199): for each k,
// count (analyze_kmers with the previous round's contigs), traverse the de Bruijn graph, and hand the contigs
// to the next k. Prints, per round, the contigs as "K <k>" then sorted "<canonical seq> <depth>" lines.
//   dbjg_test gpu    <seqqual.txt> <k1,k2,...>   counting on the GPU (libmhmkc through mhmkc_kcount.hpp)
//   dbjg_test oracle <seqqual.txt> <k1,k2,...>   counting by the CPU oracle (oracle/liboracle.so, the checker)
// Both sides then run the same traversal (include/mhmkc_dbjg.hpp), so equal tables give equal contigs.
#include <cstdio>
#include <fstream>
#include <iostream>
#include <sstream>

#include "mhmkc_dbjg.hpp"

using namespace mhm2;

extern "C" {  // oracle/kcount_oracle.c (test infrastructure)
void *orc_kcount_ctgs(const uint8_t *, const uint64_t *, uint64_t, const char *, const uint64_t *, const uint16_t *,
                      uint64_t, int, int, int, int, double);
uint64_t orc_table_size(const void *);
void orc_table_fetch(const void *, uint64_t *, uint16_t *, char *, char *);
void orc_table_free(void *);
}

static std::string canon(const std::string &s) {
  std::string r(s.rbegin(), s.rend());
  for (char &c : r) c = dbjg_comp(c);
  return std::min(s, r);
}

template <int MAX_K>
void round_k(bool gpu, int k, int prev_k, PackedReads &pr, Contigs &ctgs) {
  Kmer<MAX_K>::set_k(k);
  RankInfo ri;
  ri.table_only = !gpu;
  KmerDHT<MAX_K> dht(1000, 1 << 20, 100, false, true, ri);
  if (gpu) {
    std::vector<PackedReads *> list{&pr};
    analyze_kmers<MAX_K>(k, prev_k, 33, list, 2, ctgs, dht, false);
  } else {  // the oracle's table into the same KmerMap (via the adapter's insert path is not needed: build it)
    std::string cs;
    std::vector<uint64_t> co{0};
    std::vector<uint16_t> cd;
    for (auto &c : ctgs) {
      cs += c.seq;
      co.push_back(cs.size());
      cd.push_back(c.get_uint16_t_depth());
    }
    const int nl = Kmer<MAX_K>::N_LONGS;
    void *t = orc_kcount_ctgs(pr.bytes(), pr.offsets(), pr.get_local_num_reads(), cs.data(), co.data(), cd.data(),
                              cd.size(), k, nl, 20, 2, 0.9);
    if (!t) die("oracle failed");
    const uint64_t n = orc_table_size(t);
    std::vector<uint64_t> keys(n * nl);
    std::vector<uint16_t> cnt(n);
    std::vector<char> l(n), r(n);
    orc_table_fetch(t, keys.data(), cnt.data(), l.data(), r.data());
    orc_table_free(t);
    dht.load_table(keys.data(), cnt.data(), l.data(), r.data(), n);
  }
  Contigs out;
  traverse_debruijn_graph<MAX_K>(k, dht, out);
  std::vector<std::string> lines;
  for (auto &c : out) {
    char buf[64];
    std::snprintf(buf, sizeof buf, " %.6f", c.depth);
    lines.push_back(canon(c.seq) + buf);
  }
  std::sort(lines.begin(), lines.end());
  std::cout << "K " << k << " " << out.size() << "\n";
  for (auto &x : lines) std::cout << x << "\n";
  ctgs = out;
}

int main(int argc, char **argv) {
  if (argc < 4) return 2;
  const bool gpu = std::string(argv[1]) == "gpu";
  std::ifstream in(argv[2]);
  std::string line;
  PackedReads pr(33);
  while (std::getline(in, line)) {
    std::istringstream ss(line);
    std::string s, q;
    ss >> s >> q;
    pr.add_read("@r/1", s, q);
  }
  std::vector<int> ks;
  std::stringstream kl(argv[3]);
  for (std::string x; std::getline(kl, x, ',');) ks.push_back(std::atoi(x.c_str()));
  Contigs ctgs;
  int prev = 0;
  for (int k : ks) {
    if (k < 32)
      round_k<32>(gpu, k, prev, pr, ctgs);
    else if (k < 64)
      round_k<64>(gpu, k, prev, pr, ctgs);
    else if (k < 96)
      round_k<96>(gpu, k, prev, pr, ctgs);
    else
      round_k<128>(gpu, k, prev, pr, ctgs);
    prev = k;
  }
  return 0;
}
