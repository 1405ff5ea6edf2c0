// Drives the reference-shaped C++ adapter (include/mhmkc_kcount.hpp) the way contigging.cpp drives
// analyze_kmers (src/contigging.cpp:109-119), then prints the table sorted by k-mer in dump_kmers
// format. Modes:
//   adapter_test kat                      Kmer<MAX_K> known answers only (no GPU)
//   adapter_test reads <k> <seqqual.txt> [- <dmin>]  analyze_kmers over PackedReads (dmin_thres = 2 by
//                                                    default), then dump_kmers (per_rank/.../kmers-<k>.txt.gz)
//   adapter_test seqs  <k> <seqqual.txt>  SeqBlockInserter::process_seq over lowercase-masked strings
//   adapter_test ctgs  <k> <seqqual.txt> <ctgs.txt>  analyze_kmers with a Contigs list ("SEQ DEPTH" lines)
//   adapter_test fastq <k> <reads.fq>     FASTQ text through KmerDHT::add_fastq (device parse + pack)
#include <algorithm>
#include <fstream>
#include <iostream>
#include <iterator>
#include <sstream>

#include "mhmkc_kcount.hpp"

using namespace mhm2;

template <int MAX_K>
int run(const std::string &mode, int k, const std::string &path, const std::string &ctg_path, int dmin) {
  Kmer<MAX_K>::set_k(k);
  std::ifstream in(path);
  std::string line;
  PackedReads pr(33);
  std::vector<std::pair<std::string, std::string>> reads;
  while (mode != "fastq" && std::getline(in, line)) {
    std::istringstream ss(line);
    std::string s, q;
    ss >> s >> q;
    pr.add_read("@r/1", s, q);
    reads.emplace_back(s, q);
  }
  KmerDHT<MAX_K> dht(1000, 1 << 20, 100, false, true);  // as contigging.cpp:115-116 builds it
  Contigs ctgs;
  if (mode == "ctgs") {
    std::ifstream cin_(ctg_path);
    int64_t id = 0;
    while (std::getline(cin_, line)) {
      std::istringstream ss(line);
      Contig c;
      c.id = id++;
      ss >> c.seq >> c.depth;
      ctgs.push_back(c);
    }
  }
  if (mode == "fastq") {
    std::ifstream fq(path, std::ios::binary);
    std::string text((std::istreambuf_iterator<char>(fq)), std::istreambuf_iterator<char>());
    dht.add_fastq(text);
    PackedReads back(33);
    dht.inserter().fastq_packed_reads(back);
    std::cerr << "fastq reads " << back.get_local_num_reads() << "\n";
    dht.flush_updates();
    dht.finish_updates();
  } else if (mode == "reads" || mode == "ctgs") {
    std::vector<PackedReads *> list{&pr};
    analyze_kmers<MAX_K>(k, 0, 33, list, dmin, ctgs, dht, mode == "reads");
  } else {
    SeqBlockInserter<MAX_K> sbi(33, dht.get_minimizer_len());
    for (auto &r : reads) {  // count_kmers: lowercase bases below the quality cutoff (kcount.cpp:80-85)
      std::string s = r.first;
      if (s.size() < (size_t)k) continue;
      for (size_t i = 0; i < s.size(); i++) {
        int q = std::min(r.second[i] - 33, 31);
        if (q < 20) s[i] = (char)std::tolower(s[i]);
      }
      sbi.process_seq(s, 0, dht);
    }
    sbi.done_processing(dht);
    dht.flush_updates();
    dht.finish_updates();
  }
  std::vector<std::string> lines;
  for (auto it = dht.local_kmers_begin(); it != dht.local_kmers_end(); ++it) {
    std::ostringstream os;
    os << it->first.to_string() << " " << it->second.count << " " << it->second.left << " " << it->second.right;
    lines.push_back(os.str());
  }
  std::sort(lines.begin(), lines.end());
  for (auto &l : lines) std::cout << l << "\n";
  return 0;
}

int main(int argc, char **argv) {
  std::string mode = argc > 1 ? argv[1] : "kat";
  if (mode == "kat") {
    Kmer<32>::set_k(21);
    Kmer<32> a("ACGTACGTACGTACGTACGTA");
    Kmer<64>::set_k(63);
    Kmer<64> b("CGCTGTTCCAGATGACGAACCAGGAATTCCGCCAGGTATTCGACTTTATTCGCGAAGTCAAGA");
    Kmer<32> c("CGCTGTTCCAGATGACGAACC");
    bool ok = a.get_longs()[0] == 0x1b1b1b1b1b000000ull && a.hash() == 0xa47f0f8106be6783ull &&
              b.get_longs()[0] == 0x67bd48e1814a0f59ull && b.get_longs()[1] == 0x4acf61fcf660b420ull &&
              b.hash() == 0x470509568a42d5b5ull && a.revcomp().revcomp() == a &&
              a.revcomp().to_string() == "TACGTACGTACGTACGTACGT" &&
              // get_minimizer_fast / minimizer_hash_fast known answers
              a.get_minimizer_fast(15) == 0xb1b1b1b000000000ull && a.minimizer_hash_fast(15) == 0x7b9cf376cdbe4a50ull &&
              c.get_minimizer_fast(15) == 0xdb4de81000000000ull && c.minimizer_hash_fast(15) == 0xfbeed8639c5ae34full &&
              b.get_minimizer_fast(27) == 0xcf61fcf660b42000ull && b.minimizer_hash_fast(27) == 0xaa95c0beb14e494full &&
              quick_hash(0) == 0x7b439d0c1fd00de3ull;
    std::cout << (ok ? "KAT OK" : "KAT FAIL") << "\n";
    return ok ? 0 : 1;
  }
  int k = std::atoi(argv[2]);
  const std::string ctg_path = argc > 4 ? argv[4] : "";
  const int dmin = argc > 5 ? std::atoi(argv[5]) : 2;
  if (k < 32) return run<32>(mode, k, argv[3], ctg_path, dmin);
  if (k < 64) return run<64>(mode, k, argv[3], ctg_path, dmin);
  if (k < 96) return run<96>(mode, k, argv[3], ctg_path, dmin);
  return run<128>(mode, k, argv[3], ctg_path, dmin);
}
