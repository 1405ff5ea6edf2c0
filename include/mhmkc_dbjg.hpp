// mhmkc_dbjg.hpp — the consumer of the count table: a single-rank restatement of the reference's de Bruijn
// graph traversal (ajpowelsnl/mhm2_proxy src/dbjg_traversal.cpp:569-596) over the KmerMap that
// include/mhmkc_kcount.hpp fills from libmhmkc, so a round of contigging (src/contigging.cpp:93-158:
// analyze_kmers, then traverse_debruijn_graph, whose contigs feed the next k's contig pass) runs end to end.
//
// At one rank every k-mer is local, so a walk never leaves get_next_step (:165-239), no fragment is ever
// reached from another walk (the predecessor of a k-mer through its left extension is unique, so two walks
// cannot enter one chain) and clean_frag_links / connect_frags (:392-567) have no links to follow: every walk
// is one uutig. What the reference does per walk is kept exactly:
//   - a walk starts at a k-mer not yet visited whose extensions are both unique (:301-307);
//   - it goes left, then right from the same k-mer (revisiting the start is allowed once, :253-254), and
//     stops at a missing k-mer (DEADEND), an 'X' (DEADEND), an 'F' (FORK), an extension that does not lead
//     back (CONFLICT) or a k-mer already visited by this walk (REPEAT) (:171-205);
//   - the uutig is the reversed left-walk fronts + start[1..k-2] + the right-walk backs (:245-289); the depth
//     sum counts the start k-mer in both walks (:224);
//   - uutigs shorter than k are dropped, depth = sum / (len - k + 2) (:404-407,539-541).
// The reference starts walks in KmerMap iteration order; here they start in Kmer order (operator<), which
// only matters for cycles (where the start chooses the rotation) and makes the result deterministic.
#pragma once

#include <algorithm>
#include <string>
#include <vector>

#include "mhmkc_kcount.hpp"

namespace mhm2 {

// comp_nucleotide (src/utils.cpp:121-143) for the characters a walk meets
inline char dbjg_comp(char c) {
  switch (c) {
    case 'A': return 'T';
    case 'C': return 'G';
    case 'G': return 'C';
    case 'T': return 'A';
  }
  return c;
}

template <int MAX_K>
struct DbjgKmer {  // Kmer front/back/forward_base/backward_base (src/kmer.cpp:513-561) on a string
  std::string s;
  char front() const { return s.front(); }
  char back() const { return s.back(); }
  DbjgKmer forward_base(char b) const { return {s.substr(1) + b}; }
  DbjgKmer backward_base(char b) const { return {std::string(1, b) + s.substr(0, s.size() - 1)}; }
  DbjgKmer revcomp() const {
    std::string r(s.rbegin(), s.rend());
    for (char &c : r) c = dbjg_comp(c);
    return {r};
  }
};

// traverse_debruijn_graph (src/dbjg_traversal.cpp:569-596) at one rank: my_uutigs gets the uutigs, ids from 0.
template <int MAX_K>
void traverse_debruijn_graph(unsigned kmer_len, KmerDHT<MAX_K> &kmer_dht, Contigs &my_uutigs) {
  using K = Kmer<MAX_K>;
  enum Status { RUNNING, DEADEND, FORK, CONFLICT, VISITED, REPEAT };
  my_uutigs.clear();
  std::vector<const K *> order;
  order.reserve((size_t)kmer_dht.get_local_num_kmers());
  for (auto it = kmer_dht.local_kmers_begin(); it != kmer_dht.local_kmers_end(); ++it) {
    it->second.uutig_frag = nullptr;
    order.push_back(&it->first);
  }
  std::sort(order.begin(), order.end(), [](const K *a, const K *b) { return *a < *b; });
  std::vector<char> frag_ids;  // the address of frag_ids[i] is walk i's mark (uutig_frag)
  frag_ids.resize(order.size() + 1);
  size_t n_walks = 0;
  for (const K *start : order) {
    KmerCounts *sc = kmer_dht.get_local_kmer_counts(*start);
    if (sc->uutig_frag) continue;
    if (sc->left == 'X' || sc->left == 'F' || sc->right == 'X' || sc->right == 'F') continue;
    void *frag = &frag_ids[n_walks++];
    std::string uutig;
    int64_t sum_depths = 0;
    for (int dirn = 0; dirn < 2; dirn++) {  // 0 = LEFT, 1 = RIGHT (traverse_dirn, :245-289)
      const bool left_dirn = dirn == 0;
      DbjgKmer<MAX_K> kmer{start->to_string()};
      char prev_ext = 0, next_ext = left_dirn ? kmer.front() : kmer.back();
      bool revisit_allowed = !left_dirn;
      std::string walk;
      if (!left_dirn) walk = kmer.s.substr(1, kmer.s.size() - 2);
      for (;;) {  // get_next_step (:165-239)
        DbjgKmer<MAX_K> canon = kmer, rc = kmer.revcomp();
        bool is_rc = false;
        if (rc.s < kmer.s) {
          canon = rc;
          is_rc = true;
        }
        K key(canon.s.c_str());
        KmerCounts *kc = kmer_dht.get_local_kmer_counts(key);
        Status status = RUNNING;
        if (!kc) {
          status = DEADEND;
        } else {
          char left = kc->left, right = kc->right;
          if (left == 'X' || right == 'X') {
            status = DEADEND;
          } else if (left == 'F' || right == 'F') {
            status = FORK;
          } else {
            if (is_rc) {
              std::swap(left, right);
              left = dbjg_comp(left);
              right = dbjg_comp(right);
            }
            if (prev_ext && ((left_dirn && prev_ext != right) || (!left_dirn && prev_ext != left))) {
              status = CONFLICT;
            } else if (kc->uutig_frag && kc->uutig_frag != frag) {
              status = VISITED;  // another walk's k-mer (not reachable at one rank, kept for the rule's sake)
            } else if (kc->uutig_frag == frag && !revisit_allowed) {
              status = REPEAT;
            } else {
              kc->uutig_frag = frag;
              walk += next_ext;
              next_ext = left_dirn ? left : right;
              if (left_dirn) {
                prev_ext = kmer.back();
                kmer = kmer.backward_base(next_ext);
              } else {
                prev_ext = kmer.front();
                kmer = kmer.forward_base(next_ext);
              }
              sum_depths += kc->count;
              revisit_allowed = false;
            }
          }
        }
        if (status != RUNNING) break;
      }
      if (left_dirn) std::reverse(walk.begin(), walk.end());
      uutig += walk;
    }
    if (uutig.size() < kmer_len) continue;  // connect_frags: frag_len < kmer_len (:518)
    my_uutigs.push_back(Contig{(int64_t)my_uutigs.size(), uutig, (double)sum_depths / (uutig.size() - kmer_len + 2)});
  }
}

}  // namespace mhm2
