// mhmkc_kcount.hpp — the reference's kcount C++ interface rebuilt over the C ABI of libmhmkc.so.
//
// Shapes kept from ajpowelsnl/mhm2_proxy so contigging.cpp / dbjg_traversal.cpp style callers compile
// against the same names:
//   Kmer<MAX_K>                      src/kmer.hpp:61-160   (longs layout, set_k/get_k, hash, revcomp, ...)
//   KmerCounts                       src/kcount/kmer_dht.hpp:62-68
//   KmerMap<MAX_K>                   src/kcount/kmer_dht.hpp:92-93 (an open-addressing map, as the reference's
//                                    bytell_hash_map; the container type does not affect the contents)
//   PackedReads                      src/packed_reads.hpp:120-167 (contiguous bytes + offsets)
//   HashTableInserter<MAX_K>         src/kcount/kmer_dht.hpp:95-116
//   SeqBlockInserter<MAX_K>          src/kcount/kcount.hpp:57-69
//   KmerDHT<MAX_K>                   src/kcount/kmer_dht.hpp:118-172 (one rank; UPC++ dist_object dropped)
//   analyze_kmers<MAX_K>(...)        src/kcount/kcount.hpp:71-73
//   _dmin_thres                      src/kcount/kmer_dht.hpp:57 (set by analyze_kmers, read at finish)
// Errors abort with a message, as the reference's DIE does (upcxx-utils log.hpp:251). dump_kmers writes
// gzip through zlib: link with -lz.
#pragma once

#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <zlib.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <unordered_map>
#include <utility>
#include <vector>

#include "mhmkc.h"

namespace mhm2 {

using kmer_count_t = uint16_t;

// the depth threshold of get_ext: a global in the reference (src/kcount/kmer_dht.hpp:57), set by
// analyze_kmers (src/kcount/kcount.cpp:145) and read when the table is finished (kcount_cpu.cpp:178)
inline int _dmin_thres = 2;

// quick_hash (src/hash_funcs.c:332-342)
inline uint64_t quick_hash(uint64_t v) {
  v = v * 3935559000370003845ull + 2691343689449507681ull;
  v ^= v >> 21;
  v ^= v << 37;
  v ^= v >> 4;
  v *= 4768777513237032717ull;
  v ^= v << 20;
  v ^= v >> 41;
  v ^= v << 5;
  return v;
}

[[noreturn]] inline void die(const std::string &msg) {
  std::fprintf(stderr, "mhmkc: %s\n", msg.c_str());
  std::fflush(stderr);
  std::abort();
}

inline void check(int rc, mhmkc_t h, const char *what) {
  if (rc != MHMKC_OK) die(std::string(what) + ": " + mhmkc_last_error(h));
}

// ---------------------------------------------------------------------------------------------
// Kmer<MAX_K>

template <int MAX_K>
class Kmer {
 public:
  static constexpr int N_LONGS = (MAX_K + 31) / 32;

 private:
  inline static unsigned k = 0;
  std::array<uint64_t, N_LONGS> longs{};

  static uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
  static uint64_t fmix(uint64_t v) {
    v ^= v >> 33;
    v *= 0xff51afd7ed558ccdull;
    v ^= v >> 33;
    v *= 0xc4ceb9fe1a85ec53ull;
    v ^= v >> 33;
    return v;
  }

 public:
  Kmer() = default;
  explicit Kmer(const uint64_t *other) { std::memcpy(longs.data(), other, sizeof longs); }
  explicit Kmer(const char *s) { set_kmer(s); }

  static void set_k(unsigned kk) { k = kk; }
  static unsigned get_k() { return k; }
  static unsigned get_N_LONGS() { return N_LONGS; }
  static unsigned get_MAX_K() { return MAX_K; }

  void set_kmer(const char *s) {  // src/kmer.cpp:274-296
    longs.fill(0);
    for (unsigned i = 0; i < k; i++) {
      uint64_t x = ((uint64_t)s[i] & 4) >> 1;
      longs[i / 32] |= (x + ((x ^ ((uint64_t)s[i] & 2)) >> 1)) << (2 * (31 - i % 32));
    }
  }
  const uint64_t *get_longs() const { return longs.data(); }
  bool operator<(const Kmer &o) const { return longs < o.longs; }  // word-wise unsigned (src/kmer.cpp:265-272)
  bool operator==(const Kmer &o) const { return longs == o.longs; }
  bool operator!=(const Kmer &o) const { return !(*this == o); }

  // MurmurHash3_x64_64(longs, 8*N_LONGS) with seed 313 (src/kmer.cpp:465-468, src/hash_funcs.c:77-190)
  uint64_t hash() const {
    const uint64_t c1 = 0x87c37b91114253d5ull, c2 = 0x4cf5ad432745937full;
    uint64_t h1 = 313, h2 = 313;
    for (int b = 0; b < N_LONGS / 2; b++) {
      uint64_t k1 = longs[2 * b] * c1, k2 = longs[2 * b + 1] * c2;
      h1 ^= rotl(k1, 31) * c2;
      h1 = rotl(h1, 27) + h2;
      h1 = h1 * 5 + 0x52dce729;
      h2 ^= rotl(k2, 33) * c1;
      h2 = rotl(h2, 31) + h1;
      h2 = h2 * 5 + 0x38495ab5;
    }
    if (N_LONGS & 1) h1 ^= rotl(longs[N_LONGS - 1] * c1, 31) * c2;
    h1 ^= 8 * N_LONGS;
    h2 ^= 8 * N_LONGS;
    h1 += h2;
    h2 += h1;
    h1 = fmix(h1);
    h2 = fmix(h2);
    return h1 + h2;
  }

  Kmer revcomp() const {  // same result as src/kmer.cpp:485-505
    std::string s = to_string(), r(s.rbegin(), s.rend());
    for (char &c : r) c = c == 'A' ? 'T' : c == 'C' ? 'G' : c == 'G' ? 'C' : 'A';
    return Kmer(r.c_str());
  }

  std::string to_string() const {  // src/kmer.cpp:595-634
    std::string s(k, 'N');
    for (unsigned i = 0; i < k; i++) s[i] = "ACGT"[(longs[i / 32] >> (2 * (31 - i % 32))) & 3];
    return s;
  }

  // get_minimizer_fast(m, least_complement = true) (src/kmer.cpp:344-403): the greatest, over the m-mer
  // positions, of min(forward m-mer, its reverse complement), left-aligned with the low bits zero
  uint64_t get_minimizer_fast(int m) const {
    const uint64_t mm = (1ull << (2 * m)) - 1;
    uint64_t f = 0, r = 0, best = 0;
    for (unsigned j = 0; j < k; j++) {
      const uint64_t b = (longs[j / 32] >> (62 - 2 * (j % 32))) & 3;
      f = ((f << 2) | b) & mm;
      r = (r >> 2) | ((3 - b) << (2 * m - 2));
      if ((int)j >= m - 1) best = std::max(best, std::min(f << (64 - 2 * m), r << (64 - 2 * m)));
    }
    return best;
  }
  uint64_t minimizer_hash_fast(int m) const { return quick_hash(get_minimizer_fast(m)); }  // src/kmer.cpp:454-463
};

template <int MAX_K>
struct KmerHash {
  size_t operator()(const Kmer<MAX_K> &km) const { return km.hash(); }
};

// ---------------------------------------------------------------------------------------------
// KmerCounts / KmerMap

struct KmerCounts {
  void *uutig_frag = nullptr;  // global_ptr<FragElem> in the reference; dbjg's visited mark
  kmer_count_t count = 0;
  char left = 0, right = 0;
};

// KmerMap<MAX_K>: an open-addressing map in the spirit of the reference's ska::bytell_hash_map (USE_BYTELL,
// src/utils.hpp:57-64; KmerMap = HASH_TABLE<Kmer<MAX_K>, KmerCounts>, src/kcount/kmer_dht.hpp:92-93): one flat slot
// array, linear probing over a power-of-two capacity, a one-byte tag per slot (0 empty, 0x80 | 7 hash bits) so
// that a probe compares keys only on a tag match, load <= 7/8. It offers what the reference's callers use
// (find / end, begin..end iteration, insert / emplace / operator[], size, reserve, clear, swap; no erase: kcount
// and dbjg never erase) plus fill(): the bulk insert of a fetched table with the slots of the next rows
// prefetched, so that filling a table larger than the caches is not one DRAM round trip per row
// (insert_into_local_hashtable's loop, src/kcount/kcount_cpu.cpp:503-522; a node-allocating std::unordered_map
// took 136 ns per row at C2).
// Worker threads of a KmerMap bulk fill (fill_begin .. fill_end): started once, then each chunk's job is handed to them
// (a chunk is one D2H's worth of rows: spawning threads per chunk cost more than placing the chunk's rows).
class FillPool {
 public:
  explicit FillPool(int n) : n_(n) {
    for (int t = 1; t < n; t++) th_.emplace_back([this, t] { loop(t); });
  }
  ~FillPool() {
    {
      std::lock_guard<std::mutex> l(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto &x : th_) x.join();
  }
  FillPool(const FillPool &) = delete;
  FillPool &operator=(const FillPool &) = delete;
  int size() const { return n_; }
  // f(t) for every t in [0, size()), the caller as thread 0; returns when all are done (the caller sleeps on a
  // condition variable, not in a yield loop: with several ranks per node the fill threads of one rank would otherwise
  // compete with a spinning caller for the rank's CPUs)
  void run(const std::function<void(int)> &f) {
    {
      std::lock_guard<std::mutex> l(mu_);
      job_ = &f;
      left_ = n_ - 1;
      gen_++;
    }
    cv_.notify_all();
    f(0);
    std::unique_lock<std::mutex> l(mu_);
    done_cv_.wait(l, [&] { return left_ == 0; });
  }

 private:
  void loop(int t) {
    uint64_t seen = 0;
    while (true) {
      const std::function<void(int)> *j;
      {
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        j = job_;
      }
      (*j)(t);
      std::lock_guard<std::mutex> l(mu_);
      if (--left_ == 0) done_cv_.notify_one();
    }
  }
  int n_;
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)> *job_ = nullptr;
  uint64_t gen_ = 0;
  bool stop_ = false;
  int left_ = 0;  // (under mu_)
};

template <int MAX_K>
class KmerMap {
 public:
  using key_type = Kmer<MAX_K>;
  using mapped_type = KmerCounts;
  using value_type = std::pair<key_type, mapped_type>;  // first is not const: slots move when the map grows

  template <bool CONST>
  class iter {
    using M = typename std::conditional<CONST, const KmerMap, KmerMap>::type;
    using V = typename std::conditional<CONST, const value_type, value_type>::type;
    M *m_ = nullptr;
    size_t i_ = 0;
    void skip() {
      while (i_ < m_->cap_ && !m_->tag_[i_]) i_++;
    }
    friend class KmerMap;

   public:
    iter() = default;
    iter(M *m, size_t i, bool do_skip) : m_(m), i_(i) {
      if (do_skip) skip();
    }
    operator iter<true>() const { return iter<true>(m_, i_, false); }
    V &operator*() const { return m_->slot_[i_]; }
    V *operator->() const { return &m_->slot_[i_]; }
    iter &operator++() {
      i_++;
      skip();
      return *this;
    }
    iter operator++(int) {
      iter t = *this;
      ++*this;
      return t;
    }
    bool operator==(const iter &o) const { return i_ == o.i_; }
    bool operator!=(const iter &o) const { return i_ != o.i_; }
  };
  using iterator = iter<false>;
  using const_iterator = iter<true>;

  KmerMap() = default;
  // not copyable (two buffers of up to tens of GB); a move leaves the source an empty map that can be used again
  KmerMap(const KmerMap &) = delete;
  KmerMap &operator=(const KmerMap &) = delete;
  KmerMap(KmerMap &&o) noexcept { swap(o); }
  KmerMap &operator=(KmerMap &&o) noexcept {
    if (this != &o) {
      KmerMap t;
      t.swap(o);
      swap(t);
    }
    return *this;
  }
  size_t size() const { return size_; }
  bool empty() const { return size_ == 0; }
  size_t bucket_count() const { return cap_; }
  iterator begin() { return iterator(this, 0, true); }
  iterator end() { return iterator(this, cap_, false); }
  const_iterator begin() const { return const_iterator(this, 0, true); }
  const_iterator end() const { return const_iterator(this, cap_, false); }
  void clear() {
    if (cap_) std::memset(tag_.get(), 0, cap_);
    size_ = 0;
  }
  void swap(KmerMap &o) {
    std::swap(tag_, o.tag_);
    std::swap(slot_, o.slot_);
    std::swap(cap_, o.cap_);
    std::swap(size_, o.size_);
    std::swap(shift_, o.shift_);
  }
  void reserve(size_t n) {
    size_t c = 16;
    while (c - c / 8 < n) c <<= 1;
    if (c > cap_) rehash(c);
  }

  iterator find(const key_type &k) {
    if (!cap_) return end();
    const size_t i = locate(k, hash_of(k));
    return iterator(this, tag_[i] ? i : cap_, false);
  }
  const_iterator find(const key_type &k) const {
    const size_t i = cap_ ? const_cast<KmerMap *>(this)->locate(k, hash_of(k)) : 0;
    return const_iterator(this, cap_ && tag_[i] ? i : cap_, false);
  }
  size_t count(const key_type &k) const { return find(k) != end(); }
  std::pair<iterator, bool> emplace(const key_type &k, const mapped_type &v) { return put(k, v, hash_of(k)); }
  std::pair<iterator, bool> insert(const value_type &kv) { return put(kv.first, kv.second, hash_of(kv.first)); }
  mapped_type &operator[](const key_type &k) { return put(k, mapped_type(), hash_of(k)).first->second; }

  // Bulk insert of n finished rows in mhmkc_fetch's layout (keys: N_LONGS words per row). Rows whose key is
  // already present keep the present entry (as insert does). fill = fill_begin + one fill_chunk + fill_end.
  void fill(const uint64_t *keys, const uint16_t *counts, const char *left, const char *right, uint64_t n,
            int threads = 0) {
    fill_begin(n, threads);
    fill_chunk(keys, counts, left, right, n);
    fill_end();
  }

  // A bulk insert in chunks, in order (a table streamed from the device chunk by chunk: HashTableInserter's
  // insert_into_local_hashtable): fill_begin(rows in all chunks), fill_chunk per chunk, fill_end. Into an empty map,
  // rows in mhmkc_fetch_ordered's order (non-decreasing home slot) are placed by `threads` threads (0: fill_threads())
  // without probing (chunk_ordered); from the first chunk that is not in that order on, rows go through the one-thread
  // prefetched loop (chunk_loop).
  void fill_begin(uint64_t n, int threads = 0) {
    reserve(size_ + n);
    fs_threads_ = threads > 0 ? threads : fill_threads();
    fs_ordered_ = size_ == 0 && fs_threads_ > 1 && cap_ <= (1ull << 32);
    fs_pos_ = -1;
    fs_prev32_ = 0;
    fs_any_ = false;
    fs_wrapped_.clear();
    fs_pool_.reset();
    if (fs_threads_ > 1) fs_pool_.reset(new FillPool(fs_threads_));
    fs_hash_.resize(fs_threads_);
  }
  void fill_chunk(const uint64_t *keys, const uint16_t *counts, const char *left, const char *right, uint64_t n) {
    if (!n) return;
    if (fs_ordered_) {
      if (chunk_ordered(keys, counts, left, right, n)) return;
      fs_ordered_ = false;
      flush_wrapped();  // (the rows of earlier chunks go in first, so that a repeated key keeps its first entry)
    }
    chunk_loop(keys, counts, left, right, n);
  }
  // fill_begin left the map ready for fill_chunk_slots: it was empty, the fill has several threads, and it has at most
  // 2^32 slots
  bool fill_by_slots() const { return fs_ordered_ && fs_pool_ != nullptr; }
  // Rows with the slots and tags mhmkc_fetch_map_range computed on the device for this map's capacity (bucket_count()
  // after fill_begin), in that order (the rows of all chunks, each chunk in turn): the fill threads write each row
  // straight to its slot in one pass, with no hashing and no probing on the host; a row whose slot is 0xFFFFFFFF (past
  // the last slot) is placed by put() at fill_end. The rows' keys must be unique (a finished table's are). Only between
  // fill_begin and fill_end of a map for which fill_by_slots() is true, and not mixed with fill_chunk in one fill.
  void fill_chunk_slots(const uint64_t *keys, const uint16_t *counts, const char *left, const char *right,
                        const uint32_t *slots, const uint8_t *tags, uint64_t n) {
    if (!n) return;
    if (!fill_by_slots()) die("KmerMap::fill_chunk_slots: the map was not empty at fill_begin, or one fill thread");
    const int nl = key_type::N_LONGS;
    const int T = (int)std::min<uint64_t>((uint64_t)fs_pool_->size(), n / 4096 + 1);
    std::vector<std::vector<uint64_t>> wrapped(T);
    std::vector<uint64_t> placed(T, 0);
    const std::function<void(int)> worker = [&](int t) {
      if (t >= T) return;
      const uint64_t a = n * (uint64_t)t / (uint64_t)T, b = n * (uint64_t)(t + 1) / (uint64_t)T;
      uint64_t m = 0;
      for (uint64_t i = a; i < b; i++) {
        const uint32_t p = slots[i];
        if (p == 0xffffffffu || p >= cap_) {
          wrapped[t].push_back(i);
          continue;
        }
        tag_[p] = tags[i];
        value_type &v = slot_[p];
        v.first = key_type(keys + i * nl);
        v.second = KmerCounts();
        v.second.count = counts[i];
        v.second.left = left[i];
        v.second.right = right[i];
        m++;
      }
      placed[t] = m;
    };
    fs_pool_->run(worker);
    for (int t = 0; t < T; t++) {
      size_ += placed[t];
      for (uint64_t i : wrapped[t]) {
        KmerCounts kc;
        kc.count = counts[i];
        kc.left = left[i];
        kc.right = right[i];
        fs_wrapped_.emplace_back(key_type(keys + i * nl), kc);
      }
    }
  }
  void fill_end() {
    flush_wrapped();
    fs_pool_.reset();
    fs_hash_.clear();
    fs_hash_.shrink_to_fit();
  }

  // Threads of a bulk fill: OMP_NUM_THREADS when set (the rank's CPU share), else the CPUs this process may run on
  // (its affinity mask: a rank pinned to its share of the node's cores fills with that many), at most 16.
  static int fill_threads() {
    if (const char *e = getenv("OMP_NUM_THREADS"))
      if (atoi(e) > 0) return std::min(64, atoi(e));
    cpu_set_t cs;
    int cpus = 0;
    if (sched_getaffinity(0, sizeof cs, &cs) == 0) cpus = CPU_COUNT(&cs);
    if (cpus <= 0) cpus = (int)std::thread::hardware_concurrency();
    return std::max(1, std::min(16, cpus));
  }

 private:
  // the one-thread insert loop, three stages per row: A (row i + kAhead2) hashes the key and prefetches its home tags;
  // B (row i + kAhead1) scans the tags, now cached, for the slot the insert will take (the end of the probe run: at load
  // 3/4 it is several cache lines past the home slot) and prefetches that slot; C (row i) inserts
  void chunk_loop(const uint64_t *keys, const uint16_t *counts, const char *left, const char *right, uint64_t n) {
    constexpr int kAhead2 = 48, kAhead1 = 16, kRing = 64;
    uint64_t h[kRing];
    const int nl = key_type::N_LONGS;
    auto stage_a = [&](uint64_t j) {
      h[j % kRing] = hash_words(keys + j * nl);
      __builtin_prefetch(&tag_[home(h[j % kRing])], 1, 1);
    };
    auto stage_b = [&](uint64_t j) {
      const uint64_t hj = h[j % kRing];
      const uint8_t t = tag_of(hj);
      size_t i = home(hj);
      for (int q = 0; q < 64 && tag_[i] && tag_[i] != t; q++) i = (i + 1) & (cap_ - 1);
      __builtin_prefetch(&slot_[i], 1, 1);
    };
    for (uint64_t j = 0; j < n && j < (uint64_t)kAhead2; j++) stage_a(j);
    for (uint64_t j = 0; j < n && j < (uint64_t)kAhead1; j++) stage_b(j);
    for (uint64_t i = 0; i < n; i++) {
      if (i + kAhead2 < n) stage_a(i + kAhead2);
      if (i + kAhead1 < n) stage_b(i + kAhead1);
      KmerCounts kc;
      kc.count = counts[i];
      kc.left = left[i];
      kc.right = right[i];
      put(key_type(keys + i * nl), kc, h[i % kRing]);
    }
  }

  // Parallel placement of rows sorted by home slot (mhmkc_fetch_ordered: the top 32 bits of the hash, which order the
  // homes for any capacity up to 2^32) into a map that holds only the earlier such rows. Linear probing that inserts in
  // home order puts row i at
  //     pos_i = max(home_i, pos_{i-1} + 1)
  // (the first free slot at or after its home: every slot of [home_i, pos_{i-1}] is taken by earlier rows), so the
  // positions are a running maximum: over a range of rows with the position c of the row before it,
  //     pos_last = max(c + n_range, pos_last with no row before it),
  // and threads over contiguous row ranges need only the ranges' two numbers, combined in order, to place every row
  // (fs_pos_ carries c from chunk to chunk). Each thread then writes a disjoint slot range (the positions increase).
  // Rows placed past the last slot wrap to the front, where linear probing continues: those few go through put() at
  // fill_end. A row whose key equals an earlier row's (the same top-32 hash bits, so within a few rows) keeps the
  // earlier entry, as insert does. Returns false, with nothing written, when the rows are not in home order.
  bool chunk_ordered(const uint64_t *keys, const uint16_t *counts, const char *left, const char *right, uint64_t n) {
    const int nl = key_type::N_LONGS;
    const int T = (int)std::min<uint64_t>((uint64_t)(fs_pool_ ? fs_pool_->size() : 1), n / 4096 + 1);
    struct Part {
      int64_t last = -1;  // pos of the range's last row with nothing before it (-1: no row)
      uint64_t rows = 0;  // rows that take a slot (not repeats)
      bool sorted = true;
      std::vector<uint64_t> wrapped;  // rows placed past the last slot
    };
    std::vector<Part> part(T);
    auto lo_of = [&](int t) { return n * (uint64_t)t / (uint64_t)T; };
    auto hash32 = [&](uint64_t i) { return hash_words(keys + i * nl) >> 32; };
    auto same = [&](uint64_t i, uint64_t j) { return std::memcmp(keys + j * nl, keys + i * nl, 8 * (size_t)nl) == 0; };
    // the chunk's leading rows with the previous chunk's last top bits may repeat a row already in the map: decided
    // here, before any thread writes
    std::vector<uint8_t> lead;
    if (fs_any_)
      for (uint64_t i = 0; i < n; i++) {
        const uint64_t hw = hash_words(keys + i * nl);
        if ((hw >> 32) != fs_prev32_) break;
        const key_type ki(keys + i * nl);
        bool d = tag_[locate(ki, hw)] != 0;
        // (an earlier chunk's row placed past the last slot waits in fs_wrapped_, not yet in the map)
        for (size_t j = fs_wrapped_.size(); j-- > 0 && !d;) d = fs_wrapped_[j].first == ki;
        for (uint64_t j = 0; j < i && !d; j++) d = same(i, j);
        lead.push_back(d);
      }
    // row i repeats an earlier row of the chunk (equal keys have equal hashes: one run of equal top bits)
    auto repeat = [&](uint64_t i, uint64_t h32) {
      if (i < lead.size()) return lead[i] != 0;
      for (uint64_t j = i; j-- > 0;) {
        if (hash32(j) != h32) return false;
        if (same(i, j)) return true;
      }
      return false;
    };
    // (pass 1 keeps each row's hash for pass 2 in its thread's buffer)
    auto run = [&](int t, bool place, int64_t carry) {
      Part &p = part[t];
      const uint64_t a = lo_of(t), b = lo_of(t + 1);
      std::vector<uint64_t> &hb = fs_hash_[t];
      if (!place && hb.size() < b - a) hb.resize(b - a);
      uint64_t prev = a ? hash32(a - 1) : fs_prev32_;
      int64_t pos = place ? carry : -1;
      for (uint64_t i = a; i < b; i++) {
        const uint64_t hw = place ? hb[i - a] : (hb[i - a] = hash_words(keys + i * nl)), h32 = hw >> 32;
        if (h32 < prev) {
          p.sorted = false;
          return;
        }
        const bool maybe = i < lead.size() || (i > 0 && h32 == prev);
        prev = h32;
        if (maybe && repeat(i, h32)) continue;
        pos = std::max<int64_t>((int64_t)home(hw), pos + 1);
        if (!place) {
          p.rows++;
          continue;
        }
        if ((uint64_t)pos >= cap_) {
          p.wrapped.push_back(i);
          continue;
        }
        tag_[pos] = tag_of(hw);
        slot_[pos].first = key_type(keys + i * nl);
        KmerCounts &kc = slot_[pos].second;
        kc = KmerCounts();
        kc.count = counts[i];
        kc.left = left[i];
        kc.right = right[i];
      }
      if (!place) p.last = pos;
    };
    // one thread per range for both passes: the ranges' numbers are combined by thread 0 between them
    std::vector<int64_t> carry(T + 1, fs_pos_);
    std::atomic<int> arrived{0};
    std::atomic<int> go{0};  // 1: carries ready, 2: not in order (no second pass)
    const std::function<void(int)> worker = [&](int t) {
      if (t >= T) return;
      run(t, false, 0);
      arrived.fetch_add(1);
      if (t == 0) {
        while (arrived.load() < T) std::this_thread::yield();
        bool sorted = true;
        for (auto &p : part) sorted &= p.sorted;
        for (int u = 1; u <= T; u++)  // the carry into each range: the position of the last row before it
          carry[u] = std::max<int64_t>(carry[u - 1] + (int64_t)part[u - 1].rows, part[u - 1].last);
        go.store(sorted ? 1 : 2);
      } else {
        while (!go.load()) std::this_thread::yield();
      }
      if (go.load() == 1) run(t, true, carry[t]);
    };
    if (fs_pool_) {
      fs_pool_->run(worker);
    } else {
      std::vector<std::thread> th;
      for (int t = 1; t < T; t++) th.emplace_back(worker, t);
      worker(0);
      for (auto &x : th) x.join();
    }
    if (go.load() != 1) return false;
    for (auto &p : part) {
      size_ += p.rows - p.wrapped.size();
      for (uint64_t i : p.wrapped) {
        KmerCounts kc;
        kc.count = counts[i];
        kc.left = left[i];
        kc.right = right[i];
        fs_wrapped_.emplace_back(key_type(keys + i * nl), kc);
      }
    }
    fs_pos_ = carry[T];
    fs_prev32_ = hash32(n - 1);
    fs_any_ = true;
    return true;
  }
  void flush_wrapped() {
    for (auto &kv : fs_wrapped_) put(kv.first, kv.second, hash_of(kv.first));
    fs_wrapped_.clear();
  }

  // tags and slots of a large map live in 2 MB-aligned anonymous memory advised for transparent huge pages: a table
  // larger than the caches is touched at random, and with 4 KB pages every probe would also miss the TLB. Below 1 MB
  // (a small map: a test, a tiny rank share) plain zeroed heap memory.
  struct Free {
    size_t bytes = 0;  // 0: from calloc
    void operator()(void *p) const {
      if (!p) return;
      if (bytes)
        munmap(p, bytes);
      else
        std::free(p);
    }
  };
  template <typename T>
  using Buf = std::unique_ptr<T[], Free>;
  template <typename T>
  static Buf<T> alloc(size_t n) {
    if (n * sizeof(T) < (1u << 20)) {
      void *p = std::calloc(n ? n : 1, sizeof(T));
      if (!p) die("KmerMap: out of memory");
      return Buf<T>((T *)p, Free{0});
    }
    const size_t bytes = ((n * sizeof(T)) + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
    void *p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) die("KmerMap: out of memory");
    (void)madvise(p, bytes, MADV_HUGEPAGE);
    return Buf<T>((T *)p, Free{bytes});  // zero-filled by the kernel; value_type is trivially copyable
  }
  Buf<uint8_t> tag_;
  Buf<value_type> slot_;
  size_t cap_ = 0, size_ = 0;
  int shift_ = 64;  // 64 - log2(cap_): the home slot is the top bits of the hash
  // state of a chunked fill (fill_begin .. fill_end)
  int fs_threads_ = 1;
  bool fs_ordered_ = false, fs_any_ = false;
  int64_t fs_pos_ = -1;     // position of the last row placed in order (-1: none)
  uint64_t fs_prev32_ = 0;  // the top 32 hash bits of the last row of the previous chunk
  std::vector<value_type> fs_wrapped_;
  std::unique_ptr<FillPool> fs_pool_;            // the fill's worker threads
  std::vector<std::vector<uint64_t>> fs_hash_;  // per fill thread: its rows' hashes (pass 1 -> pass 2)
  // the key words' multiply-xorshift mix (mhmkc_map_hash: the device orders mhmkc_fetch_ordered's rows by its top
  // bits, the home slot here, so that a fill in that order streams through the slot array)
  static uint64_t hash_words(const uint64_t *w) { return mhmkc_map_hash(w, key_type::N_LONGS); }
  static uint64_t hash_of(const key_type &k) { return hash_words(k.get_longs()); }
  static uint8_t tag_of(uint64_t h) { return (uint8_t)(0x80u | (h & 0x7fu)); }
  size_t home(uint64_t h) const { return (size_t)(h >> shift_); }
  // the slot holding k, or the empty slot ending its probe sequence (cap_ > 0, load < 1). Eight tags per step
  // (SWAR zero-byte tests on a 64-bit load: the first empty tag and the tag matches), one at a time at the wrap.
  size_t locate(const key_type &k, uint64_t h) {
    const uint8_t t = tag_of(h);
    constexpr uint64_t L1 = 0x0101010101010101ull, H8 = 0x8080808080808080ull;
    size_t i = home(h);
    while (true) {
      if (i + 8 <= cap_) {
        uint64_t x;
        std::memcpy(&x, &tag_[i], 8);
        const uint64_t y = x ^ (L1 * t);
        const uint64_t zero = (x - L1) & ~x & H8;  // bytes that are empty (exact below the first one)
        uint64_t match = (y - L1) & ~y & H8;       // bytes equal to t (exact below the first one)
        const int first_empty = zero ? __builtin_ctzll(zero) >> 3 : 8;
        while (match) {
          const int b = __builtin_ctzll(match) >> 3;
          if (b >= first_empty) break;
          if (tag_[i + b] == t && slot_[i + b].first == k) return i + b;
          match &= match - 1;
        }
        if (first_empty < 8) return i + first_empty;
        i = (i + 8) & (cap_ - 1);
      } else {
        if (!tag_[i]) return i;
        if (tag_[i] == t && slot_[i].first == k) return i;
        i = (i + 1) & (cap_ - 1);
      }
    }
  }
  std::pair<iterator, bool> put(const key_type &k, const mapped_type &v, uint64_t h) {
    if (size_ + 1 > cap_ - cap_ / 8) rehash(cap_ ? 2 * cap_ : 16);
    const size_t i = locate(k, h);
    if (tag_[i]) return {iterator(this, i, false), false};
    tag_[i] = tag_of(h);
    slot_[i].first = k;
    slot_[i].second = v;
    size_++;
    return {iterator(this, i, false), true};
  }
  void rehash(size_t c) {
    Buf<uint8_t> ot = alloc<uint8_t>(c);
    Buf<value_type> os = alloc<value_type>(c);
    ot.swap(tag_);
    os.swap(slot_);
    const size_t oc = cap_;
    cap_ = c;
    shift_ = 64 - __builtin_ctzll((unsigned long long)c);
    size_ = 0;
    for (size_t i = 0; i < oc; i++)
      if (ot[i]) put(os[i].first, os[i].second, hash_of(os[i].first));
  }
};

// ---------------------------------------------------------------------------------------------
// PackedReads (byte layout of src/packed_reads.cpp:73-109)

class PackedReads {
  std::vector<uint8_t> bytes_;
  std::vector<uint64_t> offsets_{0};
  int qual_offset_;

 public:
  explicit PackedReads(int qual_offset) : qual_offset_(qual_offset) {}
  void add_read(const std::string & /*read_id*/, const std::string &seq, const std::string &quals) {
    if (seq.size() > 65535) die("read longer than 65535");
    for (size_t i = 0; i < seq.size(); i++) {
      uint8_t code;
      switch (seq[i]) {
        case 'A': code = 0; break;
        case 'C': code = 1; break;
        case 'G': code = 2; break;
        case 'T': code = 3; break;
        case 'N': case 'U': case 'R': case 'Y': case 'K': case 'M': case 'S':
        case 'W': case 'B': case 'D': case 'H': case 'V': code = 4; break;
        default: die(std::string("Illegal char in comp nucleotide of '") + seq[i] + "'");
      }
      int q = quals[i] - qual_offset_;
      bytes_.push_back((uint8_t)(code | ((unsigned char)(q < 31 ? q : 31) << 3)));
    }
    offsets_.push_back(bytes_.size());
  }
  // the reads packed on the device by mhmkc_add_fastq (HashTableInserter::fastq_packed_reads)
  void assign(std::vector<uint8_t> bytes, std::vector<uint64_t> offsets) {
    bytes_ = std::move(bytes);
    offsets_ = std::move(offsets);
  }
  int get_qual_offset() const { return qual_offset_; }
  int64_t get_local_num_reads() const { return (int64_t)offsets_.size() - 1; }
  const uint8_t *bytes() const { return bytes_.data(); }
  const uint64_t *offsets() const { return offsets_.data(); }
};

struct Contig {
  int64_t id;
  std::string seq;
  double depth;
  uint16_t get_uint16_t_depth() const { return (depth > UINT16_MAX ? UINT16_MAX : depth); }  // contigs.hpp:65
};
using Contigs = std::vector<Contig>;

// ---------------------------------------------------------------------------------------------
// HashTableInserter / KmerDHT / SeqBlockInserter

// Where this rank sits. n_ranks > 1: the exchange runs over RCCL (comm_id from mhmkc_comm_id on rank 0,
// broadcast by the host) or over the host's own transport (UPC++ / MPI, mhmkc_set_transport), and the
// finished k-mers end on the reference's owner rank (get_kmer_target_rank), where dbjg looks them up.
struct RankInfo {
  int rank = 0, n_ranks = 1;
  const uint8_t *comm_id = nullptr;
  const mhmkc_transport *transport = nullptr;
  int device = -1;
  int output_owner = MHMKC_OWNER_MINIMIZER;
  bool table_only = false;  // no counter: the KmerDHT only holds a table given to load_table (no GPU used)
};

// The finished table of a handle into `map`, streamed in the KmerMap's slot order (mhmkc_fetch_ordered_range):
// while chunk c is placed by KmerMap::fill_chunk, a helper thread copies chunk c + 1 from the device, so the D2H hides
// behind the fill and the host never holds the whole table outside the map. Replaces insert_into_local_hashtable's
// loop over the local table (src/kcount/kcount_cpu.cpp:503-522).
// where load_ordered's time went (milliseconds; optional)
struct LoadTimes {
  double first_fetch = 0, fill = 0, wait_fetch = 0;
  double begin = 0, end = 0;  // the chunk buffers + fill_begin (map allocation, fill threads); fill_end
};

template <int MAX_K>
void load_ordered(mhmkc_t h, KmerMap<MAX_K> &map, uint64_t n, int threads = 0, uint64_t chunk_rows = 4u << 20,
                  LoadTimes *times = nullptr) {
  using clk = std::chrono::steady_clock;
  auto ms_since = [](clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); };
  LoadTimes lt;
  const auto tb = clk::now();
  const int nl = Kmer<MAX_K>::N_LONGS;
  const uint64_t m = std::min<uint64_t>(std::max<uint64_t>(chunk_rows, 1), std::max<uint64_t>(n, 1));
  // a chunk's arrays in one block of pinned host memory from the library (one DMA per array straight into it, and the
  // block reused by the next hand-off), else of the heap (then the fetch copies through the library's staging)
  struct Block {
    void *p = nullptr;
    bool pinned = false;
    ~Block() {
      if (pinned)
        mhmkc_host_free(p);
      else
        delete[] (char *)p;
    }
  };
  struct Chunk {  // (not zero-filled: the fetch writes every row it is read for)
    Block blk;
    uint64_t *keys = nullptr;
    uint16_t *counts = nullptr;
    char *left = nullptr, *right = nullptr;
    uint32_t *slots = nullptr;
    uint8_t *tags = nullptr;
  } buf[2];
  map.fill_begin(n, threads);
  // into an empty map (the usual case): each row's slot and tag come from the device (mhmkc_fetch_map_range, a prefix
  // maximum over the ordered rows' home slots), and the fill threads write the rows straight to their slots
  const bool by_slots = map.fill_by_slots();
  const uint64_t cap = map.bucket_count();
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const size_t kb = al(m * 8 * nl), cb = al(m * 2), lb = al(m), sb = by_slots ? al(m * 4) : 0, gb = by_slots ? al(m) : 0;
  for (auto &b : buf) {
    const size_t tot = kb + cb + 2 * lb + sb + gb;
    b.blk.p = mhmkc_host_alloc(tot);
    b.blk.pinned = b.blk.p != nullptr;
    if (!b.blk.p) b.blk.p = new char[tot];
    char *q = (char *)b.blk.p;
    b.keys = (uint64_t *)q;
    b.counts = (uint16_t *)(q + kb);
    b.left = q + kb + cb;
    b.right = q + kb + cb + lb;
    if (by_slots) {
      b.slots = (uint32_t *)(q + kb + cb + 2 * lb);
      b.tags = (uint8_t *)(q + kb + cb + 2 * lb + sb);
    }
  }
  auto fetch = [&](uint64_t c) {
    Chunk &b = buf[c & 1];
    const uint64_t r0 = c * m;
    if (by_slots)
      return mhmkc_fetch_map_range(h, cap, r0, std::min(m, n - r0), b.keys, b.counts, b.left, b.right, b.slots, b.tags);
    return mhmkc_fetch_ordered_range(h, r0, std::min(m, n - r0), b.keys, b.counts, b.left, b.right);
  };
  const uint64_t n_ch = (n + m - 1) / m;
  // (the map's fresh memory is faulted in by the fill threads as they write it: a separate parallel pass to fault it in
  // while the first chunk was on the wire measured no faster)
  lt.begin = ms_since(tb);
  auto t0 = clk::now();
  int rc = n_ch ? fetch(0) : MHMKC_OK;
  lt.first_fetch = ms_since(t0);
  // the prefetch thread is joined on every way out of an iteration (a fill that throws would otherwise destroy a
  // joinable std::thread: std::terminate)
  struct Joiner {
    std::thread t;
    ~Joiner() {
      if (t.joinable()) t.join();
    }
  };
  for (uint64_t c = 0; c < n_ch; c++) {
    check(rc, h, "mhmkc_fetch_ordered_range");
    int rc_next = MHMKC_OK;
    Joiner jf;
    std::thread &f = jf.t;
    if (c + 1 < n_ch) f = std::thread([&, c] { rc_next = fetch(c + 1); });
    const Chunk &b = buf[c & 1];
    auto t1 = clk::now();
    if (by_slots)
      map.fill_chunk_slots(b.keys, b.counts, b.left, b.right, b.slots, b.tags, std::min(m, n - c * m));
    else
      map.fill_chunk(b.keys, b.counts, b.left, b.right, std::min(m, n - c * m));
    lt.fill += ms_since(t1);
    t1 = clk::now();
    if (f.joinable()) f.join();
    lt.wait_fetch += ms_since(t1);
    rc = rc_next;
  }
  auto t2 = clk::now();
  map.fill_end();
  lt.end = ms_since(t2);
  if (times) *times = lt;
}

template <int MAX_K>
class HashTableInserter {
  mhmkc_t h_ = nullptr;
  std::string seq_buf_, ctg_buf_;
  std::vector<uint64_t> seq_offs_{0}, ctg_offs_{0};
  std::vector<uint16_t> ctg_depths_;
  bool using_ctg_kmers_ = false;

 public:
  HashTableInserter() = default;
  ~HashTableInserter() { mhmkc_destroy(h_); }
  HashTableInserter(const HashTableInserter &) = delete;
  HashTableInserter &operator=(const HashTableInserter &) = delete;

  // kcount_cpu.cpp:425-443; the estimate only sized the CPU table, the GPU path sizes itself exactly. The
  // depth threshold is not known yet: analyze_kmers sets _dmin_thres later (kcount.cpp:145).
  void init(int /*num_elems*/, bool /*use_qf*/, const RankInfo &ri = RankInfo()) {
    if (ri.table_only) return;
    mhmkc_config cfg;
    mhmkc_config_init(&cfg);
    cfg.k = (int)Kmer<MAX_K>::get_k();
    cfg.n_longs = Kmer<MAX_K>::N_LONGS;
    cfg.rank = ri.rank;
    cfg.n_ranks = ri.n_ranks;
    cfg.comm_id = ri.comm_id;
    cfg.device = ri.device;
    cfg.output_owner = ri.output_owner;
    check(mhmkc_create(&h_, &cfg), nullptr, "mhmkc_create");
    if (ri.n_ranks > 1 && !ri.comm_id) {
      if (!ri.transport) die("n_ranks > 1 needs RankInfo::comm_id or RankInfo::transport");
      check(mhmkc_set_transport(h_, ri.transport), h_, "mhmkc_set_transport");
    }
  }
  // kcount_cpu.cpp:445-448: later supermers are contig supermers (insert_supermer_from_ctg)
  void init_ctg_kmers(int /*max_elems*/) {
    flush_inserts();
    using_ctg_kmers_ = true;
  }

  // kcount_cpu.cpp:450-463 (buffered; flushed in flush_inserts). Read supermers have count 1; contig
  // supermers carry the contig depth and are applied after every read, in order (mhmkc_add_ctgs).
  void insert_supermer(const std::string &supermer_seq, kmer_count_t count) {
    if (using_ctg_kmers_) {
      ctg_buf_ += supermer_seq;
      ctg_offs_.push_back(ctg_buf_.size());
      ctg_depths_.push_back(count);
      return;
    }
    if (count > 1) die("read supermer with count > 1");
    seq_buf_ += supermer_seq;
    seq_offs_.push_back(seq_buf_.size());
  }
  void add_packed_reads(const PackedReads &pr) {
    check(mhmkc_add_reads(h_, pr.bytes(), pr.offsets(), (uint64_t)pr.get_local_num_reads()), h_, "mhmkc_add_reads");
  }
  // FASTQ text parsed and packed on the device (FastqReader + PackedRead, src/fastq.cpp:504-551,
  // src/packed_reads.cpp:73-109), then counted; malformed input DIEs as the reference does
  void add_fastq(const std::string &text) {
    check(mhmkc_add_fastq(h_, text.data(), text.size()), h_, "mhmkc_add_fastq");
  }
  // a FASTQ file read in blocks, each parsed and counted on the device while the next is read
  void add_fastq_file(const std::string &path, bool pairs = false) {
    check(pairs ? mhmkc_add_fastq_pairs_file(h_, path.c_str()) : mhmkc_add_fastq_file(h_, path.c_str()), h_,
          "mhmkc_add_fastq_file");
  }
  // the PackedReads of the last add_fastq, copied back (for a host that keeps them, as main.cpp does)
  void fastq_packed_reads(PackedReads &pr) const {
    uint64_t n_reads = 0, n_bases = 0;
    check(mhmkc_fastq_packed(h_, nullptr, nullptr, &n_reads, &n_bases), h_, "mhmkc_fastq_packed");
    std::vector<uint8_t> b(n_bases);
    std::vector<uint64_t> o(n_reads + 1);
    check(mhmkc_fastq_fetch(h_, b.data(), o.data()), h_, "mhmkc_fastq_fetch");
    pr.assign(std::move(b), std::move(o));
  }
  void flush_inserts() {
    if (seq_offs_.size() > 1) {
      check(mhmkc_add_seqs(h_, seq_buf_.data(), seq_offs_.data(), seq_offs_.size() - 1, 1), h_, "mhmkc_add_seqs");
      seq_buf_.clear();
      seq_offs_.assign(1, 0);
    }
    if (ctg_offs_.size() > 1) {
      check(mhmkc_add_ctgs(h_, ctg_buf_.data(), ctg_offs_.data(), ctg_depths_.data(), ctg_offs_.size() - 1), h_,
            "mhmkc_add_ctgs");
      ctg_buf_.clear();
      ctg_offs_.assign(1, 0);
      ctg_depths_.clear();
    }
  }
  // kcount_cpu.cpp:490-528 (get_ext reads the global _dmin_thres at this point, :178)
  void insert_into_local_hashtable(KmerMap<MAX_K> &local_kmers) {
    flush_inserts();
    check(mhmkc_set_dmin_thres(h_, _dmin_thres), h_, "mhmkc_set_dmin_thres");
    uint64_t n = 0;
    check(mhmkc_finish(h_, &n), h_, "mhmkc_finish");
    // rows in the map's slot order (a device sort), chunk by chunk, each placed while the next is copied
    load_ordered(h_, local_kmers, n);
  }
  mhmkc_stats stats() const {
    mhmkc_stats s;
    check(mhmkc_get_stats(h_, &s), h_, "mhmkc_get_stats");
    return s;
  }
};

template <int MAX_K>
class KmerDHT {
  KmerMap<MAX_K> local_kmers;
  HashTableInserter<MAX_K> ht_inserter;
  RankInfo ri;
  int minimizer_len;

 public:
  // src/kcount/kmer_dht.cpp:106-154: the same arguments (the store sizes and RPC limits have no meaning
  // without UPC++'s aggregation stores; the estimate only sized the CPU table) + where this rank sits
  KmerDHT(uint64_t my_num_kmers, int /*max_kmer_store_bytes*/, int /*max_rpcs_in_flight*/, bool /*useHHSS*/,
          bool use_qf, const RankInfo &rank_info = RankInfo())
      : ri(rank_info) {
    minimizer_len = std::min(27, std::max(15, (int)Kmer<MAX_K>::get_k() * 2 / 3 + 1));
    if (use_qf) my_num_kmers = (uint64_t)(my_num_kmers * 0.6);
    ht_inserter.init((int)my_num_kmers, use_qf, ri);
  }
  int get_minimizer_len() const { return minimizer_len; }
  void add_supermer(const std::string &seq, kmer_count_t count) { ht_inserter.insert_supermer(seq, count); }
  void init_ctg_kmers(int max_elems) { ht_inserter.init_ctg_kmers(max_elems); }  // kmer_dht.cpp:169-172
  void add_packed_reads(const PackedReads &pr) { ht_inserter.add_packed_reads(pr); }
  void add_fastq(const std::string &text) { ht_inserter.add_fastq(text); }
  void add_fastq_file(const std::string &path, bool pairs = false) { ht_inserter.add_fastq_file(path, pairs); }
  void flush_updates() { ht_inserter.flush_inserts(); }
  void finish_updates() { ht_inserter.insert_into_local_hashtable(local_kmers); }
  // fill the local KmerMap from a finished table in mhmkc_fetch's layout (n_longs = N_LONGS words per key)
  void load_table(const uint64_t *keys, const uint16_t *counts, const char *left, const char *right, uint64_t n) {
    local_kmers.fill(keys, counts, left, right, n);
  }
  KmerCounts *get_local_kmer_counts(const Kmer<MAX_K> &kmer) {
    auto it = local_kmers.find(kmer);
    return it == local_kmers.end() ? nullptr : &it->second;
  }
  // src/kcount/kmer_dht.cpp:193-196: minimizer_hash_fast(minimizer_len) % rank_n (the same for a k-mer and its
  // reverse complement); after finish every local k-mer satisfies it (MHMKC_OWNER_MINIMIZER)
  int get_kmer_target_rank(const Kmer<MAX_K> &kmer) const {
    return (int)(kmer.minimizer_hash_fast(minimizer_len) % (uint64_t)ri.n_ranks);
  }
  int64_t get_local_num_kmers() const { return (int64_t)local_kmers.size(); }
  typename KmerMap<MAX_K>::iterator local_kmers_begin() { return local_kmers.begin(); }
  typename KmerMap<MAX_K>::iterator local_kmers_end() { return local_kmers.end(); }
  HashTableInserter<MAX_K> &inserter() { return ht_inserter; }
  // src/kcount/kmer_dht.cpp:243-266: kmers-<k>.txt.gz in the rank's directory (get_rank_path,
  // upcxx-utils/src/log.cpp:283-312: <dir>/per_rank/<rank / 1000, 8 digits>/<rank, 8 digits>/), one
  // "KMER count L R" line per k-mer, gzip (the reference writes through zstr)
  std::string dump_kmers(const std::string &dir = ".") {
    char sub[64];
    std::snprintf(sub, sizeof sub, "%08d/%08d", ri.rank / 1000, ri.rank);
    std::string path = dir + "/per_rank";
    for (const std::string &d : {path, path + "/" + std::string(sub, 8), path + "/" + std::string(sub)}) mkdir(d.c_str(), 0777);
    path += "/" + std::string(sub) + "/kmers-" + std::to_string(Kmer<MAX_K>::get_k()) + ".txt.gz";
    gzFile f = gzopen(path.c_str(), "wb");
    if (!f) die("cannot open " + path);
    std::string buf;
    int64_t i = 0;
    for (auto &e : local_kmers) {
      buf += e.first.to_string() + " " + std::to_string(e.second.count) + " " + e.second.left + " " + e.second.right + "\n";
      if (!(++i % 1000)) {
        if (gzwrite(f, buf.data(), (unsigned)buf.size()) != (int)buf.size()) die("gzwrite " + path);
        buf.clear();
      }
    }
    if (!buf.empty() && gzwrite(f, buf.data(), (unsigned)buf.size()) != (int)buf.size()) die("gzwrite " + path);
    if (gzclose(f) != Z_OK) die("gzclose " + path);
    return path;
  }
};

template <int MAX_K>
struct SeqBlockInserter {
  SeqBlockInserter(int /*qual_offset*/, int /*minimizer_len*/) {}
  // kcount_cpu.cpp:73-103 at one rank: the whole sequence is one supermer when it has >= k+2 bases
  void process_seq(std::string &seq, kmer_count_t depth, KmerDHT<MAX_K> &dht) {
    if (!depth) depth = 1;
    if (seq.length() >= Kmer<MAX_K>::get_k() + 2) dht.add_supermer(seq, depth);
  }
  void done_processing(KmerDHT<MAX_K> &) {}
};

// src/kcount/kcount.hpp:71-73 / kcount.cpp:140-157
template <int MAX_K>
void analyze_kmers(unsigned kmer_len, unsigned /*prev_kmer_len*/, int qual_offset,
                   std::vector<PackedReads *> &packed_reads_list, int dmin_thres, Contigs &ctgs,
                   KmerDHT<MAX_K> &kmer_dht, bool dump_kmers) {
  if (kmer_len != Kmer<MAX_K>::get_k()) die("kmer_len differs from Kmer<MAX_K>::get_k()");
  _dmin_thres = dmin_thres;  // kcount.cpp:145
  for (auto *pr : packed_reads_list) {
    if (pr->get_qual_offset() != qual_offset) die("qual_offset mismatch");
    kmer_dht.add_packed_reads(*pr);
  }
  kmer_dht.flush_updates();
  if (!ctgs.empty()) {  // add_ctg_kmers (kcount.cpp:100-138): one supermer per contig at one rank, in order
    kmer_dht.init_ctg_kmers(0);
    SeqBlockInserter<MAX_K> sbi(0, kmer_dht.get_minimizer_len());
    for (auto &ctg : ctgs) {
      if (ctg.seq.length() < kmer_len + 2) continue;
      std::string seq = ctg.seq;
      sbi.process_seq(seq, ctg.get_uint16_t_depth(), kmer_dht);
    }
    sbi.done_processing(kmer_dht);
    kmer_dht.flush_updates();
  }
  kmer_dht.finish_updates();
  if (dump_kmers) kmer_dht.dump_kmers();
}

}  // namespace mhm2
