// The hand-off of a finished count into the C++ adapter's KmerMap, timed in the calling process (bench.py loads this
// library with ctypes and passes its counter's handle): exactly what HashTableInserter::insert_into_local_hashtable
// does after mhmkc_finish (include/mhmkc_kcount.hpp load_ordered: the device sort, chunked D2H on a helper thread, the
// parallel fill of a fresh map), replacing the reference's loop over the local table (src/kcount/kcount_cpu.cpp:503-522).
//   double mhmkc_handoff_ms(mhmkc_t h, int k, int threads, uint64_t chunk_rows, uint64_t *size_out, uint64_t *bad_out,
//                           double *parts_out)
// returns the milliseconds from the first fetch to the filled map (-1 on a library error); *size_out = map size;
// *bad_out = rows of a 1/64 sample (re-fetched afterwards, not timed) that the map does not hold with their values;
// parts_out[5] (may be null) = load_ordered's first fetch (incl. the device sort), fill, fetch-wait, begin (buffers +
// fill_begin), fill_end ms.
#include <chrono>
#include <cstdio>
#include <vector>

#include "mhmkc_kcount.hpp"

template <int MAX_K>
static double run(mhmkc_t h, int k, int threads, uint64_t chunk_rows, uint64_t *size_out, uint64_t *bad_out,
                  double *parts_out) {
  mhm2::Kmer<MAX_K>::set_k(k);
  mhmkc_stats st;
  if (mhmkc_get_stats(h, &st) != MHMKC_OK) return -1;
  const uint64_t n = st.n_out;
  double ms = 0;
  {
    mhm2::KmerMap<MAX_K> map;
    const auto t0 = std::chrono::steady_clock::now();
    mhm2::LoadTimes lt;
    mhm2::load_ordered<MAX_K>(h, map, n, threads, chunk_rows ? chunk_rows : (4u << 20), &lt);
    ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (parts_out) {
      parts_out[0] = lt.first_fetch;
      parts_out[1] = lt.fill;
      parts_out[2] = lt.wait_fetch;
      parts_out[3] = lt.begin;
      parts_out[4] = lt.end;
    }
    if (size_out) *size_out = map.size();
    // a sample of the rows, looked up with their values
    const int nl = mhm2::Kmer<MAX_K>::N_LONGS;
    const uint64_t m = std::min<uint64_t>(n, 1u << 20);
    std::vector<uint64_t> keys(m * nl);
    std::vector<uint16_t> counts(m);
    std::vector<char> left(m), right(m);
    uint64_t bad = 0;
    for (uint64_t r0 = 0; r0 < n; r0 += 64 * m) {
      const uint64_t c = std::min(m, n - r0);
      if (mhmkc_fetch_ordered_range(h, r0, c, keys.data(), counts.data(), left.data(), right.data()) != MHMKC_OK)
        return -1;
      for (uint64_t i = 0; i < c; i++) {
        auto it = map.find(mhm2::Kmer<MAX_K>(&keys[i * nl]));
        if (it == map.end() || it->second.count != counts[i] || it->second.left != left[i] ||
            it->second.right != right[i])
          bad++;
      }
    }
    if (bad_out) *bad_out = bad;
  }
  return ms;
}

// The ABI this tool was compiled against (mhmkc_stats lives on its stack: a tool older than the library would overflow
// it); bench.py compares it with mhmkc_abi_version() before the first call.
extern "C" int mhmkc_handoff_abi(void) { return MHMKC_ABI_VERSION; }

extern "C" double mhmkc_handoff_ms(mhmkc_t h, int k, int threads, uint64_t chunk_rows, uint64_t *size_out,
                                   uint64_t *bad_out, double *parts_out) {
  switch (k / 32 + 1) {
    case 1: return run<32>(h, k, threads, chunk_rows, size_out, bad_out, parts_out);
    case 2: return run<64>(h, k, threads, chunk_rows, size_out, bad_out, parts_out);
    case 3: return run<96>(h, k, threads, chunk_rows, size_out, bad_out, parts_out);
    case 4: return run<128>(h, k, threads, chunk_rows, size_out, bad_out, parts_out);
  }
  return -1;
}
