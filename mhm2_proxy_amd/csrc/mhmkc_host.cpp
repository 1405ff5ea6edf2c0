// Host side of libmhmkc: handle lifetime, device memory, stage orchestration, the exchange between ranks
// (RCCL or a host-staged transport), the owner hand-off and the C ABI declared in include/mhmkc.h.
//
// One handle = one GPU = one rank. The reference's per-rank state (KmerDHT + HashTableInserter,
// src/kcount/kmer_dht.hpp:95-172) maps onto this struct; its UPC++ supermer store
// (src/kcount/kmer_dht.cpp:133-149,222-224) maps onto the hash-range exchange in exchange().
//
// Work is enqueued on one stream and the host waits only where it needs a number from the device:
// a batch of reads becomes one "slab" of coarse-bucketed records whose bucket counts are copied back
// asynchronously and read at mhmkc_finish, so host batches copied in chunks on a second stream are
// extracted while the next chunk is still on the wire.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <map>
#include <string>
#include <vector>
#include <mutex>
#include <thread>

#include <fcntl.h>
#include <immintrin.h>
#include <sched.h>
#include <sys/stat.h>
#include <unistd.h>

#include "../../include/mhmkc.h"
#include "../../include/mhmkc_debug.h"
#include "kcount_launch.hpp"
#include "kmer_ops.hpp"

namespace {

thread_local std::string g_create_error;

// device bytes held by this process's handles (live, and the most at any time): mhmkc_stats.device_bytes[_peak]
std::atomic<uint64_t> g_dev_live{0}, g_dev_peak{0};

// Test-only switches (include/mhmkc_debug.h, mhmkc_debug_set): they force the rare paths the parity tests check
// (exact layouts, tiny LDS tables, a full output, a failing file read, ...). Process-wide; none is set in production.
struct DebugKnobs {
  int64_t exact = 0;          // exact (histogram) layouts for every slab and finish pass
  int64_t cap = 0;            // LDS table slots of k_count (0: the kernel's)
  int64_t fine_bits = -1;     // fine bits (-1: from the sketch)
  int64_t out_cap = -1;       // output rows the first finish pass allocates (-1: from the sketch)
  int64_t fq_read_fail = -1;  // mhmkc_add_fastq_file: the read of this block fails
  int64_t wide_records = 0;   // key-word records instead of the mixed ones (created handles)
  int64_t smer = 1;           // 0: the minimizer owner at k >= 33 takes the record exchange + hand-off
  int64_t chunk_bytes = 0;    // H2D chunk of a host batch (0: CHUNK_BYTES)
  int64_t d2h_chunk = 0;      // staging chunk of a D2H into pageable memory (0: 8 MB)
  int64_t h2d_threads = 0;   // nibble H2D: worker threads that pack (0: all)
  int64_t h2d_nt = 1;        // nibble H2D: streaming stores into the staging (0: ordinary stores)
  int64_t h2d_adapt = 1;     // nibble H2D from pinned memory: 1 raw chunks on a slow host (the model in add_host_nib), 0
                             // never, 2 every other chunk
  int64_t local_rounds = 1;  // one rank: host batches' chunks fine-partitioned as they land (created handles; 0: at finish)
  int64_t h2d_nib = -1;       // H2D of a host batch: 1 nibbles + u32 offsets, 2 nibbles + u64 offsets, 0 the PackedRead
                              // bytes, -1 1 with >= 4 host threads, else 0
  int64_t cb0[4] = {0, 0, 0, 0};  // coarse bits by key words (0: the default)
};
DebugKnobs g_dbg;

struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap && p) return hipSuccess;
    release();
    size_t want = bytes + bytes / 16 + 4096;
    hipError_t e = hipMalloc(&p, want);
    if (e != hipSuccess) {
      p = nullptr;
      return e;
    }
    cap = want;
    const uint64_t live = g_dev_live.fetch_add(want) + want;
    uint64_t pk = g_dev_peak.load();
    while (live > pk && !g_dev_peak.compare_exchange_weak(pk, live)) {
    }
    return hipSuccess;
  }
  void release() {
    if (p) {
      (void)hipFree(p);
      g_dev_live.fetch_sub(cap);
    }
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T *as() const {
    return (T *)p;
  }
};

// Pinned host memory (asynchronous copies to and from it).
struct PinBuf {
  void *p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap && p) return hipSuccess;
    release();
    size_t want = bytes + bytes / 8 + 4096;
    hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
    if (e != hipSuccess) {
      p = nullptr;
      return e;
    }
    cap = want;
    return hipSuccess;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T *as() const {
    return (T *)p;
  }
};

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Records of one batch (or one H2D chunk), partitioned by coarse bucket (hash range). Every coarse bucket b
// is E_NSUB segments i = b * E_NSUB + s (one per group of blocks sharing an XCD in the capped layout; in the
// exact layout segment s = 0 holds the whole bucket and the others are empty). Segments are in bucket
// order, so a range of buckets is one contiguous span (with gaps in the capped layout).
constexpr uint32_t NSUB = mhm::E_NSUB;
struct Slab {
  DevBuf buf;   // record planes
  DevBuf meta;  // device cursors [nseg] (sub-major) + the overflow flag word
  PinBuf pin;   // host copy of meta: initial cursors going in, final cursors coming back
  mhm::PlaneSet planes{};
  mhm::ReadsView rv{};  // the reads it came from (kept for an exact rerun at finish)
  uint64_t wins = 0;    // counted windows = records
  uint64_t n = 0;
  uint32_t tiles = 0;
  int qcut = 20;         // quality cutoff of its batch (mhmkc_add_seqs encodes quality as case: cutoff 1)
  bool pending = false;  // final cursors not read yet
  hipEvent_t ev = nullptr;  // recorded after the extraction and its cursor D2H (the pipelined exchange waits on it)
  std::vector<uint64_t> counts;  // [nb * NSUB]
  std::vector<uint64_t> bases;   // [nb * NSUB + 1] segment starts, bases[nb * NSUB] = end of the slab
  // supermer exchange: a read slab's supermers per destination (words and supermers, their exact spans), or
  // (recv) the records of the supermers this rank received
  bool recv = false;
  uint32_t bin_lo = 0, bin_hi = 0;  // recv slab of a finish pass: only coarse bins [bin_lo, bin_hi) (bin_hi 0: all)
  uint64_t *codes = nullptr, *desc = nullptr;
  uint32_t *good = nullptr;
  std::vector<uint64_t> sw, ss, swb, ssb;  // [G] words, supermers per destination and their first word / supermer
};

// Device copy of one host batch (mhmkc_add_reads); it lives until finish (a slab may be re-extracted).
struct Arena {
  DevBuf bytes, offs;
};

// Records received in one round of the pipelined exchange: one span per sending peer, each with
// the peer's segment starts / counts of this rank's owned range.
struct RecvPart {
  DevBuf buf;
  mhm::PlaneSet planes{};
  struct Span {
    uint64_t off;                 // first record of the span in planes
    std::vector<uint64_t> start;  // [n_owned * NSUB], relative to the planes
    std::vector<uint64_t> count;  // [n_owned * NSUB]
  };
  std::vector<Span> spans;
};

// A source of owned records for the fine partition: per owned coarse bucket (local index) and segment.
struct Source {
  mhm::PlaneSet planes{};
  std::vector<uint64_t> start;  // [n_owned * NSUB]
  std::vector<uint64_t> count;  // [n_owned * NSUB]
};

// The run table of a fine partition over coarse buckets [c0, c1) (local) of a list of sources: one entry per
// non-empty (source, segment) span; the device expands it into chunks of T records ordered by XCD class (coarse % 8),
// then coarse bucket, segment, source (xcd_chunk). n_c0: the chunks up to the end of coarse bucket c0 (all of c0's
// records when c0 % 8 == 0: the sketch's sample); n_c0_even: its records in even-numbered chunks.
struct RunTable {
  std::vector<mhm::SRun> runs;
  std::vector<mhm::PlaneSet> ps;
  uint64_t n_chunks = 0, n_c0 = 0, xcd_max = 0, rec_c0 = 0, rec_c0_even = 0;
  uint64_t xcd_start[9] = {0};
};

// One exchange round's fine partition on pstream (the incremental partition): its run table (kept
// until the round's copies ran) and device tables.
struct IncRound {
  RunTable rt;
  DevBuf chunks, srcs;
  PinBuf pin;  // the tables' pinned copy (a pageable source made the host wait for the partition stream's earlier work)
};

// One device-to-device transfer of the exchange: `bytes` at `ptr` to (or from) rank `peer`.
struct Xfer {
  int peer;
  void *ptr;
  uint64_t bytes;
};

struct Prof {
  int stage;
  hipEvent_t a, b;
};

// The pinned staging of pageable D2H copies, shared by the process's handles (one at a time): the reference makes a
// new KmerDHT, so a new handle, per k round, and a first hipHostMalloc of the staging cost a hand-off ~40 ms.
struct D2HStage {
  std::mutex mu;
  PinBuf buf[2];
};
D2HStage &d2h_stage() {
  static D2HStage *s = new D2HStage();  // (never freed: the process's pinned staging)
  return *s;
}

// Bytes of one H2D chunk of mhmkc_add_reads (MHMKC_CHUNK_BYTES overrides: tests force many chunks).
constexpr uint64_t CHUNK_BYTES = 128ull << 20;

// Host threads for the transcoding of host batches: the CPUs of the affinity mask, at most OMP_NUM_THREADS and 16.
int host_threads() {
  int n = 16;
  cpu_set_t cs;
  if (sched_getaffinity(0, sizeof cs, &cs) == 0) n = CPU_COUNT(&cs);
  if (const char *e = getenv("OMP_NUM_THREADS")) {
    const int v = atoi(e);
    if (v > 0) n = std::min(n, v);
  }
  return std::max(1, std::min(16, n));
}

// The process's host worker threads (host_threads() of them, the caller being number 0), shared by its handles one job
// at a time: run(fn) calls fn(t) for every t in [0, size()) and returns when all have returned.
class Workers {
 public:
  static Workers &get() {
    static std::mutex mu;
    static Workers *w = nullptr;
    std::lock_guard<std::mutex> g(mu);
    if (!w || w->pid_ != getpid()) w = new Workers(host_threads());  // (never freed; a forked child makes its own)
    return *w;
  }
  int size() const { return n_; }
  void run(const std::function<void(int)> &fn) {
    std::lock_guard<std::mutex> job(job_mu_);
    {
      std::lock_guard<std::mutex> g(mu_);
      fn_ = &fn;
      left_ = n_ - 1;
      gen_++;
    }
    cv_.notify_all();
    fn(0);
    std::unique_lock<std::mutex> g(mu_);
    done_cv_.wait(g, [&] { return left_ == 0; });
    fn_ = nullptr;
  }

 private:
  explicit Workers(int n) : n_(n), pid_(getpid()) {
    for (int t = 1; t < n; t++) std::thread([this, t] { loop(t); }).detach();
  }
  void loop(int t) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)> *fn;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return gen_ != seen; });
        seen = gen_;
        fn = fn_;
      }
      (*fn)(t);
      std::lock_guard<std::mutex> g(mu_);
      if (--left_ == 0) done_cv_.notify_one();
    }
  }
  const int n_;
  const pid_t pid_;
  std::mutex job_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)> *fn_ = nullptr;
  uint64_t gen_ = 0;
  int left_ = 0;
};

// PackedRead bytes (code | min(q, 31) << 3, src/packed_reads.cpp:98-107) as the nibbles code | (q >= qcut) << 3 the
// nibble H2D sends (k_expand_nibbles restores bytes that load_tile reads alike): n bytes of src into (n + 1) / 2 bytes
// of dst, two per byte, the first in the low half. Eight bytes at a time in one u64: the per-byte sums q + 128 - qcut
// stay below 256, so no carry crosses a byte, and bit 7 of each is q >= qcut.
void nib_pack_swar(const uint8_t *src, uint64_t n, uint8_t *dst, int qcut, uint64_t i = 0) {
  const uint32_t qc = (uint32_t)std::min(std::max(qcut, 0), 32);
  constexpr uint64_t L = 0x0101010101010101ull;
  const uint64_t bias = (0x80ull - qc) * L;
  for (; i + 8 <= n; i += 8) {
    uint64_t v;
    memcpy(&v, src + i, 8);
    const uint64_t c = v & (7 * L), q = (v >> 3) & (0x1f * L);
    uint64_t x = c | (((q + bias) >> 4) & (8 * L));
    x = (x | (x >> 4)) & 0x00ff00ff00ff00ffull;
    x = (x | (x >> 8)) & 0x0000ffff0000ffffull;
    const uint32_t y = (uint32_t)(x | (x >> 16));
    memcpy(dst + i / 2, &y, 4);
  }
  for (; i < n; i++) {
    const uint32_t b = src[i], v = (b & 7u) | ((b >> 3) >= qc ? 8u : 0u);
    if (i & 1)
      dst[i / 2] |= (uint8_t)(v << 4);
    else
      dst[i / 2] = (uint8_t)v;
  }
}

// The same 64 bytes at a time (AVX2): nibble pairs summed as n0 + 16 n1 by maddubs, packed to bytes, lanes put in order.
__attribute__((target("avx2"))) inline __m256i nib_pairs_avx2(__m256i v, __m256i qm1) {
  const __m256i q = _mm256_and_si256(_mm256_srli_epi16(v, 3), _mm256_set1_epi8(0x1f));  // q <= 31, qm1 >= -1: signed
  const __m256i ok = _mm256_and_si256(_mm256_cmpgt_epi8(q, qm1), _mm256_set1_epi8(8));
  return _mm256_maddubs_epi16(_mm256_or_si256(_mm256_and_si256(v, _mm256_set1_epi8(7)), ok), _mm256_set1_epi16(0x1001));
}

// A 32-byte aligned dst is written with streaming stores (the staging is only read by the DMA engine: no read for
// ownership, nothing evicted), fenced at the end.
__attribute__((target("avx2"))) void nib_pack_avx2(const uint8_t *src, uint64_t n, uint8_t *dst, int qcut, bool nt) {
  const __m256i qm1 = _mm256_set1_epi8((char)(std::min(std::max(qcut, 0), 32) - 1));
  uint64_t i = 0;
  if (nt && ((uintptr_t)dst & 31) == 0) {
    for (; i + 64 <= n; i += 64) {
      const __m256i a = nib_pairs_avx2(_mm256_loadu_si256((const __m256i *)(src + i)), qm1);
      const __m256i b = nib_pairs_avx2(_mm256_loadu_si256((const __m256i *)(src + i + 32)), qm1);
      _mm256_stream_si256((__m256i *)(dst + i / 2), _mm256_permute4x64_epi64(_mm256_packus_epi16(a, b), 0xd8));
    }
    _mm_sfence();
  }
  for (; i + 64 <= n; i += 64) {
    const __m256i a = nib_pairs_avx2(_mm256_loadu_si256((const __m256i *)(src + i)), qm1);
    const __m256i b = nib_pairs_avx2(_mm256_loadu_si256((const __m256i *)(src + i + 32)), qm1);
    _mm256_storeu_si256((__m256i *)(dst + i / 2), _mm256_permute4x64_epi64(_mm256_packus_epi16(a, b), 0xd8));
  }
  nib_pack_swar(src, n, dst, qcut, i);
}

void nib_pack(const uint8_t *src, uint64_t n, uint8_t *dst, int qcut, bool nt = true) {
  static const bool avx2 = __builtin_cpu_supports("avx2");
  if (avx2)
    nib_pack_avx2(src, n, dst, qcut, nt);
  else
    nib_pack_swar(src, n, dst, qcut);
}

// The pinned staging of the nibble H2D (two slots per add call), kept by the process for the next call (the reference
// makes a new handle per k round): a handle takes two buffers for the length of one add call.
struct H2DStage {
  std::mutex mu;
  std::vector<PinBuf *> free;
};
H2DStage &h2d_stage() {
  static H2DStage *s = new H2DStage();  // (never freed: the process's pinned staging)
  return *s;
}

}  // namespace

struct mhmkc {
  mhmkc_config cfg{};
  int k = 0, nl = 1, nlo = 1, mlen = 15;
  int dmin = 2;  // the finish's depth threshold (mhmkc_set_dmin_thres)
  bool packed = true;
  bool compact = false;  // compact records (kmer_ops.hpp cmix): 5 B per coarse record, 4 B per fine record
  bool mixed2 = false;   // mixed two-word records (kmer_ops.hpp m2_mix, 33 <= k <= 63): 16 B, no byte plane
  bool mixed3 = false;   // mixed three- and four-word records (kmer_ops.hpp mx_mix, 64 < k < 128): NL words
  bool mixed() const { return compact || mixed2 || mixed3; }  // the kernels' "compact" flag: bucket digits implicit
  int cb = 8, fb = 8, hbits = 0;
  uint32_t nb = 256, nf = 256;
  uint32_t own_lo = 0, own_hi = 256;  // owned coarse range [own_lo, own_hi)
  int dev = 0;
  int n_cu = 0;  // compute units: persistent k_count workgroups
  hipStream_t stream = nullptr, copy_stream = nullptr;
  bool own_stream = false;
  ncclComm_t comm = nullptr;
  mhmkc_transport xp{};
  bool has_xp = false;

  std::vector<Slab *> slabs;  // pool; first n_slabs are in use
  size_t n_slabs = 0;
  std::vector<Arena *> arenas;  // pool; first n_arenas are in use
  size_t n_arenas = 0;
  // pipelined exchange (xpipe): slabs [0, xq) have been sent, one round per slab, on xstream while
  // the next slab is extracted; received records land in parts [0, n_parts)
  bool xpipe = false;
  int xpieces = 8;  // a device batch is cut into this many slabs (so that there is a next slab to overlap)
  hipStream_t xstream = nullptr;
  std::vector<RecvPart *> parts;
  size_t n_parts = 0, xq = 0;
  uint64_t x_rounds = 0;
  bool x_all_done = false;
  double x_ms = 0;
  hipEvent_t ev_xdone = nullptr, ev_xext = nullptr;
  std::vector<hipEvent_t> x_ev;  // per round: start / end of the round's transfer on xstream
  int xround(Slab *sl, bool done);
  // incremental fine partition: the rounds' records are fine-partitioned on pstream as they land,
  // into a capped layout fixed after the first round (fine bits from the round's distinct-key sketch, extrapolated;
  // capacities from the windows every rank announced); finish then only counts, unless the layout overflowed
  bool inc = false, inc_tried = false;
  hipStream_t pstream = nullptr;
  hipEvent_t ev_pdone = nullptr;
  uint64_t inc_expect = 0, inc_announced = 0;  // this rank's windows announced by its add calls / not yet added
  uint64_t x_expect_all = 0;                   // all ranks' announced windows (the latest round's all-gather)
  std::vector<uint64_t> x_r0_coarse;           // round 0: records of each owned coarse bucket (all senders)
  uint64_t x_r0_total = 0;                     // round 0: records of all senders' slabs (every coarse bucket)
  std::vector<int> x_round_slab;               // per round: the index of this rank's slab sent in it, or -1
  std::vector<IncRound *> inc_pool;
  size_t inc_parted = 0;                       // rounds whose partition is enqueued
  double inc_distinct = 0;                     // the extrapolated distinct keys of the owned range
  double inc_ext_per_rec = 0;                  // extension adds per record of the sketch sample (stats)
  mhm::PlaneSet inc_r2{};                      // the fine records' planes of the incremental layout (in d_r2)
  std::vector<uint64_t> inc_cfit;              // its capped layout (host copy, kept until finish)
  hipEvent_t ev_tail0 = nullptr;               // finish: the exchange is over, what is left is counting
  uint64_t inc_out_est = 0;
  int inc_setup();
  int inc_round(size_t r);
  // single rank, host batches: the slabs of the H2D chunks become the incremental partition's rounds
  // as their extractions finish ("local rounds"); slabs [0, lq) are rounds
  bool lrounds = false;
  size_t lq = 0;
  int local_rounds(bool all);
  hipEvent_t round_event(size_t r) const { return lrounds ? slabs[(size_t)x_round_slab[r]]->ev : x_ev[2 * r + 1]; }
  void round_sources(size_t r, std::vector<Source> &srcs) const;
  int finish_inc(bool &done, uint64_t *n_out_ret);
  void make_runs(const std::vector<Source> &srcs, uint32_t c0, uint32_t c1, int T, RunTable &rt) const;
  int upload_runs(const RunTable &rt, DevBuf &buf, DevBuf &sbuf, hipStream_t s, mhm::PartitionParams &pp,
                  PinBuf *pin = nullptr);
  int fine_layout(const std::vector<uint64_t> &per_coarse, double slack, std::vector<uint64_t> &cfit,
                  uint64_t &r2_size) const;
  int pump();
  int resolve_one(Slab *sl, bool &redo);
  std::vector<hipEvent_t> chunk_ev;  // one per H2D chunk in flight (pool)
  // the nibble H2D of host batches (add_host): device slots of a chunk's nibbles with the event after the expansion that
  // last read each (the next copy into the slot waits for it), and the events after the copy out of each pinned slot
  DevBuf d_nib[3];
  hipEvent_t nib_ev[3] = {nullptr, nullptr, nullptr};
  bool nib_used[3] = {false, false, false};
  hipEvent_t stage_ev[2] = {nullptr, nullptr};
  int add_host_nib(const uint8_t *bytes, const uint64_t *offs, uint64_t n_reads, int qcut, uint64_t chunk);
  DevBuf d_hist, d_tiles, d_tsb, d_err, d_stats, d_fine_hist, d_fine_base, d_fine_cursor, d_chunks, d_srcs;
  DevBuf d_r2, d_out_keys, d_out_counts, d_out_left, d_out_right, d_out_cursor, d_recv, d_xg;
  DevBuf d_hll, d_dest, d_ohist, d_out2_keys, d_out2_counts, d_out2_left, d_out2_right, d_mh;
  DevBuf d_ord;  // mhmkc_fetch_ordered: sort keys, row indices, radix-sort scratch
  mhm::OutRows ord{};      // the ordered rows (in d_r2 or d_ord), valid while ord_ready
  bool ord_ready = false;  // set by order_rows, cleared by finish / reset
  int order_rows();
  char *ord_scratch = nullptr;  // the ordering's scratch (free once the rows are ordered) and its size
  size_t ord_scratch_bytes = 0;
  // mhmkc_fetch_map_range: each ordered row's KmerMap slot (u32) and tag (u8) for a map of map_cap slots
  DevBuf d_mslot;
  uint64_t map_cap = 0;  // the capacity d_mslot holds the slots of (0: none; cleared with ord_ready)
  int map_slots(uint64_t cap);
  DevBuf d_spill;  // k_count: the deferred records of cold sweeps, mhm::SPILL_RECORDS per persistent workgroup
  DevBuf d_cfit;   // capped fine layout: per coarse bucket of the pass its first record and fine-bucket capacity
  DevBuf d_inc_skip;  // incremental count: per owned coarse bucket, 1 = overflowed its capped layout (k_inc_fixup)
  double inc_slack = 0;  // the incremental layout's fine-bucket slack (inc_setup)
  // supermer exchange (smer): owner bytes of a slab's tiles; the received supermers (codes, good bits, descriptors),
  // their window counts / prefix, per-tile first supermer, scan scratch
  bool smer = false;
  DevBuf d_owners, d_rcodes, d_rgood, d_rdesc, d_rnwin, d_rwpre, d_rtiles, d_rtmp;
  mhm::SmerSource rsrc{};
  uint64_t smer_nwin = 0, smer_seen = 0;  // received windows; records extracted from them by the finish passes so far
  uint32_t smer_tiles = 0;
  Slab *smer_slab = nullptr;  // the received supermers' records of the current finish pass
  int smer_build(Slab *sl);
  int smer_exchange(std::vector<Source> &srcs);
  int smer_records(uint32_t lo, uint32_t hi, std::vector<Source> &srcs);
  PinBuf x_send, x_recv;  // host-staged exchange
  DevBuf d_xsend, d_xsegs;  // pipelined exchange: the round's dense send planes and their segment list
  std::vector<mhm::SegCopy> x_segs;
  uint64_t x_send_cap = 0;
  // FASTQ ingest (fastq.hip): text staging, chunk counts, newline positions, record lengths, scan scratch,
  // the packed reads of the last batch, first error
  DevBuf d_fq_text, d_fq_chunk, d_fq_lines, d_fq_len, d_fq_tmp, d_fq_bytes, d_fq_offs, d_fq_err;
  DevBuf d_fqa_bytes, d_fqa_offs;  // mhmkc_add_fastq_file: the PackedReads of all blocks (swapped in at the end)
  DevBuf d_fq_recoffs, d_fq_scratch, d_fq_pairinfo, d_fq_stats, d_fq_desc;  // pair merging
  uint64_t fq_reads = 0, fq_bases = 0;
  // consumed != nullptr: a block of a longer text (mhmkc_add_fastq_file) whose last record may be cut; only the
  // complete records (pairs) are parsed and *consumed is the length of their text
  int add_fastq(const char *d_text, uint64_t n, bool pairs = false, uint64_t *consumed = nullptr);
  PinBuf fq_file_buf;  // mhmkc_add_fastq_file: two blocks (one read while the other is copied; pinned)
  // contig pass (add_ctg_kmers): contigs in the PackedRead byte layout, kept on the host until finish
  std::vector<uint8_t> ctg_bytes;
  std::vector<uint64_t> ctg_offs{0}, ctg_win{0};  // byte offsets, counted-window prefix
  std::vector<uint16_t> ctg_depth;
  DevBuf d_ctg_bytes, d_ctg_offs, d_ctg_win, d_ctg_depth, d_ctg_scratch, d_ctg_state, d_ctg_bucket, d_ctg_done;
  DevBuf d_ctg_keys[4];
  uint64_t ctg_n = 0;  // folded contig k-mers of the last finish
  int prepare_ctgs();

  std::string err;
  bool finished = false;
  bool began = false;
  bool partial = false;  // a failed mhmkc_add_fastq_file left part of a file in the round (finish refuses it)
  uint64_t n_out = 0;
  mhmkc_stats st{};
  bool profiling = false;
  bool prof_heavy_only = false;  // mhmkc_set_profiling level 2: events around the heavy stages only
  bool prof_open = false;        // the last prof_begin recorded its event (its prof_end records the other)
  std::vector<Prof> prof;
  std::vector<hipEvent_t> ev_pool;
  hipEvent_t ev_begin = nullptr, ev_end = nullptr, ev_h2d0 = nullptr, ev_h2d1 = nullptr;

  int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    err = buf;
    return code;
  }
  int hip_fail(hipError_t e, const char *what) {
    (void)hipGetLastError();  // reported here: not again by the next launch's hipGetLastError check
    return fail(MHMKC_EHIP, "%s: %s (%d)", what, hipGetErrorString(e), (int)e);
  }

  hipEvent_t take_event() {
    if (!ev_pool.empty()) {
      hipEvent_t e = ev_pool.back();
      ev_pool.pop_back();
      return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
  }
  // (begin / end pairs are never nested; at level 2 only extraction, partition, exchange and count are timed: every
  // event record is a marker the next launch queues behind, 0.07-0.2 ms per C2 step with all stages)
  void prof_begin(int stage, hipStream_t s = nullptr) {
    prof_open = profiling && (!prof_heavy_only || stage == MHMKC_STAGE_ESCAT || stage == MHMKC_STAGE_SSCAT ||
                              stage == MHMKC_STAGE_XCHG || stage == MHMKC_STAGE_COUNT);
    if (!prof_open) return;
    Prof p{stage, take_event(), take_event()};
    (void)hipEventRecord(p.a, s ? s : stream);
    prof.push_back(p);
  }
  void prof_end(hipStream_t s = nullptr) {
    if (!prof_open || prof.empty()) return;
    prof_open = false;
    (void)hipEventRecord(prof.back().b, s ? s : stream);
  }
  void prof_collect() {
    for (auto &p : prof) {
      float ms = 0;
      if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
        st.ms_kernel[p.stage] += ms;
        st.launches[p.stage] += 1;
      }
      ev_pool.push_back(p.a);
      ev_pool.push_back(p.b);
    }
    prof.clear();
  }

  int G() const { return cfg.n_ranks; }
  uint32_t owner_lo(int r) const { return (uint32_t)(((uint64_t)r * nb + cfg.n_ranks - 1) / cfg.n_ranks); }
  uint32_t n_owned() const { return own_hi - own_lo; }
  size_t rec_bytes() const { return compact ? 5 : 8 * (size_t)nl + (packed ? 0 : 1); }
  // compact fine records hold the mixed key's bits below the coarse and fine digits + the ext code
  int min_fine_bits() const { return compact ? std::max(0, 2 * k - cb - 26) : 0; }

  int begin_round() {
    if (finished) return fail(MHMKC_ESTATE, "handle already finished; call mhmkc_reset first");
    if (!began) {
      began = true;
      (void)hipEventRecord(ev_begin, stream);
    }
    return MHMKC_OK;
  }

  Slab *new_slab() {
    if (n_slabs == slabs.size()) slabs.push_back(new Slab());
    Slab *sl = slabs[n_slabs++];
    sl->recv = false;
    sl->bin_lo = sl->bin_hi = 0;
    return sl;
  }
  Arena *new_arena() {
    if (n_arenas == arenas.size()) arenas.push_back(new Arena());
    return arenas[n_arenas++];
  }

  // Grow a buffer that kernels already enqueued may still read: wait for them first (a free would not).
  hipError_t grow(DevBuf &b, size_t bytes) {
    if (bytes <= b.cap && b.p) return hipSuccess;
    hipError_t e = hipStreamSynchronize(stream);
    return e != hipSuccess ? e : b.ensure(bytes);
  }

  // Record planes for n records: NL u64 word planes (+ a byte plane when the ext code is not packed);
  // compact: a u32 plane (w[0]) + a byte plane for coarse-bucketed records, the u32 plane alone for fine.
  // (sync = false: the buffer is known idle, e.g. for the incremental partition, which must not wait for the main
  // stream's extraction)
  int set_planes(DevBuf &buf, uint64_t n, mhm::PlaneSet &ps, bool fine = false, bool sync = true) {
    const uint64_t m = std::max<uint64_t>(n, 1);
    const size_t plane = align_up(m * (compact ? 4 : 8), 256);
    const size_t extb = (compact ? !fine : !packed) ? align_up(m, 256) : 0;
    const int np = compact ? 1 : nl;
    hipError_t e = sync ? grow(buf, plane * np + extb) : buf.ensure(plane * np + extb);
    if (e != hipSuccess) return hip_fail(e, "allocating record planes");
    char *b = buf.as<char>();
    for (int w = 0; w < 4; w++) ps.w[w] = w < np ? (uint64_t *)(b + plane * w) : nullptr;
    ps.ext = extb ? (uint8_t *)(b + plane * np) : nullptr;
    return MHMKC_OK;
  }

  // Move a plane set so that record index `sh` lands on its first entry (a capped slab that holds only the segments
  // from sh on: the kernels keep indexing segment i at i * cap)
  void shift_planes(mhm::PlaneSet &ps, uint64_t sh) const {
    if (!sh) return;
    if (compact) {
      ps.w[0] = (uint64_t *)((uint32_t *)ps.w[0] - sh);
    } else if (mixed2) {  // one 16-byte record per entry in the first plane's place
      ps.w[0] -= 2 * sh;
      if (ps.w[1]) ps.w[1] -= sh;
    } else {
      for (int w = 0; w < 4; w++)
        if (ps.w[w]) ps.w[w] -= sh;
    }
    if (ps.ext) ps.ext -= sh;
  }

  // Device -> host copy of `bytes` into caller (pageable) memory through two pinned staging buffers: chunk i's DMA
  // runs while chunk i - 1 is copied out of the other buffer by host threads (a plain copy into pageable memory
  // moved the C2 table at ~17 GB/s).
  hipError_t d2h(void *dst, const void *src, size_t bytes);

  int add_view(const mhm::ReadsView &rv, uint64_t wins, bool wins_known);
  int extract(Slab *sl, bool exact);
  int resolve_slabs();
  int add_host(const uint8_t *bytes, const uint64_t *offs, uint64_t n_reads, int qcut);
  int allgather_host(const void *send, void *recv, size_t bytes, hipStream_t xs = nullptr);
  int move(const std::vector<Xfer> &snd, const std::vector<Xfer> &rcv, hipStream_t xs = nullptr);
  int exchange(std::vector<Source> &srcs);
  int gather_ctgs(std::vector<uint8_t> &gb, std::vector<uint64_t> &go, std::vector<uint64_t> &gw,
                  std::vector<uint16_t> &gd);
  // every rank's contigs, gathered once per finish (prepare_ctgs runs again, locally, when an incremental count
  // falls back to the passes on this rank only)
  bool ctg_gathered = false;
  std::vector<uint8_t> ctg_gbytes;
  std::vector<uint64_t> ctg_goffs, ctg_gwin;
  std::vector<uint16_t> ctg_gdepth;
  int handoff();
  int finish(uint64_t *n_out_ret);
  int finish_passes(uint64_t owned) const;
  hipError_t grow_keep(DevBuf &b, size_t used, size_t need);
  int qcut_pending = 20;  // quality cutoff of the batch being added (add_seqs encodes quality as case)
};

// Fine partition target: distinct keys per fine bucket <= FINE_LOAD x LDS table slots (0.5: k = 77 count 10.35 ->
// 12.42 ms; 0.9: the same fine bits at C2).
constexpr double FINE_LOAD = 0.7;
// HyperLogLog estimate (Flajolet et al. 2007) with the linear-counting correction for small counts.
static double hll_estimate(const std::vector<uint32_t> &reg) {
  const double m = (double)reg.size();
  double sum = 0;
  int zeros = 0;
  for (uint32_t r : reg) {
    sum += std::ldexp(1.0, -(int)r);
    zeros += r == 0;
  }
  const double e = 0.7213 / (1.0 + 1.079 / m) * m * m / sum;
  return (e <= 2.5 * m && zeros) ? m * std::log(m / zeros) : e;
}

// ------------------------------------------------------------------------------------------------
// extraction: one batch (or chunk) of reads into a coarse-bucketed slab

// Enqueue the extraction of a slab. Capped layout (the default): every segment gets the expected share of
// the windows + 4 % + 1024 records, one scatter pass, no histogram; the final cursors come back to pinned
// memory asynchronously and are read by resolve_slabs. Exact layout (skewed input that overflowed a capped
// segment, or MHMKC_DEBUG_EXACT): a histogram pass first, which the host waits for.
int mhmkc::extract(Slab *sl, bool exact) {
  const int T = mhm::tile_bases(nl);
  const uint32_t nseg = nb * NSUB;
  hipError_t e;
  if ((e = grow(d_tiles, (size_t)sl->tiles * 4 + 64)) != hipSuccess) return hip_fail(e, "tile index");
  if ((e = grow(d_hist, (size_t)nb * 8 + 64)) != hipSuccess) return hip_fail(e, "histogram");
  if ((e = sl->meta.ensure((size_t)nseg * 8 + 64)) != hipSuccess) return hip_fail(e, "slab cursors");
  if ((e = sl->pin.ensure((size_t)nseg * 8 + 64)) != hipSuccess) return hip_fail(e, "slab cursors (host)");
  sl->counts.assign(nseg, 0);
  sl->bases.assign(nseg + 1, 0);
  mhm::ExtractParams p{};
  p.reads = sl->rv;
  p.tile_first_read = d_tiles.as<uint32_t>();
  p.n_tiles = sl->tiles;
  p.k = k;
  p.qual_cutoff = sl->qcut;
  p.coarse_bits = cb;
  p.n_bins = nb;
  p.hbits = hbits;
  p.compact = mixed();
  p.hist = d_hist.as<unsigned long long>();
  unsigned long long *dcur = sl->meta.as<unsigned long long>();
  p.cursor = dcur;
  p.err = d_err.as<unsigned int>();
  p.ovf = (unsigned int *)(dcur + nseg);
  const bool filt = sl->bin_hi != 0;  // (received supermers of a finish pass: its coarse bins only)
  const uint32_t blo = filt ? sl->bin_lo : 0, bhi = filt ? sl->bin_hi : nb;
  p.bin_lo = filt ? blo : 0;
  p.bin_hi = filt ? bhi : 0;
  uint64_t shift = 0;
  if (!sl->recv) {  // (the received supermers' tile index is made once by smer_exchange)
    // the batch's read-start bits (k_read_start_bits: the extraction loads its tile's words beside the bases, no
    // dependent round trip through the tile's first read)
    prof_begin(MHMKC_STAGE_TILEIDX);
    const uint64_t words = mhm::read_start_words(sl->tiles, nl);
    if ((e = grow(d_tsb, words * 4 + 64)) == hipSuccess) {
      e = mhm::launch_read_start_bits(sl->rv, d_tsb.as<uint32_t>(), words, stream);
      p.tile_starts = d_tsb.as<uint32_t>();
    }
    prof_end();
    if (e != hipSuccess) return hip_fail(e, "tile index");
  }
  if (exact) {
    std::vector<uint64_t> hist(nb);
    prof_begin(MHMKC_STAGE_OTHER);
    e = hipMemsetAsync(d_hist.p, 0, (size_t)nb * 8, stream);
    prof_end();
    if (e != hipSuccess) return hip_fail(e, "memset");
    prof_begin(MHMKC_STAGE_EHIST);
    e = sl->recv ? mhm::launch_smer_extract(p, rsrc, nl, packed, true, stream) : mhm::launch_extract_hist(p, nl, packed, stream);
    prof_end();
    if (e != hipSuccess) return hip_fail(e, "extract_hist");
    if ((e = hipMemcpyAsync(hist.data(), d_hist.p, (size_t)nb * 8, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
        (e = hipStreamSynchronize(stream)) != hipSuccess)
      return hip_fail(e, "extract_hist");
    uint64_t tot = 0;
    for (uint32_t b = 0; b < nb; b++) {
      sl->bases[b * NSUB] = tot;
      tot += hist[b];
      for (uint32_t q = 1; q < NSUB; q++) sl->bases[b * NSUB + q] = tot;  // empty segments
    }
    sl->bases[nseg] = tot;
    p.bin_cap = 0;
  } else {
    // every segment gets the expected share of the windows (+4 % + 1024); a filtered slab allocates only the
    // segments of its bins and shifts its planes so that segment i still starts at record i * cap
    const uint64_t expect = sl->wins / nseg;
    const uint64_t cap = align_up(expect + expect / 25 + 1024, 64);
    for (uint32_t i = 0; i <= nseg; i++) sl->bases[i] = (uint64_t)std::min(std::max(i, blo * NSUB), bhi * NSUB) * cap;
    p.bin_cap = cap;
    shift = (uint64_t)blo * NSUB * cap;
  }
  int rc;
  if ((rc = set_planes(sl->buf, sl->bases[nseg] - shift, sl->planes))) return rc;
  shift_planes(sl->planes, shift);
  // device cursors are sub-major (cursor[s * nb + b]): the 64 lanes of one atomic instruction then hit 64
  // consecutive words, which the memory-side atomic unit serves as whole lines
  uint64_t *hc = sl->pin.as<uint64_t>();
  for (uint32_t i = 0; i < nseg; i++) hc[(size_t)(i % NSUB) * nb + i / NSUB] = sl->bases[i];
  hc[nseg] = 0;  // overflow flag
  if ((e = hipMemcpyAsync(dcur, hc, (size_t)nseg * 8 + 8, hipMemcpyHostToDevice, stream)) != hipSuccess)
    return hip_fail(e, "cursor H2D");
  p.out = sl->planes;
  prof_begin(MHMKC_STAGE_ESCAT);
  e = sl->recv ? mhm::launch_smer_extract(p, rsrc, nl, packed, false, stream) : mhm::launch_extract_scatter(p, nl, packed, stream);
  prof_end();
  if (e != hipSuccess) return hip_fail(e, "extract_scatter");
  if ((e = hipMemcpyAsync(hc, dcur, (size_t)nseg * 8 + 8, hipMemcpyDeviceToHost, stream)) != hipSuccess)
    return hip_fail(e, "cursor D2H");
  if (!sl->ev && (e = hipEventCreateWithFlags(&sl->ev, hipEventDisableTiming)) != hipSuccess) return hip_fail(e, "slab event");
  if ((e = hipEventRecord(sl->ev, stream)) != hipSuccess) return hip_fail(e, "slab event");
  sl->pending = true;
  return MHMKC_OK;
}

// A batch as a device view. wins (the counted windows) comes from the host when it knows the offsets;
// otherwise a small kernel counts them (and checks the offsets) and the host waits for the number.
int mhmkc::add_view(const mhm::ReadsView &rv, uint64_t wins, bool wins_known) {
  hipError_t e;
  if (!wins_known) {
    if ((e = grow(d_hist, (size_t)nb * 8 + 64)) != hipSuccess) return hip_fail(e, "histogram");
    unsigned long long *d_wins = d_hist.as<unsigned long long>() + nb;
    unsigned int ef = 0;
    prof_begin(MHMKC_STAGE_TILEIDX);
    e = hipMemsetAsync(d_wins, 0, 8, stream);
    if (e == hipSuccess) e = mhm::launch_count_windows(rv, k, d_wins, d_err.as<unsigned int>(), stream);
    prof_end();
    if (e == hipSuccess) e = hipMemcpyAsync(&wins, d_wins, 8, hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipMemcpyAsync(&ef, d_err.p, 4, hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    if (e != hipSuccess) return hip_fail(e, "window count");
    if (ef & 4u)
      return fail(MHMKC_EINVAL, "device read offsets are not a PackedReads CSR (offs[0] == 0, non-decreasing, reads "
                                "<= 65535 bases, offs[n_reads] == n_bases)");
  }
  if (wins == 0) return MHMKC_OK;
  const int T = mhm::tile_bases(nl);
  const uint64_t tiles64 = (rv.n_bases + T - 1) / T;
  if (tiles64 >= 0x7fffffffull) return fail(MHMKC_EINVAL, "batch too large");
  Slab *sl = new_slab();
  sl->rv = rv;
  sl->wins = wins;
  sl->tiles = (uint32_t)tiles64;
  sl->qcut = qcut_pending;
  sl->n = 0;
  st.occurrences += wins;
  st.slabs++;
  // (the windows an add call announced for its whole batch, inc_expect, cover its slabs; any other slab adds its own)
  if (inc_announced >= wins) {
    inc_announced -= wins;
  } else {
    inc_expect += wins - inc_announced;
    inc_announced = 0;
  }
  if (smer) return smer_build(sl);
  int rc = extract(sl, g_dbg.exact != 0);
  return rc ? rc : pump();
}

// The final cursors of a pending slab (its event: the extraction and the cursor D2H are done). A slab whose capped
// segment overflowed (skewed input: very repetitive reads) is extracted again with exact sizes (redo: read it again).
int mhmkc::resolve_one(Slab *sl, bool &redo) {
  const uint32_t nseg = nb * NSUB;
  hipError_t e;
  redo = false;
  if ((e = hipEventSynchronize(sl->ev)) != hipSuccess) return hip_fail(e, "extract");
  const uint64_t *hc = sl->pin.as<uint64_t>();
  if (hc[nseg] & 2u) {  // a capped segment overflowed: its excess records were not written
    st.exact_reruns++;
    redo = true;
    return extract(sl, true);
  }
  uint64_t tot = 0;
  for (uint32_t i = 0; i < nseg; i++) {
    sl->counts[i] = hc[(size_t)(i % NSUB) * nb + i / NSUB] - sl->bases[i];
    tot += sl->counts[i];
  }
  if (!sl->bin_hi && tot != sl->wins) return fail(MHMKC_EHIP, "internal: slab holds %llu records, expected %llu",
                                   (unsigned long long)tot, (unsigned long long)sl->wins);
  sl->n = tot;
  sl->pending = false;
  return MHMKC_OK;
}

// Read the final cursors of every pending slab (in order; the last one's event covers the others).
int mhmkc::resolve_slabs() {
  for (size_t s = 0; s < n_slabs; s++) {
    Slab *sl = slabs[s];
    for (int pass = 0; sl->pending; pass++) {
      bool redo = false;
      int rc = resolve_one(sl, redo);
      if (rc) return rc;
      if (redo && pass) return fail(MHMKC_EHIP, "internal: exact extraction overflowed");
    }
  }
  return MHMKC_OK;
}

// Host batch: copied to a device arena in chunks of whole reads on the copy stream, each chunk extracted
// (as a slice view of the arena) as soon as its copy has landed. The host validates the offsets and counts
// each chunk's windows while the previous chunk is on the wire.
int mhmkc::add_host(const uint8_t *bytes, const uint64_t *offs, uint64_t n_reads, int qcut) {
  int rc = begin_round();
  if (rc) return rc;
  if (offs[0] != 0) return fail(MHMKC_EINVAL, "read_offsets[0] must be 0");
  const uint64_t n_bases = offs[n_reads];
  st.reads += n_reads;
  st.bases += n_bases;
  if (n_reads == 0) return MHMKC_OK;
  if (n_reads >= 0xffffffffull) return fail(MHMKC_EINVAL, "at most 2^32-2 reads per batch");
  uint64_t chunk = CHUNK_BYTES;
  if (g_dbg.chunk_bytes) chunk = std::max<uint64_t>(64, (uint64_t)g_dbg.chunk_bytes);
  if (xpipe) {  // the batch's windows, announced to the other ranks by the exchange rounds (the incremental layout)
    uint64_t w = 0;
    for (uint64_t r = 0; r < n_reads; r++) {
      const uint64_t L = offs[r + 1] >= offs[r] ? offs[r + 1] - offs[r] : 0;
      w += L > (uint64_t)k + 1 ? L - k - 1 : 0;
    }
    inc_expect += w;
    inc_announced += w;
  }
  if (g_dbg.h2d_nib > 0 || (g_dbg.h2d_nib < 0 && host_threads() >= 4))
    return add_host_nib(bytes, offs, n_reads, qcut, chunk);
  hipError_t e;
  Arena *ar = new_arena();
  if ((e = grow(ar->bytes, n_bases + 64)) != hipSuccess || (e = grow(ar->offs, (n_reads + 1) * 8)) != hipSuccess)
    return hip_fail(e, "input staging");
  qcut_pending = qcut;
  // the copies must not overwrite an arena that earlier work on the stream still reads
  (void)hipEventRecord(ev_h2d0, stream);
  if ((e = hipStreamWaitEvent(copy_stream, ev_h2d0, 0)) != hipSuccess) return hip_fail(e, "copy stream");
  (void)hipEventRecord(ev_h2d0, copy_stream);
  uint8_t *db = ar->bytes.as<uint8_t>();
  uint64_t *dofs = ar->offs.as<uint64_t>();
  const uint64_t kk = (uint64_t)k;
  size_t n_ev = 0;
  for (uint64_t r0 = 0; r0 < n_reads;) {
    // the chunk [r0, r1): whole reads, about `chunk` bytes; validate them and count their windows
    uint64_t r1 = r0, wins = 0;
    const uint64_t b0 = offs[r0];
    while (r1 < n_reads && (r1 == r0 || offs[r1] - b0 < chunk)) {
      const uint64_t a = offs[r1], b = offs[r1 + 1];
      if (b < a) return fail(MHMKC_EINVAL, "read_offsets must be non-decreasing (read %llu)", (unsigned long long)r1);
      if (b - a > 65535)
        return fail(MHMKC_EINVAL, "read %llu longer than 65535 (PackedRead read_len is uint16)", (unsigned long long)r1);
      if (b - a > kk + 1) wins += b - a - kk - 1;
      r1++;
    }
    const uint64_t b1 = offs[r1];
    if (b1 > b0 && (e = hipMemcpyAsync(db + b0, bytes + b0, b1 - b0, hipMemcpyHostToDevice, copy_stream)) != hipSuccess)
      return hip_fail(e, "input H2D");
    if ((e = hipMemcpyAsync(dofs + r0, offs + r0, (r1 - r0 + 1) * 8, hipMemcpyHostToDevice, copy_stream)) != hipSuccess)
      return hip_fail(e, "input H2D");
    if (n_ev == chunk_ev.size()) {
      hipEvent_t ev = nullptr;
      if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return hip_fail(e, "event");
      chunk_ev.push_back(ev);
    }
    hipEvent_t ev = chunk_ev[n_ev++];
    if ((e = hipEventRecord(ev, copy_stream)) != hipSuccess || (e = hipStreamWaitEvent(stream, ev, 0)) != hipSuccess)
      return hip_fail(e, "chunk event");
    st.h2d_bytes += (b1 - b0) + (r1 - r0 + 1) * 8;
    st.h2d_chunks++;
    // slice view: the bytes from the 16-byte aligned position at or below the chunk's first read (the bytes
    // before it belong to the previous chunk, copied earlier on the same stream)
    mhm::ReadsView rv{};
    rv.obase = b0 & ~15ull;
    rv.head = (uint32_t)(b0 - rv.obase);
    rv.bytes = db + rv.obase;
    rv.offs = dofs + r0;
    rv.n_reads = r1 - r0;
    rv.n_bases = b1 - rv.obase;
    if ((rc = add_view(rv, wins, true))) return rc;
    r0 = r1;
  }
  (void)hipEventRecord(ev_h2d1, copy_stream);
  // the caller's buffers are only borrowed for the call: wait for the copies (not for the extraction)
  if ((e = hipStreamSynchronize(copy_stream)) != hipSuccess) return hip_fail(e, "input H2D");
  float ms = 0;
  if (hipEventElapsedTime(&ms, ev_h2d0, ev_h2d1) == hipSuccess) st.ms_h2d = ms;
  return MHMKC_OK;
}

// add_host with the bases sent as nibbles (half the PCIe bytes). Per chunk of whole reads the host
// workers validate the offsets, count the windows and pack the bytes into a pinned slot (nib_pack) while the previous
// chunk is on the wire; the copy lands in a device slot that k_expand_nibbles turns back into PackedRead bytes in the
// arena, on the extraction's stream just before the chunk is extracted. With one rank the first chunk is a quarter of
// the others, so that the wire starts early.
int mhmkc::add_host_nib(const uint8_t *bytes, const uint64_t *offs, uint64_t n_reads, int qcut, uint64_t chunk) {
  const uint64_t n_bases = offs[n_reads];
  Workers &wk = Workers::get();
  const int T = wk.size();
  hipError_t e;
  int rc;
  Arena *ar = new_arena();
  if ((e = grow(ar->bytes, n_bases + 64)) != hipSuccess || (e = grow(ar->offs, (n_reads + 1) * 8)) != hipSuccess)
    return hip_fail(e, "input staging");
  // a chunk holds at most `chunk` bytes plus one read (<= 65535 bytes) and at most rmax reads; a slot holds its nibbles
  // and then, from byte dof, its offsets as u32 distances from its first byte (half the offsets' bytes)
  const uint64_t rmax = std::max<uint64_t>(64, chunk / 32);
  const size_t dof = (size_t)align_up(chunk / 2 + 65536 + 64, 64), slot = dof + 4 * (size_t)(rmax + 1);
  for (int s = 0; s < 3; s++) {
    if (slot > d_nib[s].cap) {
      if (nib_used[s] && (e = hipEventSynchronize(nib_ev[s])) != hipSuccess) return hip_fail(e, "nibble slot");
      if ((e = d_nib[s].ensure(slot)) != hipSuccess) return hip_fail(e, "nibble slot");
    }
    if (!nib_ev[s] && (e = hipEventCreateWithFlags(&nib_ev[s], hipEventDisableTiming)) != hipSuccess)
      return hip_fail(e, "event");
  }
  for (int s = 0; s < 2; s++)
    if (!stage_ev[s] && (e = hipEventCreateWithFlags(&stage_ev[s], hipEventDisableTiming)) != hipSuccess)
      return hip_fail(e, "event");
  // two pinned slots from the process's staging, given back (their copies done) however this call ends
  struct Slots {
    PinBuf *p[2] = {nullptr, nullptr};
    hipStream_t cs;
    ~Slots() {
      (void)hipStreamSynchronize(cs);
      H2DStage &g = h2d_stage();
      std::lock_guard<std::mutex> lk(g.mu);
      for (PinBuf *b : p)
        if (b) g.free.push_back(b);
    }
  } sl;
  sl.cs = copy_stream;
  {
    H2DStage &g = h2d_stage();
    std::lock_guard<std::mutex> lk(g.mu);
    for (PinBuf *&b : sl.p) {
      if (!g.free.empty()) {
        b = g.free.back();
        g.free.pop_back();
      } else {
        b = new PinBuf();
      }
    }
  }
  for (PinBuf *b : sl.p)
    if ((e = b->ensure(slot)) != hipSuccess) return hip_fail(e, "pinned staging");
  bool stage_used[2] = {false, false};
  double pack_ms = 0, wait_ms = 0, rounds_ms = 0;
  const bool deltas = g_dbg.h2d_nib != 2;  // (2: the offsets as they are, u64, from the caller's buffer; A/B runs)
  const int TP = g_dbg.h2d_threads > 0 ? (int)std::min<int64_t>(T, g_dbg.h2d_threads) : T;  // threads that pack
  // A chunk can go as it is (PackedRead bytes straight from the caller's buffer: twice the wire time, no host time) on
  // a host that packs much slower than the wire runs (see below; the wire at WIRE_BPMS). Only from pinned memory (a
  // pageable copy would hold the host).
  hipPointerAttribute_t pa{};
  const bool user_pinned = hipPointerGetAttributes(&pa, bytes) == hipSuccess && pa.type == hipMemoryTypeHost;
  (void)hipGetLastError();
  const int adapt = user_pinned ? (int)g_dbg.h2d_adapt : 0;  // 1: when drained, 2: every other chunk (tests)
  constexpr double WIRE_BPMS = 54e6;  // PCIe bytes per ms (the byte wire's measured 54-55 GB/s)
  double host_t = 0, packed_b = 0;  // the call's packing time and bytes packed so far
  double raw_acc = 0;                // the raw chunks owed so far (fraction)
  uint64_t raw_chunks = 0;
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto ms_since = [](std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  };
  qcut_pending = qcut;
  // the copies must not overwrite an arena that earlier work on the stream still reads
  (void)hipEventRecord(ev_h2d0, stream);
  if ((e = hipStreamWaitEvent(copy_stream, ev_h2d0, 0)) != hipSuccess) return hip_fail(e, "copy stream");
  (void)hipEventRecord(ev_h2d0, copy_stream);
  uint8_t *db = ar->bytes.as<uint8_t>();
  uint64_t *dofs = ar->offs.as<uint64_t>();
  const uint64_t kk = (uint64_t)k;
  size_t n_ev = 0;
  for (uint64_t r0 = 0, ci = 0; r0 < n_reads; ci++) {
    // the chunk [r0, r1): the first read r > r0 with offs[r] - b0 >= want ends it (a binary search; the offsets are
    // validated below, and a chunk whose end lies before its start is only validated, for the error)
    // (a quarter-size first chunk starts the wire early; not with the pipelined exchange, whose incremental layout
    // extrapolates from round 0, this chunk's slab: a smaller sample overestimated its distinct keys and output)
    const uint64_t b0 = offs[r0], want = ci == 0 && !xpipe ? std::max<uint64_t>(64, chunk / 4) : chunk;
    uint64_t lo = r0 + 1, hi = std::min(n_reads, r0 + rmax);
    while (lo < hi) {
      const uint64_t m = (lo + hi) / 2;
      if (offs[m] >= b0 && offs[m] - b0 < want)
        lo = m + 1;
      else
        hi = m;
    }
    const uint64_t r1 = lo, b1 = offs[r1];
    const bool span_ok = b1 >= b0 && b1 - b0 <= chunk + 65535;
    const int s = (int)(ci & 1), ds = (int)(ci % 3);
    auto tw = now();
    if (stage_used[s] && (e = hipEventSynchronize(stage_ev[s])) != hipSuccess)
      return hip_fail(e, "input H2D");
    wait_ms += ms_since(tw);
    uint8_t *stage = sl.p[s]->as<uint8_t>();
    uint32_t *sdelta = (uint32_t *)(stage + dof);
    const uint64_t nr = r1 - r0, nb = span_ok ? b1 - b0 : 0;
    bool raw = adapt == 2 && (ci & 1) != 0;
    if (adapt == 1 && ci >= 2 && packed_b > 0) {
      // from the third chunk on, with the packing rate of the first two: packing the whole batch P vs its nibbles on
      // the wire C. Below 1.6 C everything is packed (near P = C a raw chunk only lengthens the wire); above, a
      // fraction 2C / (P + C) of the chunks is packed and the rest sent raw, spread evenly, which balances the host's
      // f P against the wire's (2 - f) C
      const double P = host_t / packed_b * (double)n_bases, C = (double)n_bases / 2 / WIRE_BPMS;
      if (P > 1.6 * C) {
        raw_acc += 1.0 - 2 * C / (P + C);
        if (raw_acc >= 1.0) {
          raw = true;
          raw_acc -= 1.0;
        }
      }
    }
    std::vector<uint64_t> t_wins(T, 0), t_bad(T, UINT64_MAX), t_rest(T, 0);
    // (the second chunk's run also counts the windows of the reads after it: the local rounds' expected total)
    const bool announce = lrounds && ci == 1;
    std::vector<int> t_kind(T, 0);
    // local rounds due (slabs two chunks old): the calling thread enqueues them while the others pack
    const bool rounds_here = lrounds && n_slabs >= lq + 3 && T >= 2;
    const int U = rounds_here ? T - 1 : T, packers = std::min(TP, U);  // threads on the chunk's data
    int rounds_rc = MHMKC_OK;
    auto tp = now();
    wk.run([&](int t) {
      if (rounds_here && t == 0) {
        auto tl = now();
        rounds_rc = local_rounds(false);
        rounds_ms += ms_since(tl);
        return;
      }
      const int u = rounds_here ? t - 1 : t;
      // reads [r0 + u nr / U, r0 + (u + 1) nr / U): validated, their windows counted, their offsets' distances from
      // b0 staged (the last thread's also the chunk's end)
      const uint64_t ra = r0 + nr * u / U, rb = r0 + nr * (u + 1) / U;
      uint64_t w = 0;
      for (uint64_t r = ra; r < rb; r++) {
        const uint64_t a = offs[r], b = offs[r + 1];
        if (b < a || b - a > 65535) {
          t_bad[t] = r;
          t_kind[t] = b < a ? 1 : 2;
          break;
        }
        if (b - a > kk + 1) w += b - a - kk - 1;
        if (deltas) sdelta[r - r0] = (uint32_t)(a - b0);
      }
      if (deltas && u == U - 1) sdelta[nr] = (uint32_t)(b1 - b0);
      t_wins[t] = w;
      // bases [b0 + x, b0 + y) of an x that is a multiple of 64: nibbles from the 32-byte aligned byte x / 2 of the slot
      const uint64_t per = ((nb + packers - 1) / packers + 63) & ~63ull, x = std::min(nb, per * u),
                     y = std::min(nb, x + per);
      if (y > x && !raw) nib_pack(bytes + b0 + x, y - x, stage + x / 2, qcut, g_dbg.h2d_nt != 0);
      if (announce) {
        const uint64_t rest = n_reads - r1, qa = r1 + rest * u / U, qb = r1 + rest * (u + 1) / U;
        uint64_t wr = 0;
        for (uint64_t r = qa; r < qb; r++) {
          const uint64_t a = offs[r], b = offs[r + 1];
          if (b > a + kk + 1) wr += b - a - kk - 1;
        }
        t_rest[t] = wr;
      }
    });
    const double run_ms = ms_since(tp);
    pack_ms += run_ms;
    if (rounds_rc) return rounds_rc;
    if (!raw) {
      host_t += run_ms;
      packed_b += (double)nb;
    }
    uint64_t wins = 0;
    for (int t = 0; t < T; t++) {
      if (t_bad[t] != UINT64_MAX) {
        if (t_kind[t] == 1)
          return fail(MHMKC_EINVAL, "read_offsets must be non-decreasing (read %llu)", (unsigned long long)t_bad[t]);
        return fail(MHMKC_EINVAL, "read %llu longer than 65535 (PackedRead read_len is uint16)",
                    (unsigned long long)t_bad[t]);
      }
      wins += t_wins[t];
    }
    if (!span_ok) return fail(MHMKC_EHIP, "internal: H2D chunk of %llu bytes", (unsigned long long)(b1 - b0));
    if (announce) {
      uint64_t rest = 0;
      for (int t = 0; t < T; t++) rest += t_rest[t];
      inc_expect += rest;
      inc_announced += rest;
    }
    const uint64_t nbytes = raw ? nb : (nb + 1) / 2;
    uint8_t *dslot = d_nib[ds].as<uint8_t>();
    if (nib_used[ds] && (e = hipStreamWaitEvent(copy_stream, nib_ev[ds], 0)) != hipSuccess)
      return hip_fail(e, "copy stream");
    if ((nb && !raw && (e = hipMemcpyAsync(dslot, stage, nbytes, hipMemcpyHostToDevice, copy_stream)) != hipSuccess) ||
        (nb && raw && (e = hipMemcpyAsync(db + b0, bytes + b0, nb, hipMemcpyHostToDevice, copy_stream)) != hipSuccess) ||
        (deltas && (e = hipMemcpyAsync(dslot + dof, sdelta, 4 * (nr + 1), hipMemcpyHostToDevice, copy_stream)) != hipSuccess) ||
        (e = hipEventRecord(stage_ev[s], copy_stream)) != hipSuccess ||
        (!deltas && (e = hipMemcpyAsync(dofs + r0, offs + r0, (nr + 1) * 8, hipMemcpyHostToDevice, copy_stream)) != hipSuccess))
      return hip_fail(e, "input H2D");
    stage_used[s] = true;
    raw_chunks += raw;
    if (n_ev == chunk_ev.size()) {
      hipEvent_t ev = nullptr;
      if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return hip_fail(e, "event");
      chunk_ev.push_back(ev);
    }
    hipEvent_t ev = chunk_ev[n_ev++];
    if ((e = hipEventRecord(ev, copy_stream)) != hipSuccess || (e = hipStreamWaitEvent(stream, ev, 0)) != hipSuccess)
      return hip_fail(e, "chunk event");
    if ((!raw && (e = mhm::launch_expand_nibbles(dslot, db, b0, nb, stream)) != hipSuccess) ||
        (deltas && (e = mhm::launch_offs_from_deltas((const uint32_t *)(dslot + dof), dofs + r0, nr + 1, b0, stream)) != hipSuccess) ||
        (e = hipEventRecord(nib_ev[ds], stream)) != hipSuccess)
      return hip_fail(e, "nibble expansion");
    nib_used[ds] = true;
    st.h2d_bytes += nbytes + (nr + 1) * (deltas ? 4 : 8);
    st.h2d_chunks++;
    // slice view, as add_host's (the bytes before b0 in its first 16 belong to the previous chunk, expanded earlier on
    // the same stream)
    mhm::ReadsView rv{};
    rv.obase = b0 & ~15ull;
    rv.head = (uint32_t)(b0 - rv.obase);
    rv.bytes = db + rv.obase;
    rv.offs = dofs + r0;
    rv.n_reads = nr;
    rv.n_bases = b1 - rv.obase;
    if ((rc = add_view(rv, wins, true))) return rc;
    r0 = r1;
  }
  if (lrounds) {  // (the rounds that the last chunk made due)
    auto tl = now();
    if ((rc = local_rounds(false))) return rc;
    rounds_ms += ms_since(tl);
  }
  (void)hipEventRecord(ev_h2d1, copy_stream);
  if ((e = hipStreamSynchronize(copy_stream)) != hipSuccess) return hip_fail(e, "input H2D");
  float ms = 0;
  if (hipEventElapsedTime(&ms, ev_h2d0, ev_h2d1) == hipSuccess) st.ms_h2d = ms;
  st.ms_h2d_pack = pack_ms;
  st.ms_h2d_wait = wait_ms;
  st.ms_h2d_rounds = rounds_ms;
  st.h2d_raw_chunks = raw_chunks;
  return MHMKC_OK;
}

// ------------------------------------------------------------------------------------------------
// collectives between ranks: RCCL over xGMI (comm) or the caller's host transport (xp)

int mhmkc::allgather_host(const void *send, void *recv, size_t bytes, hipStream_t xs) {
  if (!xs) xs = stream;
  if (has_xp) {
    if (!xp.allgather || xp.allgather(xp.ctx, send, recv, bytes) != 0)
      return fail(MHMKC_ETRANSPORT, "transport allgather failed");
    return MHMKC_OK;
  }
  if (!comm) return fail(MHMKC_ETRANSPORT, "n_ranks > 1 needs comm_id or mhmkc_set_transport");
  const int g = G();
  hipError_t e;
  ncclResult_t nr;
  if ((e = grow(d_xg, bytes * (g + 1) + 64)) != hipSuccess) return hip_fail(e, "allgather buffer");
  char *d = d_xg.as<char>();
  if ((e = hipMemcpyAsync(d, send, bytes, hipMemcpyHostToDevice, xs)) != hipSuccess) return hip_fail(e, "allgather H2D");
  if ((nr = ncclAllGather(d, d + bytes, bytes, ncclUint8, comm, xs)) != ncclSuccess)
    return fail(MHMKC_ERCCL, "ncclAllGather: %s", ncclGetErrorString(nr));
  if ((e = hipMemcpyAsync(recv, d + bytes, bytes * g, hipMemcpyDeviceToHost, xs)) != hipSuccess ||
      (e = hipStreamSynchronize(xs)) != hipSuccess)
    return hip_fail(e, "allgather D2H");
  return MHMKC_OK;
}

// Point-to-point transfers of device buffers, given per peer in the same order on both sides (snd and rcv
// sorted by peer). RCCL: one group of ncclSend/ncclRecv. Host transport: staged through pinned memory,
// one alltoallv call.
int mhmkc::move(const std::vector<Xfer> &snd, const std::vector<Xfer> &rcv, hipStream_t xs) {
  const int g = G();
  if (!xs) xs = stream;
  hipError_t e;
  for (auto &x : snd) st.bytes_sent += x.bytes;
  for (auto &x : rcv) st.bytes_recv += x.bytes;
  if (has_xp) {
    std::vector<uint64_t> sb(g, 0), rb(g, 0);
    uint64_t ts = 0, tr = 0;
    for (auto &x : snd) sb[x.peer] += x.bytes, ts += x.bytes;
    for (auto &x : rcv) rb[x.peer] += x.bytes, tr += x.bytes;
    if ((e = x_send.ensure(ts + 64)) != hipSuccess || (e = x_recv.ensure(tr + 64)) != hipSuccess)
      return hip_fail(e, "exchange staging");
    char *hs = x_send.as<char>(), *hr = x_recv.as<char>();
    uint64_t o = 0;
    for (auto &x : snd) {
      if (x.bytes && (e = hipMemcpyAsync(hs + o, x.ptr, x.bytes, hipMemcpyDeviceToHost, xs)) != hipSuccess)
        return hip_fail(e, "exchange D2H");
      o += x.bytes;
    }
    if ((e = hipStreamSynchronize(xs)) != hipSuccess) return hip_fail(e, "exchange D2H");
    if (!xp.alltoallv || xp.alltoallv(xp.ctx, hs, sb.data(), hr, rb.data()) != 0)
      return fail(MHMKC_ETRANSPORT, "transport alltoallv failed");
    o = 0;
    for (auto &x : rcv) {
      if (x.bytes && (e = hipMemcpyAsync(x.ptr, hr + o, x.bytes, hipMemcpyHostToDevice, xs)) != hipSuccess)
        return hip_fail(e, "exchange H2D");
      o += x.bytes;
    }
    if ((e = hipStreamSynchronize(xs)) != hipSuccess) return hip_fail(e, "exchange H2D");  // x_recv is reused
    return MHMKC_OK;
  }
  if (!comm) return fail(MHMKC_ETRANSPORT, "n_ranks > 1 needs comm_id or mhmkc_set_transport");
  ncclResult_t nr;
  if ((nr = ncclGroupStart()) != ncclSuccess) return fail(MHMKC_ERCCL, "ncclGroupStart: %s", ncclGetErrorString(nr));
  for (auto &x : snd)
    if (x.bytes && (nr = ncclSend(x.ptr, x.bytes, ncclUint8, x.peer, comm, xs)) != ncclSuccess) break;
  if (nr == ncclSuccess)
    for (auto &x : rcv)
      if (x.bytes && (nr = ncclRecv(x.ptr, x.bytes, ncclUint8, x.peer, comm, xs)) != ncclSuccess) break;
  ncclResult_t ne = ncclGroupEnd();
  if (nr != ncclSuccess) return fail(MHMKC_ERCCL, "ncclSend/Recv: %s", ncclGetErrorString(nr));
  if (ne != ncclSuccess) return fail(MHMKC_ERCCL, "ncclGroupEnd: %s", ncclGetErrorString(ne));
  return MHMKC_OK;
}

// ------------------------------------------------------------------------------------------------
// hash-range exchange between ranks (replaces the UPC++ ThreeTierAggrStore<Supermer> traffic,
// src/kcount/kmer_dht.cpp:133-149,222-224, and its flush/barrier, kmer_dht.cpp:227-231)

int mhmkc::exchange(std::vector<Source> &srcs) {
  const int g = G(), me = cfg.rank;
  const uint32_t no = n_owned();
  int rc;
  // 1. number of slabs of every rank
  uint64_t my_slabs = n_slabs;
  std::vector<uint64_t> slabs_of(g);
  if ((rc = allgather_host(&my_slabs, slabs_of.data(), 8))) return rc;
  const uint64_t ms = std::max<uint64_t>(1, *std::max_element(slabs_of.begin(), slabs_of.end()));
  // 2. per slab: segment counts [nseg] and segment starts [nseg + 1] (capped slabs have gaps), of every rank
  const uint32_t nseg = nb * NSUB;
  const size_t per = 2 * (size_t)nseg + 1;
  std::vector<uint64_t> mine(ms * per, 0), all((size_t)g * ms * per, 0);
  for (size_t s = 0; s < n_slabs; s++) {
    std::copy(slabs[s]->counts.begin(), slabs[s]->counts.end(), mine.begin() + s * per);
    std::copy(slabs[s]->bases.begin(), slabs[s]->bases.end(), mine.begin() + s * per + nseg);
  }
  if ((rc = allgather_host(mine.data(), all.data(), 8 * ms * per))) return rc;
  auto cnt = [&](int r, uint64_t s, uint32_t i) { return all[((size_t)r * ms + s) * per + i]; };
  auto bas = [&](int r, uint64_t s, uint32_t i) { return all[((size_t)r * ms + s) * per + nseg + i]; };
  // 3. receive layout: for each peer p != me, for each of its slabs s, the span of my owned range
  uint64_t recv_total = 0;
  struct Seg {
    int peer;
    uint64_t slab, off, n;
  };
  std::vector<Seg> rsegs;
  for (int p = 0; p < g; p++) {
    if (p == me) continue;
    for (uint64_t s = 0; s < slabs_of[p]; s++) {
      const uint64_t n = bas(p, s, own_hi * NSUB) - bas(p, s, own_lo * NSUB);
      rsegs.push_back({p, s, recv_total, n});
      recv_total += n;
    }
  }
  mhm::PlaneSet rps{};
  if ((rc = set_planes(d_recv, recv_total, rps))) return rc;
  // 4. transfers, per peer in slab and plane order on both sides
  const bool aos = mixed2;  // one 16-byte record per entry in the first plane's place
  const int np = (compact || aos) ? 1 : nl;
  const size_t wb = compact ? 4 : aos ? 16 : 8;  // bytes of a word-plane entry
  std::vector<Xfer> snd, rcv;
  for (int p = 0; p < g; p++) {
    if (p == me) continue;
    const uint32_t lo = owner_lo(p), hi = owner_lo(p + 1);
    for (size_t s = 0; s < n_slabs; s++) {
      const Slab *sl = slabs[s];
      const uint64_t a = sl->bases[lo * NSUB], b = sl->bases[hi * NSUB];
      if (b == a) continue;
      for (int w = 0; w < np; w++) snd.push_back({p, (char *)sl->planes.w[w] + a * wb, (b - a) * wb});
      if (sl->planes.ext) snd.push_back({p, sl->planes.ext + a, b - a});
    }
  }
  for (const Seg &sg : rsegs) {
    if (!sg.n) continue;
    for (int w = 0; w < np; w++) rcv.push_back({sg.peer, (char *)rps.w[w] + sg.off * wb, sg.n * wb});
    if (rps.ext) rcv.push_back({sg.peer, rps.ext + sg.off, sg.n});
  }
  prof_begin(MHMKC_STAGE_XCHG);
  rc = move(snd, rcv);
  prof_end();
  if (rc) return rc;
  // 5. sources: local slabs (owned range in place) + received segments
  for (size_t s = 0; s < n_slabs; s++) {
    Source src;
    src.planes = slabs[s]->planes;
    src.start.assign(slabs[s]->bases.begin() + own_lo * NSUB, slabs[s]->bases.begin() + own_hi * NSUB);
    src.count.assign(slabs[s]->counts.begin() + own_lo * NSUB, slabs[s]->counts.begin() + own_hi * NSUB);
    srcs.push_back(std::move(src));
  }
  for (const Seg &sg : rsegs) {
    Source src;
    src.planes = rps;
    src.start.resize((size_t)no * NSUB);
    src.count.resize((size_t)no * NSUB);
    for (uint32_t i = 0; i < no * NSUB; i++) {
      src.start[i] = sg.off + (bas(sg.peer, sg.slab, own_lo * NSUB + i) - bas(sg.peer, sg.slab, own_lo * NSUB));
      src.count[i] = cnt(sg.peer, sg.slab, own_lo * NSUB + i);
    }
    srcs.push_back(std::move(src));
  }
  return MHMKC_OK;
}

// ------------------------------------------------------------------------------------------------
// pipelined hash-range exchange: one round per slab, its transfers on xstream while the main stream
// extracts the next slab (the reference ships supermers to their owners from process_seq, kmer_dht.cpp:222-224, and
// quiesces once at the end, :227-231). A round is collective: every rank takes part with its next unsent slab or with
// none, and says whether it is done (in finish, nothing left to add); rounds go on until every rank is done, so ranks
// with different numbers of slabs stay in step.

int mhmkc::xround(Slab *sl, bool done) {
  const int g = G(), me = cfg.rank;
  const uint32_t nseg = nb * NSUB, no = n_owned();
  int rc;
  hipError_t e;
  for (int pass = 0; sl && sl->pending; pass++) {
    bool redo = false;
    if ((rc = resolve_one(sl, redo))) return rc;
    if (redo && pass) return fail(MHMKC_EHIP, "internal: exact extraction overflowed");
  }
  // 1. every rank's flags (done, has a slab), the windows it announced, its slab's segment counts and starts (capped
  //    slabs have gaps)
  const size_t per = 2 * (size_t)nseg + 4;
  std::vector<uint64_t> mine(per, 0), all((size_t)g * per, 0);
  mine[0] = done;
  mine[1] = sl != nullptr;
  mine[2] = inc_expect;
  if (sl) {
    std::copy(sl->counts.begin(), sl->counts.end(), mine.begin() + 3);
    std::copy(sl->bases.begin(), sl->bases.end(), mine.begin() + 3 + nseg);
  }
  if ((rc = allgather_host(mine.data(), all.data(), 8 * per, xstream))) return rc;
  auto row = [&](int r) { return all.data() + (size_t)r * per; };
  bool all_done = true;
  x_expect_all = 0;
  for (int p = 0; p < g; p++) {
    all_done &= row(p)[0] != 0;
    x_expect_all += row(p)[2];
  }
  if (x_rounds == 0) {  // round 0's shares of the owned coarse buckets: the incremental partition's layout (inc_setup)
    x_r0_coarse.assign(no, 0);
    x_r0_total = 0;
    for (int p = 0; p < g; p++) {
      if (!row(p)[1]) continue;
      const uint64_t *pc = row(p) + 3;
      for (uint32_t i = 0; i < nseg; i++) x_r0_total += pc[i];
      for (uint32_t i = 0; i < no * NSUB; i++) x_r0_coarse[i / NSUB] += pc[own_lo * NSUB + i];
    }
  }
  // 2. receive layout: one span per peer with a slab this round, its records of my owned range, dense (the sender
  //    copies each capped segment's records back to back, step 3)
  std::vector<std::pair<int, uint64_t>> rsp;
  uint64_t recv_total = 0;
  for (int p = 0; p < g; p++) {
    if (p == me || !row(p)[1]) continue;
    const uint64_t *pc = row(p) + 3;
    uint64_t n = 0;
    for (uint32_t i = own_lo * NSUB; i < own_hi * NSUB; i++) n += pc[i];
    rsp.push_back({p, n});
    recv_total += n;
  }
  if (n_parts == parts.size()) parts.push_back(new RecvPart());
  RecvPart *rp = parts[n_parts++];
  rp->spans.clear();
  if ((rc = set_planes(rp->buf, recv_total, rp->planes))) return rc;
  uint64_t off = 0;
  for (auto &pn : rsp) {
    RecvPart::Span sp;
    sp.off = off;
    sp.start.resize((size_t)no * NSUB);
    sp.count.resize((size_t)no * NSUB);
    const uint64_t *pc = row(pn.first) + 3;
    uint64_t o = off;
    for (uint32_t i = 0; i < no * NSUB; i++) {
      sp.start[i] = o;
      sp.count[i] = pc[own_lo * NSUB + i];
      o += sp.count[i];
    }
    rp->spans.push_back(std::move(sp));
    off += pn.second;
  }
  // 3. transfers, per peer in plane order on both sides (as exchange()). The send side copies the filled part of every
  //    segment a peer owns back to back into the send planes (k_seg_gather on xstream, after the slab's extraction):
  //    a slab's owned range carries the capped segments' slack (4 % + a constant), which the wire need not (bytes
  //    per occurrence at 8 ranks 4.79 -> 4.375, the records' 5 B x 7/8)
  const bool aos = mixed2;
  const int np = (compact || aos) ? 1 : nl;
  const size_t wb = compact ? 4 : aos ? 16 : 8;
  std::vector<Xfer> snd, rcv;
  x_segs.clear();
  uint64_t send_total = 0;
  std::vector<uint64_t> peer_off(g + 1, 0);
  if (sl) {
    for (int p = 0; p < g; p++) {
      peer_off[p] = send_total;
      if (p == me) continue;
      for (uint32_t i = owner_lo(p) * NSUB; i < owner_lo(p + 1) * NSUB; i++)
        if (sl->counts[i]) {
          x_segs.push_back({sl->bases[i], send_total, sl->counts[i]});
          send_total += sl->counts[i];
        }
    }
    peer_off[g] = send_total;
  }
  mhm::PlaneSet sps{};
  if (send_total) {
    // (xstream may still send the previous round from the send planes: a larger allocation waits for it)
    const uint64_t need = send_total;
    if (x_send_cap < need && (e = hipStreamSynchronize(xstream)) != hipSuccess) return hip_fail(e, "exchange stream");
    if ((rc = set_planes(d_xsend, need, sps, false, false))) return rc;
    x_send_cap = std::max(x_send_cap, need);
    for (int p = 0; p < g; p++) {
      const uint64_t a = peer_off[p], b = p + 1 < g ? peer_off[p + 1] : send_total;
      if (p == me || b == a) continue;
      for (int w = 0; w < np; w++) snd.push_back({p, (char *)sps.w[w] + a * wb, (b - a) * wb});
      if (sps.ext) snd.push_back({p, sps.ext + a, b - a});
    }
  }
  off = 0;
  for (auto &pn : rsp) {
    if (pn.second) {
      for (int w = 0; w < np; w++) rcv.push_back({pn.first, (char *)rp->planes.w[w] + off * wb, pn.second * wb});
      if (rp->planes.ext) rcv.push_back({pn.first, rp->planes.ext + off, pn.second});
    }
    off += pn.second;
  }
  // 4. on xstream, after the slab's extraction (not after what the main stream was given since)
  while (x_ev.size() < 2 * (x_rounds + 1)) {
    hipEvent_t ev = nullptr;
    if ((e = hipEventCreate(&ev)) != hipSuccess) return hip_fail(e, "exchange event");
    x_ev.push_back(ev);
  }
  if (sl && (e = hipStreamWaitEvent(xstream, sl->ev, 0)) != hipSuccess) return hip_fail(e, "exchange wait");
  (void)hipEventRecord(x_ev[2 * x_rounds], xstream);
  if (!x_segs.empty()) {
    const size_t sb = x_segs.size() * sizeof(mhm::SegCopy);
    if (d_xsegs.cap < sb && (e = hipStreamSynchronize(xstream)) != hipSuccess) return hip_fail(e, "exchange stream");
    if ((e = d_xsegs.ensure(sb)) != hipSuccess) return hip_fail(e, "exchange segments");
    mhm::SegCopy *ds = d_xsegs.as<mhm::SegCopy>();
    // (x_segs lives in the handle until the next round, which first waits for this one's copy: the H2D is on xstream)
    if ((e = hipMemcpyAsync(ds, x_segs.data(), sb, hipMemcpyHostToDevice, xstream)) != hipSuccess)
      return hip_fail(e, "exchange segments");
    for (int w = 0; w < np && e == hipSuccess; w++)
      e = mhm::launch_seg_gather(ds, (uint32_t)x_segs.size(), sl->planes.w[w], sps.w[w], (int)wb, xstream);
    if (e == hipSuccess && sl->planes.ext)
      e = mhm::launch_seg_gather(ds, (uint32_t)x_segs.size(), sl->planes.ext, sps.ext, 1, xstream);
    if (e != hipSuccess) return hip_fail(e, "exchange gather");
  }
  if ((rc = move(snd, rcv, xstream))) return rc;
  (void)hipEventRecord(x_ev[2 * x_rounds + 1], xstream);
  x_round_slab.push_back(sl ? (int)(std::find(slabs.begin(), slabs.begin() + (long)n_slabs, sl) - slabs.begin()) : -1);
  x_rounds++;
  x_all_done = all_done;
  // the incremental partition: its layout once round 0 has landed (while round 1's transfer and the
  // next slab's extraction run), then every round on pstream as it lands
  if (!inc_tried && x_rounds >= 2 && (rc = inc_setup())) return rc;
  if (inc)
    for (; inc_parted < x_rounds; inc_parted++)
      if ((rc = inc_round(inc_parted))) return rc;
  return MHMKC_OK;
}

// Send every slab but the newest (whose extraction is what the next round overlaps).
int mhmkc::pump() {
  while (xpipe && n_slabs >= xq + 2) {
    int rc = xround(slabs[xq], false);
    if (rc) return rc;
    xq++;
  }
  return MHMKC_OK;
}

// ------------------------------------------------------------------------------------------------
// supermer exchange: MHMKC_OWNER_MINIMIZER with several ranks and keys of two or more words.
// A read slab becomes supermers per destination rank (get_kmer_target_rank, kmer_dht.cpp:193-196) instead of
// records; finish ships them (the reference's add_supermer -> ThreeTierAggrStore, kmer_dht.cpp:222-224) and every
// rank extracts the records of the supermers it received, over the whole hash range.

int mhmkc::smer_build(Slab *sl) {
  const int T = mhm::tile_bases(nl), g = G();
  hipError_t e;
  if ((e = grow(d_tiles, (size_t)sl->tiles * 4 + 64)) != hipSuccess) return hip_fail(e, "tile index");
  if ((e = grow(d_owners, (size_t)sl->tiles * T + 64)) != hipSuccess) return hip_fail(e, "supermer owners");
  constexpr int NS = mhm::SMER_SLICES;
  const size_t nc = 2 * (size_t)g * NS;  // [destination][slice][words, supermers]
  if ((e = sl->meta.ensure(nc * 16 + 64)) != hipSuccess) return hip_fail(e, "supermer counters");
  if ((e = sl->pin.ensure(nc * 16 + 64)) != hipSuccess) return hip_fail(e, "supermer counters (host)");
  unsigned long long *hist = sl->meta.as<unsigned long long>(), *cur = hist + nc;
  mhm::SmerParams sp{};
  sp.reads = sl->rv;
  sp.tile_first_read = d_tiles.as<uint32_t>();
  sp.n_tiles = sl->tiles;
  sp.k = k;
  sp.m = mlen;
  sp.n_ranks = g;
  sp.qual_cutoff = sl->qcut;
  sp.owners = d_owners.as<uint8_t>();
  sp.hist = hist;
  sp.cursor = cur;
  sp.err = d_err.as<unsigned int>();
  prof_begin(MHMKC_STAGE_TILEIDX);
  e = mhm::launch_tile_first_read(sl->rv, d_tiles.as<uint32_t>(), sl->tiles, T, stream);
  prof_end();
  if (e == hipSuccess) e = hipMemsetAsync(hist, 0, nc * 8, stream);
  if (e != hipSuccess) return hip_fail(e, "supermer owners");
  prof_begin(MHMKC_STAGE_EHIST);
  e = mhm::launch_smer_owner(sp, nl, stream);
  prof_end();
  if (e != hipSuccess) return hip_fail(e, "smer_owner");
  uint64_t *hc = sl->pin.as<uint64_t>();
  if ((e = hipMemcpyAsync(hc, hist, nc * 8, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
      (e = hipStreamSynchronize(stream)) != hipSuccess)
    return hip_fail(e, "supermer counts");
  sl->sw.assign(g, 0), sl->ss.assign(g, 0), sl->swb.assign(g + 1, 0), sl->ssb.assign(g + 1, 0);
  uint64_t *hcur = hc + nc;  // cursors: destination-major spans, each cut into its slices in order
  uint64_t wacc = 0, sacc = 0;
  for (int d = 0; d < g; d++) {
    for (int q = 0; q < NS; q++) {
      const size_t i = 2 * ((size_t)d * NS + q);
      hcur[i] = wacc;
      hcur[i + 1] = sacc;
      wacc += hc[i];
      sacc += hc[i + 1];
      sl->sw[d] += hc[i];
      sl->ss[d] += hc[i + 1];
    }
    sl->swb[d + 1] = sl->swb[d] + sl->sw[d];
    sl->ssb[d + 1] = sl->ssb[d] + sl->ss[d];
  }
  const uint64_t W = sl->swb[g], S = sl->ssb[g];
  const size_t cb_ = align_up(W * 8 + 16, 256), gb_ = align_up(W * 4 + 16, 256);
  if ((e = grow(sl->buf, cb_ + gb_ + S * 8 + 64)) != hipSuccess) return hip_fail(e, "supermer planes");
  sl->codes = sl->buf.as<uint64_t>();
  sl->good = (uint32_t *)(sl->buf.as<char>() + cb_);
  sl->desc = (uint64_t *)(sl->buf.as<char>() + cb_ + gb_);
  if ((e = hipMemcpyAsync(cur, hcur, nc * 8, hipMemcpyHostToDevice, stream)) != hipSuccess)
    return hip_fail(e, "supermer cursors");
  sp.codes = sl->codes;
  sp.good = sl->good;
  sp.desc = sl->desc;
  sp.n_words = W;
  sp.n_smer = S;
  prof_begin(MHMKC_STAGE_ESCAT);
  e = mhm::launch_smer_pack(sp, nl, stream);
  prof_end();
  if (e != hipSuccess) return hip_fail(e, "smer_pack");
  sl->n = sl->wins;
  sl->pending = false;
  st.smer_words += W;
  st.smer_count += S;
  // the pinned counters are read back into the host vectors above; the pack's cursor copy must land before the
  // next slab reuses them (one pinned buffer per slab: no reuse within a round)
  return MHMKC_OK;
}

int mhmkc::smer_exchange(std::vector<Source> &srcs) {
  const int g = G(), me = cfg.rank;
  int rc;
  hipError_t e;
  // 1. every rank's per-slab span sizes (words, supermers per destination)
  uint64_t my_slabs = n_slabs;
  std::vector<uint64_t> slabs_of(g);
  if ((rc = allgather_host(&my_slabs, slabs_of.data(), 8))) return rc;
  const uint64_t ms = std::max<uint64_t>(1, *std::max_element(slabs_of.begin(), slabs_of.end()));
  const size_t per = 2 * (size_t)g;
  std::vector<uint64_t> mine(ms * per, 0), all((size_t)g * ms * per, 0);
  for (size_t s = 0; s < n_slabs; s++)
    for (int d = 0; d < g; d++) {
      mine[s * per + 2 * d] = slabs[s]->sw[d];
      mine[s * per + 2 * d + 1] = slabs[s]->ss[d];
    }
  if ((rc = allgather_host(mine.data(), all.data(), 8 * ms * per))) return rc;
  auto W_of = [&](int p, uint64_t s) { return all[((size_t)p * ms + s) * per + 2 * me]; };
  auto S_of = [&](int p, uint64_t s) { return all[((size_t)p * ms + s) * per + 2 * me + 1]; };
  // 2. the received spans back to back in (peer, slab) order, this rank's own among them
  // a descriptor's word offset counts from the start of its sender's slab planes, where this rank's span starts
  // after the spans of the lower destinations (sb)
  struct Span {
    int peer;
    uint64_t slab, w0, s0, nw, ns, sb;
  };
  std::vector<Span> spans;
  uint64_t Wt = 0, St = 0;
  for (int p = 0; p < g; p++)
    for (uint64_t s = 0; s < slabs_of[p]; s++) {
      const uint64_t nw = W_of(p, s), ns = S_of(p, s);
      uint64_t sb = 0;
      for (int d = 0; d < me; d++) sb += all[((size_t)p * ms + s) * per + 2 * d];
      if (ns) spans.push_back({p, s, Wt, St, nw, ns, sb});
      Wt += nw;
      St += ns;
    }
  if ((e = grow(d_rcodes, Wt * 8 + 64)) != hipSuccess || (e = grow(d_rgood, Wt * 4 + 64)) != hipSuccess ||
      (e = grow(d_rdesc, St * 8 + 64)) != hipSuccess || (e = grow(d_rnwin, (St + 1) * 8 + 64)) != hipSuccess ||
      (e = grow(d_rwpre, (St + 1) * 8 + 64)) != hipSuccess)
    return hip_fail(e, "supermer receive buffers");
  uint64_t *rcodes = d_rcodes.as<uint64_t>(), *rdesc = d_rdesc.as<uint64_t>();
  uint32_t *rgood = d_rgood.as<uint32_t>();
  std::vector<Xfer> snd, rcv;
  for (int p = 0; p < g; p++) {
    if (p == me) continue;
    for (size_t s = 0; s < n_slabs; s++) {
      const Slab *sl = slabs[s];
      if (!sl->ss[p]) continue;
      snd.push_back({p, sl->codes + sl->swb[p], sl->sw[p] * 8});
      snd.push_back({p, sl->good + sl->swb[p], sl->sw[p] * 4});
      snd.push_back({p, sl->desc + sl->ssb[p], sl->ss[p] * 8});
    }
  }
  for (const Span &sp : spans) {
    if (sp.peer == me) {  // this rank's own supermers: device copies
      const Slab *sl = slabs[sp.slab];
      if ((e = hipMemcpyAsync(rcodes + sp.w0, sl->codes + sl->swb[me], sp.nw * 8, hipMemcpyDeviceToDevice, stream)) != hipSuccess ||
          (e = hipMemcpyAsync(rgood + sp.w0, sl->good + sl->swb[me], sp.nw * 4, hipMemcpyDeviceToDevice, stream)) != hipSuccess ||
          (e = hipMemcpyAsync(rdesc + sp.s0, sl->desc + sl->ssb[me], sp.ns * 8, hipMemcpyDeviceToDevice, stream)) != hipSuccess)
        return hip_fail(e, "own supermers");
      continue;
    }
    rcv.push_back({sp.peer, rcodes + sp.w0, sp.nw * 8});
    rcv.push_back({sp.peer, rgood + sp.w0, sp.nw * 4});
    rcv.push_back({sp.peer, rdesc + sp.s0, sp.ns * 8});
  }
  prof_begin(MHMKC_STAGE_XCHG);
  rc = move(snd, rcv);
  prof_end();
  if (rc) return rc;
  // 3. descriptors rebased to the concatenated stream, the window prefix, the tile index
  unsigned long long *nwin = d_rnwin.as<unsigned long long>(), *wpre = d_rwpre.as<unsigned long long>();
  prof_begin(MHMKC_STAGE_OTHER);
  for (const Span &sp : spans)
    if ((e = mhm::launch_smer_rebase(rdesc + sp.s0, sp.ns, sp.w0 - sp.sb, nwin + sp.s0, stream)) != hipSuccess) break;
  if (e == hipSuccess) e = hipMemsetAsync(nwin + St, 0, 8, stream);
  const size_t tb = mhm::fq_scan_tmp_bytes(St + 1);
  if (e == hipSuccess) e = grow(d_rtmp, tb + 64);
  if (e == hipSuccess) e = mhm::fq_scan(d_rtmp.p, tb, nwin, wpre, St + 1, stream);
  prof_end();
  if (e != hipSuccess) return hip_fail(e, "supermer descriptors");
  unsigned long long n_win = 0;
  if ((e = hipMemcpyAsync(&n_win, wpre + St, 8, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
      (e = hipStreamSynchronize(stream)) != hipSuccess)
    return hip_fail(e, "supermer windows");
  const int T = mhm::tile_bases(nl);
  const uint64_t tiles64 = (n_win + T - 1) / T;
  if (tiles64 >= 0x7fffffffull) return fail(MHMKC_EINVAL, "too many received windows in one round");
  if ((e = grow(d_rtiles, (tiles64 + 2) * 8)) != hipSuccess) return hip_fail(e, "supermer tiles");
  prof_begin(MHMKC_STAGE_TILEIDX);
  e = mhm::launch_smer_tiles((const uint64_t *)wpre, St, d_rtiles.as<uint64_t>(), (uint32_t)tiles64, T, stream);
  prof_end();
  if (e != hipSuccess) return hip_fail(e, "supermer tiles");
  rsrc = mhm::SmerSource{rcodes, rgood, rdesc, (const uint64_t *)wpre, d_rtiles.as<uint64_t>(), St, n_win, Wt + 2};
  // 4. the received windows' records are extracted per finish pass (smer_records), one more slab
  smer_nwin = n_win;
  smer_tiles = (uint32_t)tiles64;
  (void)srcs;
  return MHMKC_OK;
}

// The records of the received supermers whose coarse bucket is in [lo, hi) (a finish pass; all of them when the pass
// covers the whole range), as the recv slab (capped layout; an overflow reruns it exactly); appended to srcs.
int mhmkc::smer_records(uint32_t lo, uint32_t hi, std::vector<Source> &srcs) {
  if (!smer_nwin) return MHMKC_OK;
  int rc;
  if (!smer_slab) smer_slab = new Slab();
  Slab *rs = smer_slab;
  rs->recv = true;
  rs->rv = mhm::ReadsView{};
  rs->wins = smer_nwin;
  rs->tiles = smer_tiles;
  rs->qcut = cfg.qual_cutoff;
  rs->n = 0;
  rs->bin_lo = lo;
  rs->bin_hi = (lo == 0 && hi == nb) ? 0 : hi;
  if ((rc = extract(rs, g_dbg.exact != 0))) return rc;
  for (int pass = 0; rs->pending; pass++) {
    bool redo = false;
    if ((rc = resolve_one(rs, redo))) return rc;
    if (redo && pass) return fail(MHMKC_EHIP, "internal: exact extraction overflowed");
  }
  uint64_t tot = 0;
  for (uint64_t c : rs->counts) tot += c;
  smer_seen += tot;
  Source src;
  src.planes = rs->planes;
  src.start.assign(rs->bases.begin(), rs->bases.begin() + (size_t)nb * NSUB);
  src.count = rs->counts;
  srcs.push_back(std::move(src));
  return MHMKC_OK;
}

// ------------------------------------------------------------------------------------------------
// contig pass: extract, fold and bucket the contig k-mers (kcount_ctg.hip); k_count applies them

// With several ranks every rank needs the contigs of all ranks, in one order, for the k-mers of its hash
// range: the contigs are all-gathered (rank order). They are small next to the reads (an assembly's
// contigs are about the genome; the reads are 30x it).
int mhmkc::gather_ctgs(std::vector<uint8_t> &gb, std::vector<uint64_t> &go, std::vector<uint64_t> &gw,
                       std::vector<uint16_t> &gd) {
  const int g = G();
  int rc;
  uint64_t mine[2] = {ctg_depth.size(), ctg_bytes.size()};
  std::vector<uint64_t> sizes(2 * (size_t)g);
  if ((rc = allgather_host(mine, sizes.data(), 16))) return rc;
  uint64_t max_c = 0, max_b = 0, tot_c = 0;
  for (int r = 0; r < g; r++) {
    max_c = std::max(max_c, sizes[2 * r]);
    max_b = std::max(max_b, sizes[2 * r + 1]);
    tot_c += sizes[2 * r];
  }
  gb.clear();
  go.assign(1, 0);
  gw.assign(1, 0);
  gd.clear();
  if (!tot_c) return MHMKC_OK;
  // one record per rank: [lengths: max_c u64][depths: max_c u16, padded to 8][bytes: max_b, padded to 8]
  const size_t rec = 8 * max_c + align_up(2 * max_c, 8) + align_up(max_b, 8);
  std::vector<uint8_t> mr(rec, 0), all(rec * g);
  for (size_t i = 0; i < ctg_depth.size(); i++) ((uint64_t *)mr.data())[i] = ctg_offs[i + 1] - ctg_offs[i];
  if (!ctg_depth.empty()) memcpy(mr.data() + 8 * max_c, ctg_depth.data(), 2 * ctg_depth.size());
  if (!ctg_bytes.empty()) memcpy(mr.data() + 8 * max_c + align_up(2 * max_c, 8), ctg_bytes.data(), ctg_bytes.size());
  if ((rc = allgather_host(mr.data(), all.data(), rec))) return rc;
  for (int r = 0; r < g; r++) {
    const uint8_t *q = all.data() + rec * r;
    const uint64_t *lens = (const uint64_t *)q;
    const uint16_t *dep = (const uint16_t *)(q + 8 * max_c);
    const uint8_t *byt = q + 8 * max_c + align_up(2 * max_c, 8);
    gb.insert(gb.end(), byt, byt + sizes[2 * r + 1]);
    for (uint64_t i = 0; i < sizes[2 * r]; i++) {
      const uint64_t L = lens[i];
      go.push_back(go.back() + L);
      gw.push_back(gw.back() + (L >= (uint64_t)k + 2 ? L - k - 1 : 0));
      gd.push_back(dep[i]);
    }
  }
  if (gw.back() >= 0xffffffffull) return fail(MHMKC_EINVAL, "at most 2^32-1 contig k-mers per round");
  return MHMKC_OK;
}

int mhmkc::prepare_ctgs() {
  ctg_n = 0;
  const std::vector<uint8_t> *cb_ = &ctg_bytes;
  const std::vector<uint64_t> *co = &ctg_offs, *cw = &ctg_win;
  const std::vector<uint16_t> *cd = &ctg_depth;
  if (G() > 1) {
    if (!ctg_gathered) {  // (collective: every rank gathers exactly once per finish)
      int rc = gather_ctgs(ctg_gbytes, ctg_goffs, ctg_gwin, ctg_gdepth);
      if (rc) return rc;
      ctg_gathered = true;
    }
    cb_ = &ctg_gbytes, co = &ctg_goffs, cw = &ctg_gwin, cd = &ctg_gdepth;
  }
  const uint64_t W = cw->back();
  if (!W) return MHMKC_OK;
  hipError_t e;
  const uint64_t nc = cd->size();
  if ((e = grow(d_ctg_bytes, cb_->size() + 64)) != hipSuccess || (e = grow(d_ctg_offs, (nc + 1) * 8)) != hipSuccess ||
      (e = grow(d_ctg_win, (nc + 1) * 8)) != hipSuccess || (e = grow(d_ctg_depth, nc * 2 + 2)) != hipSuccess)
    return hip_fail(e, "contig staging");
  if ((e = hipMemcpyAsync(d_ctg_bytes.p, cb_->data(), cb_->size(), hipMemcpyHostToDevice, stream)) != hipSuccess ||
      (e = hipMemcpyAsync(d_ctg_offs.p, co->data(), (nc + 1) * 8, hipMemcpyHostToDevice, stream)) != hipSuccess ||
      (e = hipMemcpyAsync(d_ctg_win.p, cw->data(), (nc + 1) * 8, hipMemcpyHostToDevice, stream)) != hipSuccess ||
      (e = hipMemcpyAsync(d_ctg_depth.p, cd->data(), nc * 2, hipMemcpyHostToDevice, stream)) != hipSuccess)
    return hip_fail(e, "contig H2D");
  const size_t sb = mhm::ctg_scratch_bytes(W, nl);
  if ((e = grow(d_ctg_scratch, sb)) != hipSuccess) return hip_fail(e, "contig scratch");
  uint64_t *keys[4] = {nullptr, nullptr, nullptr, nullptr};
  for (int w = 0; w < nl; w++) {
    if ((e = grow(d_ctg_keys[w], W * 8)) != hipSuccess) return hip_fail(e, "contig keys");
    keys[w] = d_ctg_keys[w].as<uint64_t>();
  }
  if ((e = grow(d_ctg_state, W * 4)) != hipSuccess || (e = grow(d_ctg_bucket, W * 4)) != hipSuccess ||
      (e = grow(d_ctg_done, W)) != hipSuccess)
    return hip_fail(e, "contig entries");
  mhm::CtgView cv{d_ctg_bytes.as<uint8_t>(), d_ctg_offs.as<uint64_t>(), d_ctg_depth.as<uint16_t>(),
                  d_ctg_win.as<uint64_t>(), nc, W};
  prof_begin(MHMKC_STAGE_OTHER);
  // the synchronous copies above keep the host vectors alive long enough: ctg_prepare waits for its
  // fold count before returning
  const mhm::CtgOwner ow{smer ? G() : 0, cfg.rank, mlen};  // supermer exchange: keep this rank's target k-mers
  e = mhm::ctg_prepare(cv, k, nl, mixed(), 1, dmin, 1.0 - cfg.dyn_min_depth, cb, fb, own_lo, own_hi, ow,
                       d_ctg_scratch.p, sb, keys, d_ctg_state.as<uint32_t>(), d_ctg_bucket.as<uint32_t>(), &ctg_n,
                       d_err.as<unsigned int>(), stream);
  prof_end();
  if (e != hipSuccess) return hip_fail(e, "contig pass");
  st.ctg_kmers = ctg_n;
  return MHMKC_OK;
}

// ------------------------------------------------------------------------------------------------
// owner hand-off: move every finished k-mer to get_kmer_target_rank (MHMKC_OWNER_MINIMIZER)

int mhmkc::handoff() {
  const int g = G(), me = cfg.rank;
  hipError_t e;
  int rc;
  const uint64_t n = n_out;
  if ((e = grow(d_dest, n + 64)) != hipSuccess || (e = grow(d_ohist, 16 * (size_t)g + 64)) != hipSuccess)
    return hip_fail(e, "hand-off buffers");
  std::vector<uint64_t> hist(g, 0), start(g, 0);
  prof_begin(MHMKC_STAGE_OTHER);
  e = hipMemsetAsync(d_ohist.p, 0, 8 * (size_t)g, stream);
  if (e == hipSuccess)
    e = mhm::launch_owner_hist(d_out_keys.as<uint64_t>(), n, nlo, k, mlen, g, d_dest.as<uint8_t>(),
                               d_ohist.as<unsigned long long>(), stream);
  prof_end();
  if (e == hipSuccess) e = hipMemcpyAsync(hist.data(), d_ohist.p, 8 * (size_t)g, hipMemcpyDeviceToHost, stream);
  if (e == hipSuccess) e = hipStreamSynchronize(stream);
  if (e != hipSuccess) return hip_fail(e, "owner histogram");
  for (int r = 1; r < g; r++) start[r] = start[r - 1] + hist[r - 1];
  // rows grouped by owner into the second output set
  if ((e = grow(d_out2_keys, n * 8 * nlo + 64)) != hipSuccess || (e = grow(d_out2_counts, n * 2 + 64)) != hipSuccess ||
      (e = grow(d_out2_left, n + 64)) != hipSuccess || (e = grow(d_out2_right, n + 64)) != hipSuccess)
    return hip_fail(e, "hand-off buffers");
  mhm::OutRows in{d_out_keys.as<uint64_t>(), d_out_counts.as<uint16_t>(), d_out_left.as<char>(), d_out_right.as<char>()};
  mhm::OutRows grp{d_out2_keys.as<uint64_t>(), d_out2_counts.as<uint16_t>(), d_out2_left.as<char>(),
                   d_out2_right.as<char>()};
  prof_begin(MHMKC_STAGE_OTHER);
  e = hipMemcpyAsync(d_ohist.as<uint64_t>() + g, start.data(), 8 * (size_t)g, hipMemcpyHostToDevice, stream);
  if (e == hipSuccess)
    e = mhm::launch_owner_scatter(in, n, nlo, d_dest.as<uint8_t>(), g, d_ohist.as<unsigned long long>() + g, grp, stream);
  prof_end();
  if (e != hipSuccess) return hip_fail(e, "owner scatter");
  // who sends whom how many rows
  std::vector<uint64_t> mat((size_t)g * g);
  if ((rc = allgather_host(hist.data(), mat.data(), 8 * (size_t)g))) return rc;
  auto M = [&](int from, int to) { return mat[(size_t)from * g + to]; };
  uint64_t new_n = 0;
  std::vector<uint64_t> roff(g, 0);
  roff[me] = 0;
  new_n = M(me, me);
  for (int p = 0; p < g; p++) {
    if (p == me) continue;
    roff[p] = new_n;
    new_n += M(p, me);
  }
  // the final rows go back into the first output set (its old contents were grouped into the second)
  if ((e = hipStreamSynchronize(stream)) != hipSuccess) return hip_fail(e, "owner scatter");
  if ((e = grow(d_out_keys, new_n * 8 * nlo + 64)) != hipSuccess || (e = grow(d_out_counts, new_n * 2 + 64)) != hipSuccess ||
      (e = grow(d_out_left, new_n + 64)) != hipSuccess || (e = grow(d_out_right, new_n + 64)) != hipSuccess)
    return hip_fail(e, "hand-off output");
  const size_t kb = 8 * (size_t)nlo;
  char *ok = d_out_keys.as<char>(), *oc = d_out_counts.as<char>(), *ol = d_out_left.as<char>(),
       *orr = d_out_right.as<char>();
  char *gk = d_out2_keys.as<char>(), *gc = d_out2_counts.as<char>(), *gl = d_out2_left.as<char>(),
       *gr = d_out2_right.as<char>();
  const uint64_t mine_n = hist[me], ms = start[me];
  if (mine_n) {
    if ((e = hipMemcpyAsync(ok, gk + ms * kb, mine_n * kb, hipMemcpyDeviceToDevice, stream)) != hipSuccess ||
        (e = hipMemcpyAsync(oc, gc + ms * 2, mine_n * 2, hipMemcpyDeviceToDevice, stream)) != hipSuccess ||
        (e = hipMemcpyAsync(ol, gl + ms, mine_n, hipMemcpyDeviceToDevice, stream)) != hipSuccess ||
        (e = hipMemcpyAsync(orr, gr + ms, mine_n, hipMemcpyDeviceToDevice, stream)) != hipSuccess)
      return hip_fail(e, "hand-off copy");
  }
  std::vector<Xfer> snd, rcv;
  for (int p = 0; p < g; p++) {
    if (p == me) continue;
    const uint64_t a = start[p], c = hist[p];
    if (c) {
      snd.push_back({p, gk + a * kb, c * kb});
      snd.push_back({p, gc + a * 2, c * 2});
      snd.push_back({p, gl + a, c});
      snd.push_back({p, gr + a, c});
      st.handoff_sent += c;
    }
    const uint64_t rn = M(p, me), ro = roff[p];
    if (rn) {
      rcv.push_back({p, ok + ro * kb, rn * kb});
      rcv.push_back({p, oc + ro * 2, rn * 2});
      rcv.push_back({p, ol + ro, rn});
      rcv.push_back({p, orr + ro, rn});
      st.handoff_recv += rn;
    }
  }
  const uint64_t sent0 = st.bytes_sent, recv0 = st.bytes_recv;
  prof_begin(MHMKC_STAGE_XCHG);
  rc = move(snd, rcv);
  prof_end();
  st.bytes_sent = sent0;  // bytes_* count the record exchange only
  st.bytes_recv = recv0;
  if (rc) return rc;
  if ((e = hipStreamSynchronize(stream)) != hipSuccess) return hip_fail(e, "hand-off");
  n_out = new_n;
  st.n_out = new_n;
  return MHMKC_OK;
}

// ------------------------------------------------------------------------------------------------
// fine partition + LDS count + finalize

// Fine buckets are capped at 1.25x their expected size (+256): a single scatter pass, no histogram. If a
// bucket overflows, the count kernel returns at once and the pass is redone with part_hist + scan.
//
// Finish passes (memory): the owned coarse range is counted in P contiguous parts, each fine-partitioned into the
// same buffer, counted, and its survivors appended to the output. One pass holds 1/P of the fine records (and, with
// the supermer exchange, of the received windows' records, extracted per pass from the received supermers), so a
// shard larger than free device memory (or several ranks sharing one GPU) still counts. P: MHMKC_PASSES, else the
// smallest power of two whose pass fits 80 % of the free device memory. The output is sized from the distinct-key
// sketch (half the estimated distinct keys + 1M rows: the survivors, count >= 2, are a fraction of them); a pass
// that fills it stops writing, and is redone after the output has grown to the rows its cursor counted.
int mhmkc::finish_passes(uint64_t owned) const {
  const uint32_t no = n_owned();
  if (const char *env = getenv("MHMKC_PASSES")) return std::max(1, std::min<int>(atoi(env), (int)std::max(1u, no)));
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) return 1;
  double need = (double)owned * (double)(compact ? 4 : rec_bytes()) * 1.3;  // capped fine records
  if (smer) need += (double)owned * (double)rec_bytes() * 1.1;              // the received windows' coarse records
  // what every pass shares: k_count's spill area, the fine tables of the largest pass (at most 2^11 fine buckets per
  // coarse bucket, base + cursor + histogram), the output (sized later from the sketch; survivors are a fraction of
  // the records: 1/24 at C2, 1/16 at C4, budgeted at 1/8)
  const double fixed = (nl <= mhm::DYN_SWEEP_MAX_NL
                            ? (double)n_cu * mhm::C_SPLIT * mhm::SPILL_RECORDS * (compact ? 4 : rec_bytes())
                            : 0.0) +
                       (double)no * 2048.0 * 24.0 + (double)owned / 8.0 * (8.0 * nlo + 4.0);
  const double have = 0.8 * (double)fr + (double)d_r2.cap + (smer_slab ? (double)smer_slab->buf.cap : 0.0) +
                      (double)d_spill.cap + (double)d_out_keys.cap - fixed;
  int P = 1;
  while (P < (int)no && need / P > have) P *= 2;
  return std::min<int>(P, (int)std::max(1u, no));
}

// A device buffer grown to `need` bytes with its first `used` bytes kept (the output of earlier passes).
hipError_t mhmkc::grow_keep(DevBuf &b, size_t used, size_t need) {
  if (need <= b.cap && b.p) return hipSuccess;
  hipError_t e = hipStreamSynchronize(stream);
  if (e != hipSuccess) return e;
  DevBuf nb_;
  if ((e = nb_.ensure(need)) != hipSuccess) return e;
  if (used && b.p && (e = hipMemcpy(nb_.p, b.p, std::min(used, b.cap), hipMemcpyDeviceToDevice)) != hipSuccess) {
    nb_.release();
    return e;
  }
  b.release();
  b = nb_;
  return hipSuccess;
}

void mhmkc::make_runs(const std::vector<Source> &srcs, uint32_t c0, uint32_t c1, int T, RunTable &rt) const {
  rt.runs.clear();
  rt.ps.clear();
  rt.n_chunks = rt.n_c0 = rt.xcd_max = rt.rec_c0 = rt.rec_c0_even = 0;
  for (auto &sr : srcs) rt.ps.push_back(sr.planes);
  for (uint32_t x = 0; x < 8; x++) {
    rt.xcd_start[x] = rt.n_chunks;
    for (uint32_t c = c0 + ((x + 8 - c0 % 8) % 8); c < c1; c += 8) {
      for (uint32_t q = 0; q < NSUB; q++)
        for (size_t s_ = 0; s_ < srcs.size(); s_++) {
          const uint32_t i = c * NSUB + q;
          const uint64_t cnt = srcs[s_].count[i];
          if (!cnt) continue;
          rt.runs.push_back({srcs[s_].start[i], cnt, (uint32_t)s_, c - c0, (uint32_t)rt.n_chunks, 0});
          if (c == c0) {  // (the sketch launches one workgroup per chunk: its even chunks are the half sample)
            rt.rec_c0 += cnt;
            for (uint64_t j = 0; j < cnt; j += (uint64_t)T)
              if (!((rt.n_chunks + j / T) & 1)) rt.rec_c0_even += std::min<uint64_t>((uint64_t)T, cnt - j);
          }
          rt.n_chunks += (cnt + T - 1) / T;
        }
      if (c == c0) rt.n_c0 = rt.n_chunks;
    }
  }
  rt.xcd_start[8] = rt.n_chunks;
  for (int x = 0; x < 8; x++) rt.xcd_max = std::max(rt.xcd_max, rt.xcd_start[x + 1] - rt.xcd_start[x]);
}

// The run table on the device (buf: runs | chunk index, expanded on s; sbuf: the plane sets), and the partition
// parameters that point at it. The host vectors of rt must live until the copies on s ran.
int mhmkc::upload_runs(const RunTable &rt, DevBuf &buf, DevBuf &sbuf, hipStream_t s, mhm::PartitionParams &pp,
                       PinBuf *pin) {
  const int T = mhm::chunk_records(nl);
  if (rt.n_chunks >= 0x7fffffffull) return fail(MHMKC_EINVAL, "too many chunks");
  hipError_t e;
  const size_t rb = align_up(std::max<size_t>(1, rt.runs.size()) * sizeof(mhm::SRun), 256);
  const bool main = s == stream;  // (main stream: earlier kernels may still read the buffers, grow waits for them)
  const size_t cb_ = sizeof(mhm::SChunk) * (rt.n_chunks + 1) + 256;
  if ((e = main ? grow(buf, rb + cb_) : buf.ensure(rb + cb_)) != hipSuccess)
    return hip_fail(e, "chunk table");
  const size_t sb = std::max<size_t>(1, rt.ps.size()) * sizeof(mhm::PlaneSet) + 64;
  if ((e = main ? grow(sbuf, sb) : sbuf.ensure(sb)) != hipSuccess) return hip_fail(e, "source table");
  mhm::SRun *d_runs = buf.as<mhm::SRun>();
  mhm::SChunk *d_chunk_run = (mhm::SChunk *)(buf.as<char>() + rb);
  const void *h_runs = rt.runs.data(), *h_ps = rt.ps.data();
  if (pin) {  // (the caller keeps *pin until the copies have run)
    const size_t rbytes = rt.runs.size() * sizeof(mhm::SRun), pbytes = rt.ps.size() * sizeof(mhm::PlaneSet);
    if ((e = pin->ensure(rb + pbytes + 64)) != hipSuccess) return hip_fail(e, "run table staging");
    memcpy(pin->as<char>(), rt.runs.data(), rbytes);
    memcpy(pin->as<char>() + rb, rt.ps.data(), pbytes);
    h_runs = pin->as<char>();
    h_ps = pin->as<char>() + rb;
  }
  if (!rt.runs.empty()) {
    if ((e = hipMemcpyAsync(d_runs, h_runs, rt.runs.size() * sizeof(mhm::SRun), hipMemcpyHostToDevice, s)) !=
        hipSuccess)
      return hip_fail(e, "run table H2D");
    if ((e = mhm::launch_chunk_runs(d_runs, (uint32_t)rt.runs.size(), d_chunk_run, T, s)) != hipSuccess)
      return hip_fail(e, "chunk index");
  }
  if (!rt.ps.empty() &&
      (e = hipMemcpyAsync(sbuf.p, h_ps, rt.ps.size() * sizeof(mhm::PlaneSet), hipMemcpyHostToDevice, s)) != hipSuccess)
    return hip_fail(e, "source H2D");
  pp.runs = d_runs;
  pp.chunks = d_chunk_run;
  pp.n_runs = (uint32_t)rt.runs.size();
  pp.n_chunks = (uint32_t)rt.n_chunks;
  for (int x = 0; x < 9; x++) pp.xcd_start[x] = (uint32_t)rt.xcd_start[x];
  pp.grid = (uint32_t)(8 * rt.xcd_max);
  pp.srcs = sbuf.as<mhm::PlaneSet>();
  pp.k = k;
  pp.coarse_bits = cb;
  pp.fine_bits = fb;
  pp.hbits = hbits;
  pp.compact = mixed();
  pp.err = d_err.as<unsigned int>();
  return MHMKC_OK;
}

// The capped fine layout of coarse buckets with these (expected) record counts: every fine bucket of coarse bucket c
// gets (1 + slack) x its share + 256 records (multiples of 16: k_count loads compact records in quads).
int mhmkc::fine_layout(const std::vector<uint64_t> &per_coarse, double slack, std::vector<uint64_t> &cfit,
                       uint64_t &r2_size) const {
  const size_t np_ = per_coarse.size();
  cfit.assign(2 * np_, 0);  // [coarse_base | coarse_fcap]
  r2_size = 0;
  for (size_t c = 0; c < np_; c++) {
    const uint64_t ex = per_coarse[c] >> fb;
    const uint64_t fcap = align_up(ex + (uint64_t)((double)ex * slack) + 256, 16);
    cfit[c] = r2_size;
    cfit[np_ + c] = fcap;
    r2_size += fcap << fb;
  }
  return MHMKC_OK;
}

// The sources of exchange round r: this rank's slab of the round (its owned range in place) and the received spans.
void mhmkc::round_sources(size_t r, std::vector<Source> &srcs) const {
  srcs.clear();
  if (r < x_round_slab.size() && x_round_slab[r] >= 0) {
    const Slab *sl = slabs[(size_t)x_round_slab[r]];
    Source src;
    src.planes = sl->planes;
    src.start.assign(sl->bases.begin() + own_lo * NSUB, sl->bases.begin() + own_hi * NSUB);
    src.count.assign(sl->counts.begin() + own_lo * NSUB, sl->counts.begin() + own_hi * NSUB);
    srcs.push_back(std::move(src));
  }
  if (r < n_parts)
    for (auto &sp : parts[r]->spans) {
      Source src;
      src.planes = parts[r]->planes;
      src.start = sp.start;
      src.count = sp.count;
      srcs.push_back(std::move(src));
    }
}

// Local rounds (one rank, host batches): every slab but the two newest (whose extractions may still
// run; `all`: every slab) becomes a round of the incremental partition once its extraction is done, with the windows the
// add calls announced as the expected total. The layout is set once the rounds hold 40 % of those windows (the
// exchange's is set after two rounds, §3.5f), from a sketch of all of them, and then each round is fine-partitioned on
// pstream while the later chunks are on the wire: finish is then k_count alone.
int mhmkc::local_rounds(bool all) {
  int rc;
  // (between chunks at most two rounds are partitioned per call, so that the backlog of the round that sets the layout
  // is spread over the next chunks instead of holding one chunk's packing back)
  int budget = all ? 1 << 30 : 2;
  while (lq < n_slabs && (all || n_slabs >= lq + 3)) {
    Slab *sl = slabs[lq];
    for (int pass = 0; sl->pending; pass++) {
      bool redo = false;
      if ((rc = resolve_one(sl, redo))) return rc;
      if (redo && pass) return fail(MHMKC_EHIP, "internal: exact extraction overflowed");
    }
    if (!inc_tried) {  // the sampled rounds' shares of the coarse buckets (all owned: one rank)
      if (x_rounds == 0) {
        x_r0_coarse.assign(n_owned(), 0);
        x_r0_total = 0;
      }
      for (uint32_t i = 0; i < nb * NSUB; i++) {
        x_r0_coarse[i / NSUB] += sl->counts[i];
        x_r0_total += sl->counts[i];
      }
    }
    x_expect_all = inc_expect;
    x_round_slab.push_back((int)lq);
    x_rounds++;
    lq++;
    // the layout once the rounds hold 40 % of the announced windows: a genome k-mer has then been seen about 10 times
    // at C2's coverage and the sketch's two-point extrapolation sees the errors' slope (at 1/48 of the reads, two
    // rounds, it took the still rising genome part for errors, 3-5x too many distinct keys), or at finish
    if (!inc_tried && x_rounds >= 2 && (double)x_r0_total >= 0.4 * (double)x_expect_all && (rc = inc_setup()))
      return rc;
    if (inc)
      for (; inc_parted < x_rounds && budget > 0; inc_parted++, budget--)
        if ((rc = inc_round(inc_parted))) return rc;
  }
  if (inc)  // (what the budget left, and at finish all of it)
    for (; inc_parted < x_rounds && budget > 0; inc_parted++, budget--)
      if ((rc = inc_round(inc_parted))) return rc;
  if (all && !inc_tried && x_rounds >= 2) {
    if ((rc = inc_setup())) return rc;
    if (inc)
      for (; inc_parted < x_rounds; inc_parted++)
        if ((rc = inc_round(inc_parted))) return rc;
  }
  return MHMKC_OK;
}

// The incremental partition's layout, after round 0 has landed. The fine bits need the distinct keys
// per coarse bucket, which round 0 samples: a HyperLogLog sketch of its records of the first owned coarse bucket, and a
// second one of about half of them (the even chunks), give the distinct keys D at two sample sizes n; with
// D(n) = G + e n (the genome's k-mers are all seen after a few x of coverage, sequencing errors add new keys in
// proportion to the reads) they extrapolate to the bucket's expected records N. The expected records per coarse bucket
// are the windows every rank announced (its add calls' batches) times the bucket's share of round 0. A later add call
// beyond the announcement, or a skewed input, overflows a capped fine bucket: finish then redoes the partition from the
// sources, which every round keeps.
int mhmkc::inc_setup() {
  inc_tried = true;
  const uint32_t no = n_owned();
  if (!pstream || x_expect_all == 0 || x_r0_total == 0 || (n_parts < 1 && !lrounds) || g_dbg.exact || no == 0)
    return MHMKC_OK;
  hipError_t e;
  std::vector<Source> srcs;
  round_sources(0, srcs);
  if (lrounds)  // local rounds: the sample is every round so far (set up at 40 % of the windows, local_rounds())
    for (size_t r = 1; r < x_rounds; r++) {
      std::vector<Source> more;
      round_sources(r, more);
      for (auto &src : more) srcs.push_back(std::move(src));
    }
  const int T = mhm::chunk_records(nl);
  IncRound sk;
  make_runs(srcs, 0, 1, T, sk.rt);  // the first owned coarse bucket of round 0
  if (!sk.rt.n_c0 || sk.rt.rec_c0 < 4096) return MHMKC_OK;
  mhm::PartitionParams sp{};
  if ((e = hipStreamWaitEvent(pstream, round_event(0), 0)) != hipSuccess) return hip_fail(e, "partition stream");
  int rc = upload_runs(sk.rt, sk.chunks, sk.srcs, pstream, sp);
  if (rc) return rc;
  // (the records per fine digit too, at SKETCH_FB bits, when the stored key bits below the coarse digit have them)
  const bool fh_ok = !(compact && 2 * k - cb < mhm::SKETCH_FB) && !(mixed2 && k - cb < mhm::SKETCH_FB);
  const size_t words = mhm::SKETCH_WORDS + (size_t)mhm::SKETCH_FH;
  std::vector<uint32_t> reg(words);
  if (fh_ok) sp.fine_bits = mhm::SKETCH_FB;
  prof_begin(MHMKC_STAGE_OTHER, pstream);
  if ((e = d_hll.ensure(4 * words + 64)) != hipSuccess || (e = hipMemsetAsync(d_hll.p, 0, 4 * words, pstream)) != hipSuccess ||
      (e = mhm::launch_sketch(sp, (uint32_t)sk.rt.n_c0, d_hll.as<unsigned int>(), nl, packed, pstream, fh_ok)) != hipSuccess)
    return hip_fail(e, "distinct sketch");
  prof_end(pstream);
  if ((e = hipMemcpyAsync(reg.data(), d_hll.p, 4 * words, hipMemcpyDeviceToHost, pstream)) != hipSuccess ||
      (e = hipStreamSynchronize(pstream)) != hipSuccess)
    return hip_fail(e, "sketch D2H");
  sk.chunks.release();
  sk.srcs.release();
  const double d_f = hll_estimate(std::vector<uint32_t>(reg.begin(), reg.begin() + mhm::SKETCH_M));
  const double d_h = hll_estimate(std::vector<uint32_t>(reg.begin() + mhm::SKETCH_M + 1, reg.begin() + mhm::SKETCH_WORDS));
  const double n_f = (double)sk.rt.rec_c0, n_h = (double)sk.rt.rec_c0_even;
  inc_ext_per_rec = (double)reg[mhm::SKETCH_M] / n_f;
  // the expected records of every owned coarse bucket (at least what round 0 brought)
  std::vector<uint64_t> per_coarse(no);
  for (uint32_t c = 0; c < no; c++)
    per_coarse[c] = std::max<uint64_t>(x_r0_coarse[c], (uint64_t)((double)x_expect_all * (double)x_r0_coarse[c] / (double)x_r0_total));
  const double n_exp = (double)per_coarse[0];
  const double slope = (n_f > n_h && d_f > d_h) ? (d_f - d_h) / (n_f - n_h) : 0.0;
  const double d_n = std::min(std::max(d_f + slope * (n_exp - n_f), d_f), d_f * n_exp / n_f);
  const uint32_t cap_slots = (uint32_t)mhm::count_cap(nl, compact);
  int f = 4;
  while (f < 11 && d_n / (double)(1u << f) > FINE_LOAD * cap_slots) f++;
  if (g_dbg.fine_bits >= 0) f = (int)std::min<int64_t>(11, g_dbg.fine_bits);
  fb = std::max(f, min_fine_bits());
  nf = 1u << fb;
  // The slack of the capped fine buckets: a key's copies all land in one fine bucket, so at high coverage the buckets'
  // loads spread wider than the record count alone says (small buckets most: a test's 1000-record buckets of 24
  // genome k-mers x 40 copies). The sampled coarse bucket's loads per fine bucket (without its fullest, where a very
  // frequent k-mer would sit) give their coefficient of variation; 5 of it, at least 1/4, at most 2.
  double slack = 0.25;
  if (fh_ok) {
    const uint32_t G = 1u << fb, per = 1u << (mhm::SKETCH_FB - fb);
    std::vector<double> ld(G, 0.0);
    for (uint32_t i = 0; i < (uint32_t)mhm::SKETCH_FH; i++) ld[i / per] += reg[mhm::SKETCH_WORDS + i];
    std::sort(ld.begin(), ld.end());
    ld.pop_back();
    double m = 0, v = 0;
    for (double x : ld) m += x;
    m /= (double)ld.size();
    for (double x : ld) v += (x - m) * (x - m);
    v /= (double)ld.size();
    if (m > 0) slack = std::min(2.0, std::max(0.25, 5.0 * std::sqrt(v) / m));
  }
  inc_slack = slack;
  uint64_t r2_size = 0;
  fine_layout(per_coarse, slack, inc_cfit, r2_size);
  // room for it (the finish then needs no more than the output and k_count's spill area)
  size_t fr = 0, tot = 0;
  const double rec_b = compact ? 4.0 : (double)rec_bytes();
  if (hipMemGetInfo(&fr, &tot) != hipSuccess ||
      (double)r2_size * rec_b > 0.7 * (double)fr + (double)d_r2.cap)
    return MHMKC_OK;
  const uint32_t n_fine = no << fb;
  if ((rc = set_planes(d_r2, r2_size, inc_r2, true, false))) return rc;
  if ((e = d_fine_base.ensure((size_t)n_fine * 8)) != hipSuccess ||
      (e = d_fine_cursor.ensure((size_t)n_fine * 8)) != hipSuccess || (e = d_cfit.ensure(16 * (size_t)no + 64)) != hipSuccess)
    return hip_fail(e, "fine layout");
  unsigned long long *cf = d_cfit.as<unsigned long long>();
  if ((e = hipMemcpyAsync(cf, inc_cfit.data(), 16 * (size_t)no, hipMemcpyHostToDevice, pstream)) != hipSuccess ||
      (e = mhm::launch_init_fine(cf, cf + no, no, fb, d_fine_base.as<unsigned long long>(),
                                 d_fine_cursor.as<unsigned long long>(), pstream)) != hipSuccess)
    return hip_fail(e, "fine layout");
  inc_distinct = d_n * no;
  inc = true;
  return MHMKC_OK;
}

// Round r's records into the incremental layout, on pstream once the round's transfer has landed.
int mhmkc::inc_round(size_t r) {
  const uint32_t no = n_owned();
  while (inc_pool.size() <= r) inc_pool.push_back(new IncRound());
  IncRound *ir = inc_pool[r];
  std::vector<Source> srcs;
  round_sources(r, srcs);
  make_runs(srcs, 0, no, mhm::chunk_records(nl), ir->rt);
  if (!ir->rt.n_chunks) return MHMKC_OK;
  hipError_t e;
  if ((e = hipStreamWaitEvent(pstream, round_event(r), 0)) != hipSuccess) return hip_fail(e, "partition stream");
  mhm::PartitionParams pp{};
  int rc = upload_runs(ir->rt, ir->chunks, ir->srcs, pstream, pp, &ir->pin);
  if (rc) return rc;
  unsigned long long *cf = d_cfit.as<unsigned long long>();
  pp.fine_hist = nullptr;
  pp.fine_cursor = d_fine_cursor.as<unsigned long long>();
  pp.coarse_base = cf;
  pp.coarse_fcap = cf + no;
  pp.out = inc_r2;
  prof_begin(MHMKC_STAGE_SSCAT, pstream);
  e = mhm::launch_part_scatter(pp, nl, packed, pstream);
  prof_end(pstream);
  if (e != hipSuccess) return hip_fail(e, "part_scatter");
  st.inc_rounds++;
  return MHMKC_OK;
}

int mhmkc::finish(uint64_t *n_out_ret) {
  if (partial) return fail(MHMKC_ESTATE, "a failed mhmkc_add_fastq_file left part of the file in this round; call mhmkc_reset");
  int rc = begin_round();
  if (rc) return rc;
  ord_ready = false;
  ctg_gathered = false;
  if ((rc = resolve_slabs())) return rc;
  hipError_t e;
  const uint32_t no = n_owned();
  std::vector<Source> srcs;
  if (smer) {
    if ((rc = smer_exchange(srcs))) return rc;
  } else if (G() > 1 && xpipe) {
    (void)hipEventRecord(ev_xext, stream);  // every extraction is enqueued: the exchange's exposed time starts here
    for (; xq < n_slabs; xq++)
      if ((rc = xround(slabs[xq], xq + 1 == n_slabs))) return rc;
    while (!x_all_done)
      if ((rc = xround(nullptr, true))) return rc;
    (void)hipEventRecord(ev_xdone, xstream);
    if ((e = hipStreamWaitEvent(stream, ev_xdone, 0)) != hipSuccess || (e = hipEventSynchronize(ev_xdone)) != hipSuccess)
      return hip_fail(e, "exchange");
    x_ms = 0;
    for (uint64_t r = 0; r < x_rounds; r++) {
      float ms = 0;
      if (hipEventElapsedTime(&ms, x_ev[2 * r], x_ev[2 * r + 1]) == hipSuccess) x_ms += ms;
    }
    float exposed = 0;
    if (hipEventElapsedTime(&exposed, ev_xext, ev_xdone) != hipSuccess || exposed < 0) exposed = 0;
    st.xchg_rounds = x_rounds;
    st.ms_xchg = x_ms;
    st.ms_xchg_exposed = exposed;
    if (inc) {  // every round's partition is enqueued on pstream (xround): the count waits for them
      for (; inc_parted < x_rounds; inc_parted++)
        if ((rc = inc_round(inc_parted))) return rc;
      if ((e = hipEventRecord(ev_pdone, pstream)) != hipSuccess || (e = hipStreamWaitEvent(stream, ev_pdone, 0)) != hipSuccess)
        return hip_fail(e, "partition stream");
    }
    if (profiling) {
      st.ms_kernel[MHMKC_STAGE_XCHG] += x_ms;
      st.launches[MHMKC_STAGE_XCHG] += x_rounds;
    }
    for (size_t s = 0; s < n_slabs; s++) {  // local slabs: the owned range in place
      Source src;
      src.planes = slabs[s]->planes;
      src.start.assign(slabs[s]->bases.begin() + own_lo * NSUB, slabs[s]->bases.begin() + own_hi * NSUB);
      src.count.assign(slabs[s]->counts.begin() + own_lo * NSUB, slabs[s]->counts.begin() + own_hi * NSUB);
      srcs.push_back(std::move(src));
    }
    for (size_t q = 0; q < n_parts; q++)
      for (auto &sp : parts[q]->spans) {
        Source src;
        src.planes = parts[q]->planes;
        src.start = sp.start;
        src.count = sp.count;
        srcs.push_back(std::move(src));
      }
  } else if (G() > 1) {
    if ((rc = exchange(srcs))) return rc;
  } else {
    if (lrounds && lq > 0) {  // local rounds began in an add call: the remaining slabs are rounds too
      if ((rc = local_rounds(true))) return rc;
      if (inc && ((e = hipEventRecord(ev_pdone, pstream)) != hipSuccess || (e = hipStreamWaitEvent(stream, ev_pdone, 0)) != hipSuccess))
        return hip_fail(e, "partition stream");
    }
    for (size_t s = 0; s < n_slabs; s++) {
      Source src;
      src.planes = slabs[s]->planes;
      src.start.assign(slabs[s]->bases.begin(), slabs[s]->bases.begin() + (size_t)nb * NSUB);
      src.count = slabs[s]->counts;
      srcs.push_back(std::move(src));
    }
  }
  (void)hipEventRecord(ev_tail0, stream);  // (the exchange is over: what follows on the stream is the count)
  uint64_t owned = smer ? smer_nwin : 0;  // (the received windows' records are extracted per pass)
  for (auto &s : srcs)
    for (uint32_t i = 0; i < no * NSUB; i++) owned += s.count[i];
  st.owned_records = owned;
  st.coarse_record_bytes = rec_bytes();
  st.fine_record_bytes = compact ? 4 : rec_bytes();
  smer_seen = 0;

  const int T = mhm::chunk_records(nl);  // records per partition chunk
  const uint32_t cap_slots = (uint32_t)mhm::count_cap(nl, compact);
  const bool exact_dbg = g_dbg.exact != 0;
  uint64_t out_cap = 0, out_used = 0;  // output rows allocated / written by the earlier passes
  unsigned long long acc_stats[mhm::STAT_ALLOC] = {0};
  double est_fine = 0;  // estimated distinct keys per fine bucket (0: no estimate)
  unsigned int errf = 0;
  st.fine_buckets = 0;
  // k_count's parameters for the fine buckets of a pass that starts at local coarse bucket c0 (all but the records
  // and the output, which the attempts set)
  int rc_cp = MHMKC_OK;
  auto count_params = [&](uint32_t c0, uint32_t n_fine) {
    mhm::CountParams cp{};
    cp.bucket_base = d_fine_base.as<unsigned long long>();
    cp.bucket_end = d_fine_cursor.as<unsigned long long>();
    cp.hbits = hbits;
    cp.compact = mixed();
    cp.coarse_bits = cb;
    cp.fine_bits = fb;
    cp.bucket0 = (own_lo + c0) << fb;
    cp.n_buckets = n_fine;
    cp.grid = (uint32_t)std::max(0, n_cu * mhm::C_SPLIT);  // persistent workgroups filling every CU's LDS
    cp.k = k;
    cp.cap = mhm::count_cap(nl, compact);
    // (The fine bucket count is a power of two, so its distinct keys fill between FINE_LOAD / 2 and FINE_LOAD of the
    // LDS table, 0.44 at C2; a table cut to 0.6-0.8 of the estimate was measured slower, 6.28 -> 7.14-10.2 ms: the
    // home-group hit rate falls faster than the per-slot clear and finalize work.)
    st.table_slots = (uint64_t)cp.cap;
    if (g_dbg.cap) cp.cap = std::min<int>(cp.cap, (int)std::max<int64_t>(64, g_dbg.cap) & ~3);
    cp.dmin_thres = dmin;
    cp.dyn_mult = 1.0 - cfg.dyn_min_depth;
    cp.nlo = nlo;
    cp.out_cursor = d_out_cursor.as<unsigned long long>();
    cp.stats = d_stats.as<unsigned long long>();
    cp.err = d_err.as<unsigned int>();
    cp.ctg_n = ctg_n;
    for (int w = 0; w < 4; w++) cp.ctg_keys[w] = w < nl ? d_ctg_keys[w].as<uint64_t>() : nullptr;
    cp.ctg_state = d_ctg_state.as<uint32_t>();
    cp.ctg_bucket = d_ctg_bucket.as<uint32_t>();
    cp.ctg_done = d_ctg_done.as<uint8_t>();
    cp.ctg_base = c0 << fb;
    if (cp.grid && nl <= mhm::DYN_SWEEP_MAX_NL)  // dynamic cold sweeps defer into it (one- and two-word keys)
      rc_cp = set_planes(d_spill, (uint64_t)cp.grid * mhm::SPILL_RECORDS, cp.spill, true);
    if (rc_cp) cp.grid = 0;
    return cp;
  };
  auto grow_output = [&](uint64_t rows) -> int {
    hipError_t e_;
    if ((e_ = grow(d_out_keys, rows * 8 * nlo)) != hipSuccess || (e_ = grow(d_out_counts, rows * 2)) != hipSuccess ||
        (e_ = grow(d_out_left, rows)) != hipSuccess || (e_ = grow(d_out_right, rows)) != hipSuccess ||
        (e_ = grow(d_out_cursor, 8)) != hipSuccess)
      return hip_fail(e_, "output");
    return MHMKC_OK;
  };

  // The incremental partition put every round's records into their fine buckets already: count them.
  // A coarse bucket with a fine bucket past its capped segment (skewed input: a very frequent k-mer) is emptied by
  // k_inc_fixup and skipped by k_count; the passes below then count just those coarse buckets again, from the sources,
  // with exact bucket sizes. A full output grows and counts again (the layout stays). Anything else unexpected sends
  // the whole finish through the passes.
  bool inc_done = false;
  std::vector<std::pair<uint32_t, uint32_t>> ranges;  // the local coarse ranges the passes below count
  if (inc) {
    const uint32_t n_fine = no << fb;
    nf = 1u << fb;
    st.distinct_estimate = (uint64_t)inc_distinct;
    st.inc_slack = inc_slack;
    st.lds_ext_adds = (uint64_t)(inc_ext_per_rec * (double)owned);
    if ((rc = prepare_ctgs())) return rc;
    out_cap = std::min<uint64_t>(owned / 2, (uint64_t)(0.5 * inc_distinct) + (1u << 20));
    if (g_dbg.out_cap >= 0) out_cap = (uint64_t)g_dbg.out_cap;
    out_cap += ctg_n + 1;
    if ((rc = grow_output(out_cap))) return rc;
    mhm::CountParams cp = count_params(0, n_fine);
    if (rc_cp) return rc_cp;
    if ((e = d_inc_skip.ensure((size_t)no + 64)) != hipSuccess) return hip_fail(e, "skip flags");
    unsigned long long *cf = d_cfit.as<unsigned long long>();
    prof_begin(MHMKC_STAGE_OTHER);
    e = mhm::launch_inc_fixup(cf, cf + no, no, fb, d_fine_cursor.as<unsigned long long>(), d_inc_skip.as<uint8_t>(),
                              d_err.as<unsigned int>(), stream);
    prof_end();
    if (e != hipSuccess) return hip_fail(e, "layout fixup");
    cp.recs = inc_r2;
    cp.coarse_skip = d_inc_skip.as<uint8_t>();
    std::vector<uint8_t> skip(no);
    for (int attempt = 0; attempt < 4 && !inc_done; attempt++) {
      cp.out_keys = d_out_keys.as<uint64_t>();
      cp.out_counts = d_out_counts.as<uint16_t>();
      cp.out_left = d_out_left.as<char>();
      cp.out_right = d_out_right.as<char>();
      cp.out_cap = out_cap;
      unsigned long long stats[mhm::STAT_ALLOC], cursor_end = 0;
      const unsigned long long cur0 = 0;
      prof_begin(MHMKC_STAGE_OTHER);
      e = hipMemcpyAsync(d_out_cursor.p, &cur0, 8, hipMemcpyHostToDevice, stream);
      if (e == hipSuccess) e = hipMemsetAsync(d_stats.p, 0, 8 * mhm::STAT_ALLOC, stream);
      if (e == hipSuccess && ctg_n) e = hipMemsetAsync(d_ctg_done.p, 0, ctg_n, stream);
      prof_end();
      if (e != hipSuccess) return hip_fail(e, "count setup");
      prof_begin(MHMKC_STAGE_COUNT);
      e = mhm::launch_count(cp, nl, packed, stream);
      prof_end();
      if (e != hipSuccess) return hip_fail(e, "count");
      (void)hipEventRecord(ev_end, stream);
      if ((e = hipMemcpyAsync(stats, d_stats.p, sizeof stats, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
          (e = hipMemcpyAsync(&errf, d_err.p, 4, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
          (e = hipMemcpyAsync(&cursor_end, d_out_cursor.p, 8, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
          (e = hipMemcpyAsync(skip.data(), d_inc_skip.p, no, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
          (e = hipStreamSynchronize(stream)) != hipSuccess)
        return hip_fail(e, "finish");
      if (errf & 2u) break;  // (not expected: k_inc_fixup cleared it)
      if (errf & 16u) {  // the output is full: grow it to the rows the cursor counted, count again
        out_cap = cursor_end + cursor_end / 16 + 1024;
        if ((rc = grow_output(out_cap))) return rc;
        st.out_reruns++;
        errf &= ~16u;
        if ((e = hipMemcpy(d_err.p, &errf, 4, hipMemcpyHostToDevice)) != hipSuccess) return hip_fail(e, "flag reset");
        continue;
      }
      if (stats[mhm::STAT_N - 1]) return fail(MHMKC_EHIP, "internal: LDS probe bound exceeded");
      for (int i = 0; i < mhm::STAT_ALLOC; i++) acc_stats[i] = stats[i];
      out_used = cursor_end;
      st.fine_buckets = n_fine;
      inc_done = true;
    }
    if (inc_done) {
      for (uint32_t c = 0; c < no; c++) {
        if (!skip[c]) continue;
        st.inc_redone_coarse++;
        if (!ranges.empty() && ranges.back().second == c)
          ranges.back().second = c + 1;
        else
          ranges.push_back({c, c + 1});
      }
    } else {
      st.inc_fallbacks++;
      errf &= ~(2u | 16u);
      if ((e = hipMemcpy(d_err.p, &errf, 4, hipMemcpyHostToDevice)) != hipSuccess) return hip_fail(e, "flag reset");
    }
  }
  if (!inc_done) {
    const int passes = finish_passes(owned);
    for (int q = 0; q < passes; q++)
      ranges.push_back({(uint32_t)((uint64_t)no * q / passes), (uint32_t)((uint64_t)no * (q + 1) / passes)});
  }
  st.finish_passes = (inc_done ? 1 : 0) + (uint64_t)ranges.size();
  for (size_t pass = 0; pass < ranges.size(); pass++) {
    const uint32_t c0 = ranges[pass].first, c1 = ranges[pass].second;
    const uint32_t np_ = c1 - c0;  // coarse buckets of this pass
    if (!np_) continue;
    const size_t n_srcs0 = srcs.size();
    if (smer && (rc = smer_records(own_lo + c0, own_lo + c1, srcs))) return rc;
    std::vector<uint64_t> per_coarse(np_, 0);
    uint64_t owned_p = 0;
    for (auto &s : srcs)
      for (uint32_t i = c0 * NSUB; i < c1 * NSUB; i++) {
        per_coarse[i / NSUB - c0] += s.count[i];
        owned_p += s.count[i];
      }
    for (uint32_t c = 0; c < np_; c++)  // k_count indexes a bucket with 32 bits
      if (per_coarse[c] >= 0xffffffffull)
        return fail(MHMKC_EUNSUPPORTED, "more than 2^32 records in one hash bucket (split the input into batches of ranks)");

    // run table: one entry per non-empty (source, segment) span of the pass's coarse buckets; the device expands it
    // into chunks, ordered by XCD class (coarse % 8), then coarse bucket, segment, source (see xcd_chunk)
    std::vector<mhm::SRun> runs;
    std::vector<mhm::PlaneSet> ps;
    uint64_t n_chunks = 0, n_c0 = 0;  // n_c0: chunks of the pass's first coarse bucket (they come first)
    uint64_t xcd_start[9] = {0};
    for (size_t s = 0; s < srcs.size(); s++) ps.push_back(srcs[s].planes);
    for (uint32_t x = 0; x < 8; x++) {
      xcd_start[x] = n_chunks;
      for (uint32_t c = c0 + ((x + 8 - c0 % 8) % 8); c < c1; c += 8) {
        for (uint32_t q = 0; q < NSUB; q++)
          for (size_t s = 0; s < srcs.size(); s++) {
            const uint32_t i = c * NSUB + q;
            const uint64_t cnt = srcs[s].count[i];
            if (!cnt) continue;
            runs.push_back({srcs[s].start[i], cnt, (uint32_t)s, c - c0, (uint32_t)n_chunks, 0});
            n_chunks += (cnt + T - 1) / T;
          }
        if (c == c0) n_c0 = n_chunks;
      }
    }
    xcd_start[8] = n_chunks;
    if (n_chunks >= 0x7fffffffull) return fail(MHMKC_EINVAL, "too many chunks");
    uint64_t xcd_max = 0;
    for (int x = 0; x < 8; x++) xcd_max = std::max(xcd_max, xcd_start[x + 1] - xcd_start[x]);
    if ((e = grow(d_chunks, align_up(std::max<size_t>(1, runs.size()) * sizeof(mhm::SRun), 256) +
                                sizeof(mhm::SChunk) * (n_chunks + 1) + 256)) !=
        hipSuccess)
      return hip_fail(e, "chunk table");
    mhm::SRun *d_runs = d_chunks.as<mhm::SRun>();
    mhm::SChunk *d_chunk_run = (mhm::SChunk *)(d_chunks.as<char>() + align_up(runs.size() * sizeof(mhm::SRun), 256));
    if ((e = grow(d_srcs, std::max<size_t>(1, ps.size()) * sizeof(mhm::PlaneSet) + 64)) != hipSuccess ||
        (e = grow(d_cfit, 16 * (size_t)np_ + 64)) != hipSuccess)
      return hip_fail(e, "source table");
    unsigned long long *cfit_d = d_cfit.as<unsigned long long>();
    // the tables are small: their copies are waited for below (the host vectors go out of scope)
    if (!runs.empty()) {
      if ((e = hipMemcpyAsync(d_runs, runs.data(), runs.size() * sizeof(mhm::SRun), hipMemcpyHostToDevice, stream)) !=
          hipSuccess)
        return hip_fail(e, "run table H2D");
      if ((e = mhm::launch_chunk_runs(d_runs, (uint32_t)runs.size(), d_chunk_run, T, stream)) != hipSuccess)
        return hip_fail(e, "chunk index");
    }
    if (!ps.empty() && (e = hipMemcpyAsync(d_srcs.p, ps.data(), ps.size() * sizeof(mhm::PlaneSet),
                                           hipMemcpyHostToDevice, stream)) != hipSuccess)
      return hip_fail(e, "source H2D");

    if (pass == 0 && !inc_done) {  // (a redo after the incremental count keeps its fine bits, contigs and output)
      // fine bits: at most FINE_LOAD x the LDS table slots of distinct keys per fine bucket, with
      // the distinct keys of the first owned coarse bucket estimated by a HyperLogLog sketch (the ratio of distinct
      // keys to records grows with k and the error rate, so the record count alone misjudges it); the same fine bits
      // for every pass (the contig pass buckets its k-mers with them once)
      fb = 4;
      double est = 0;
      if (n_c0) {
        mhm::PartitionParams sp{};
        sp.runs = d_runs;
        sp.chunks = d_chunk_run;
        sp.n_runs = (uint32_t)runs.size();
        sp.n_chunks = (uint32_t)n_chunks;
        sp.srcs = d_srcs.as<mhm::PlaneSet>();
        sp.k = k;
        sp.coarse_bits = cb;
        sp.hbits = hbits;
        sp.compact = mixed();
        std::vector<uint32_t> reg(mhm::SKETCH_M + 1);
        prof_begin(MHMKC_STAGE_OTHER);
        if ((e = grow(d_hll, 4 * mhm::SKETCH_WORDS + 64)) != hipSuccess ||
            (e = hipMemsetAsync(d_hll.p, 0, 4 * mhm::SKETCH_WORDS, stream)) != hipSuccess ||
            (e = mhm::launch_sketch(sp, (uint32_t)n_c0, d_hll.as<unsigned int>(), nl, packed, stream)) != hipSuccess)
          return hip_fail(e, "distinct sketch");
        prof_end();
        if ((e = hipMemcpyAsync(reg.data(), d_hll.p, 4 * mhm::SKETCH_M + 4, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
            (e = hipStreamSynchronize(stream)) != hipSuccess)
          return hip_fail(e, "sketch D2H");
        // extension adds of the sampled coarse bucket, scaled to all owned records (the LDS op mix, stats only)
        if (per_coarse[0]) st.lds_ext_adds = (uint64_t)((double)reg[mhm::SKETCH_M] * (double)owned / (double)per_coarse[0]);
        reg.resize(mhm::SKETCH_M);
        est = hll_estimate(reg);
        st.distinct_estimate = (uint64_t)(est * no);
        while (fb < 11 && est / (double)(1u << fb) > FINE_LOAD * cap_slots) fb++;
        est_fine = est;
      } else {  // no records in the first coarse bucket: ~4 records per slot
        const uint64_t avg_coarse = owned / std::max<uint32_t>(no, 1);
        while (fb < 11 && (avg_coarse >> fb) > (uint64_t)cap_slots * 4) fb++;
      }
      if (g_dbg.fine_bits >= 0) fb = (int)std::min<int64_t>(11, g_dbg.fine_bits);
      fb = std::max(fb, min_fine_bits());
      nf = 1u << fb;
      est_fine /= nf;
      if ((rc = prepare_ctgs())) return rc;
      // the output: survivors have count >= 2, so at most owned / 2 read k-mers (+ the contig k-mers); the sketch
      // bounds them by the distinct keys, of which half is a generous guess (C2: 52M survivors of 207M distinct)
      out_cap = owned / 2;
      if (est > 0) out_cap = std::min<uint64_t>(out_cap, (uint64_t)(0.5 * est * no) + (1u << 20));
      if (g_dbg.out_cap >= 0) out_cap = (uint64_t)g_dbg.out_cap;
      out_cap += ctg_n + 1;
      if ((rc = grow_output(out_cap))) return rc;
    }
    const uint32_t n_fine = np_ * nf;
    st.fine_buckets += n_fine;

    // capped fine layout of the pass
    std::vector<uint64_t> cfit(2 * (size_t)np_);  // [coarse_base | coarse_fcap]
    uint64_t r2_size = 0;
    for (uint32_t c = 0; c < np_; c++) {
      const uint64_t ex = per_coarse[c] >> fb;
      const uint64_t fcap = align_up(ex + ex / 4 + 256, 16);
      cfit[c] = r2_size;
      cfit[np_ + c] = fcap;
      r2_size += fcap << fb;
    }
    if ((e = hipMemcpyAsync(cfit_d, cfit.data(), 16 * (size_t)np_, hipMemcpyHostToDevice, stream)) != hipSuccess)
      return hip_fail(e, "layout H2D");
    if ((e = grow(d_fine_hist, (size_t)n_fine * 8)) != hipSuccess) return hip_fail(e, "fine histogram");
    if ((e = grow(d_fine_base, (size_t)n_fine * 8)) != hipSuccess) return hip_fail(e, "fine bases");
    if ((e = grow(d_fine_cursor, (size_t)n_fine * 8)) != hipSuccess) return hip_fail(e, "fine cursor");

    mhm::PartitionParams pp{};
    pp.runs = d_runs;
    pp.chunks = d_chunk_run;
    pp.n_runs = (uint32_t)runs.size();
    pp.n_chunks = (uint32_t)n_chunks;
    for (int x = 0; x < 9; x++) pp.xcd_start[x] = (uint32_t)xcd_start[x];
    pp.grid = (uint32_t)(8 * xcd_max);
    pp.srcs = d_srcs.as<mhm::PlaneSet>();
    pp.k = k;
    pp.coarse_bits = cb;
    pp.fine_bits = fb;
    pp.hbits = hbits;
    pp.compact = mixed();
    pp.fine_hist = d_fine_hist.as<unsigned long long>();
    pp.fine_cursor = d_fine_cursor.as<unsigned long long>();
    pp.err = d_err.as<unsigned int>();

    mhm::CountParams cp = count_params(c0, n_fine);
    if (rc_cp) return rc_cp;
    bool exact = exact_dbg || inc_done;  // (a coarse bucket the incremental count skipped is known to be skewed)
    unsigned long long stats[mhm::STAT_ALLOC], cursor_end = 0;
    for (int attempt = 0;; attempt++) {
      if (attempt >= 4) return fail(MHMKC_EHIP, "internal: finish pass %d did not settle", pass);
      mhm::PlaneSet r2{};
      if (exact) {  // (k_scan rounds every bucket up to a multiple of 4 records)
        if ((rc = set_planes(d_r2, owned_p + 3 * (uint64_t)n_fine + 4, r2, true))) return rc;
      } else {
        if ((rc = set_planes(d_r2, r2_size, r2, true))) return rc;
      }
      cp.out_keys = d_out_keys.as<uint64_t>();
      cp.out_counts = d_out_counts.as<uint16_t>();
      cp.out_left = d_out_left.as<char>();
      cp.out_right = d_out_right.as<char>();
      cp.out_cap = out_cap;
      const unsigned long long cur0 = out_used;
      prof_begin(MHMKC_STAGE_OTHER);
      e = hipMemcpyAsync(d_out_cursor.p, &cur0, 8, hipMemcpyHostToDevice, stream);
      if (e == hipSuccess) e = hipMemsetAsync(d_stats.p, 0, 8 * mhm::STAT_ALLOC, stream);
      if (e == hipSuccess && ctg_n) e = hipMemsetAsync(d_ctg_done.p, 0, ctg_n, stream);  // (earlier passes' are done)
      if (e == hipSuccess && exact) e = hipMemsetAsync(d_fine_hist.p, 0, (size_t)n_fine * 8, stream);
      if (e == hipSuccess && !exact)
        e = mhm::launch_init_fine(cfit_d, cfit_d + np_, np_, fb, d_fine_base.as<unsigned long long>(),
                                  d_fine_cursor.as<unsigned long long>(), stream);
      prof_end();
      if (e != hipSuccess) return hip_fail(e, "fine layout");
      if (exact) {
        pp.coarse_base = nullptr;
        pp.coarse_fcap = nullptr;
        prof_begin(MHMKC_STAGE_SHIST);
        e = mhm::launch_part_hist(pp, nl, packed, stream);
        prof_end();
        if (e != hipSuccess) return hip_fail(e, "part_hist");
        prof_begin(MHMKC_STAGE_OTHER);
        e = mhm::launch_scan(d_fine_hist.as<unsigned long long>(), d_fine_base.as<unsigned long long>(),
                             d_fine_cursor.as<unsigned long long>(), n_fine, stream);
        prof_end();
        if (e != hipSuccess) return hip_fail(e, "scan");
      } else {
        pp.coarse_base = cfit_d;
        pp.coarse_fcap = cfit_d + np_;
      }
      pp.out = r2;
      prof_begin(MHMKC_STAGE_SSCAT);
      e = mhm::launch_part_scatter(pp, nl, packed, stream);
      prof_end();
      if (e != hipSuccess) return hip_fail(e, "part_scatter");
      cp.recs = r2;
      prof_begin(MHMKC_STAGE_COUNT);
      e = mhm::launch_count(cp, nl, packed, stream);
      prof_end();
      if (e != hipSuccess) return hip_fail(e, "count");
      (void)hipEventRecord(ev_end, stream);
      if ((e = hipMemcpyAsync(stats, d_stats.p, sizeof stats, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
          (e = hipMemcpyAsync(&errf, d_err.p, 4, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
          (e = hipMemcpyAsync(&cursor_end, d_out_cursor.p, 8, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
          (e = hipStreamSynchronize(stream)) != hipSuccess)
        return hip_fail(e, "finish");
      if (!(errf & (2u | 16u))) break;
      if (errf & 2u) {  // a capped fine bucket overflowed (skewed input): the pass again with exact bucket sizes
        exact = true;
        st.exact_reruns++;
      } else if (errf & 16u) {  // the output is full: grow it to the rows the cursor counted, keep the earlier passes'
        const uint64_t need = cursor_end + cursor_end / 16 + 1024;
        if ((e = grow_keep(d_out_keys, out_used * 8 * nlo, need * 8 * nlo)) != hipSuccess ||
            (e = grow_keep(d_out_counts, out_used * 2, need * 2)) != hipSuccess ||
            (e = grow_keep(d_out_left, out_used, need)) != hipSuccess ||
            (e = grow_keep(d_out_right, out_used, need)) != hipSuccess)
          return hip_fail(e, "output growth");
        out_cap = need;
        st.out_reruns++;
      }
      errf &= ~(2u | 16u);
      if ((e = hipMemcpy(d_err.p, &errf, 4, hipMemcpyHostToDevice)) != hipSuccess) return hip_fail(e, "flag reset");
    }
    if (stats[mhm::STAT_N - 1]) return fail(MHMKC_EHIP, "internal: LDS probe bound exceeded");
    for (int i = 0; i < mhm::STAT_ALLOC; i++)
      acc_stats[i] = i == mhm::STAT_MAXBUCKET ? std::max(acc_stats[i], stats[i]) : acc_stats[i] + stats[i];
    out_used = cursor_end;
    srcs.resize(n_srcs0);  // (the pass's received-supermer records)
  }
  if (smer && smer_seen != smer_nwin)
    return fail(MHMKC_EHIP, "internal: the finish passes extracted %llu of %llu received windows",
                (unsigned long long)smer_seen, (unsigned long long)smer_nwin);
  float ms = 0;
  if (hipEventElapsedTime(&ms, ev_begin, ev_end) == hipSuccess) st.ms_total = ms;
  if (hipEventElapsedTime(&ms, ev_tail0, ev_end) == hipSuccess) st.ms_finish_tail = ms;
  finished = true;
  if (errf & 1u) return fail(MHMKC_EBADCHAR, "input byte with a base code > 4 (not A,C,G,T,N)");
  if (errf & 8u) return fail(MHMKC_EHIP, "internal: supermer spans inconsistent");
#if MHMKC_STAMP
  {  // k_count phase cycles of an MHMKC_STAMP build (diagnostics)
    const char *names[6] = {"clear", "loadwait", "insert", "barrier", "overflow", "finalize"};
    double tot = 0;
    for (int i = 0; i < 6; i++) tot += (double)acc_stats[8 + i];
    fprintf(stderr, "k_count stamps:");
    for (int i = 0; i < 6; i++) fprintf(stderr, " %s %.1f%%", names[i], tot > 0 ? 100.0 * acc_stats[8 + i] / tot : 0.0);
    fprintf(stderr, " (total %.3g wave-cycles); workgroup cycles mean %.4g max %.4g\n", tot,
            (double)acc_stats[14] / std::max(1, n_cu), (double)acc_stats[15]);
  }
#endif
  st.distinct = acc_stats[mhm::STAT_DISTINCT];
  st.n_out = acc_stats[mhm::STAT_NOUT];
  st.purged = acc_stats[mhm::STAT_PURGED];
  st.count_sum = acc_stats[mhm::STAT_COUNTSUM];
  st.overflow_sweeps = acc_stats[mhm::STAT_SWEEPS];
  st.max_bucket = acc_stats[mhm::STAT_MAXBUCKET];
  st.lds_misses = acc_stats[mhm::STAT_MISSES];
  st.dropped = 0;
  n_out = st.n_out;
  if (n_out != out_used) return fail(MHMKC_EHIP, "internal: output rows %llu, cursor %llu", (unsigned long long)n_out,
                                     (unsigned long long)out_used);
  if (cfg.output_owner == MHMKC_OWNER_MINIMIZER && G() > 1 && !smer) {  // (supermers already went to that owner)
    if ((rc = handoff())) return rc;
  }
  st.device_bytes = g_dev_live.load();
  st.device_bytes_peak = g_dev_peak.load();
  prof_collect();
  if (n_out_ret) *n_out_ret = n_out;
  return MHMKC_OK;
}

hipError_t mhmkc::d2h(void *dst, const void *src, size_t bytes) {
  const size_t CH = g_dbg.d2h_chunk > 0 ? (size_t)g_dbg.d2h_chunk : 8ull << 20;
  hipError_t e;
  hipPointerAttribute_t pa{};
  const bool pinned = hipPointerGetAttributes(&pa, dst) == hipSuccess && pa.type == hipMemoryTypeHost;
  (void)hipGetLastError();  // (pageable memory is "not a HIP pointer": not an error to keep)
  if (bytes < 2 * CH || pinned) {  // pinned caller memory: one DMA straight into it
    if ((e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, stream)) != hipSuccess) return e;
    return hipStreamSynchronize(stream);
  }
  D2HStage &stg = d2h_stage();
  std::lock_guard<std::mutex> lock(stg.mu);
  if ((e = stg.buf[0].ensure(CH)) != hipSuccess || (e = stg.buf[1].ensure(CH)) != hipSuccess) return e;
  hipEvent_t ev[2] = {take_event(), take_event()};
  const size_t n_ch = (bytes + CH - 1) / CH;
  auto drain = [&](size_t c) {  // host copy of chunk c out of its staging buffer, four threads
    const size_t off = c * CH, len = std::min(CH, bytes - off);
    const char *sp = stg.buf[c & 1].as<char>();
    char *dp = (char *)dst + off;
    // piece t is [cut(t), cut(t + 1)): quarters on 64-byte boundaries, the last one ending at len. (The pieces were
    // once q = (len / 4 + 63) & ~63 long, which rounds down when len / 4 is a multiple of 64 and len is not one of 4:
    // the chunk's last 1-3 bytes were never copied. It took the last two rows' left and right bytes of a C4 rank's
    // 65,094,658-row table, the one-row C4 mismatch of rounds 4-5)
    auto cut = [&](int t) { return t >= 4 ? len : std::min(len, (len / 4 * (size_t)t) & ~(size_t)63); };
    std::thread th[3];
    for (int t = 1; t < 4; t++) {
      const size_t a = cut(t), b = cut(t + 1);
      th[t - 1] = std::thread([=] { if (b > a) memcpy(dp + a, sp + a, b - a); });
    }
    memcpy(dp, sp, cut(1));
    for (auto &x : th) x.join();
  };
  e = hipSuccess;
  for (size_t c = 0; c < n_ch && e == hipSuccess; c++) {
    const size_t off = c * CH, len = std::min(CH, bytes - off);
    if (c >= 2 && (e = hipEventSynchronize(ev[c & 1])) != hipSuccess) break;  // (its buffer was drained below)
    if ((e = hipMemcpyAsync(stg.buf[c & 1].p, (const char *)src + off, len, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
        (e = hipEventRecord(ev[c & 1], stream)) != hipSuccess)
      break;
    if (c >= 1) {
      if ((e = hipEventSynchronize(ev[(c - 1) & 1])) != hipSuccess) break;
      drain(c - 1);
    }
  }
  if (e == hipSuccess && (e = hipEventSynchronize(ev[(n_ch - 1) & 1])) == hipSuccess) drain(n_ch - 1);
  ev_pool.push_back(ev[0]);
  ev_pool.push_back(ev[1]);
  return e;
}

// Pinned host blocks handed out by mhmkc_host_alloc, and the freed ones kept for the next caller (pinning a buffer of
// a fetch chunk's size costs more than copying through the staging buffers once; a hand-off per k round reuses them).
namespace {
struct HostPool {
  std::mutex mu;
  std::map<void *, size_t> live;            // block -> bytes
  std::multimap<size_t, void *> free_;      // bytes -> block
  size_t free_bytes = 0;
};
HostPool &host_pool() {
  static HostPool *p = new HostPool();  // (process lifetime)
  return *p;
}
constexpr size_t HOST_POOL_KEEP = 2ull << 30;  // freed blocks kept for reuse, at most this many bytes
}  // namespace

// ------------------------------------------------------------------------------------------------
// C ABI

extern "C" {

int mhmkc_abi_version(void) { return MHMKC_ABI_VERSION; }

// build.py passes -DMHMKC_BUILD_ID="<16 hex digits>" (the sources' SHA-256); the marker string is also what build.py
// looks for in the .so to decide whether it is stale
#ifndef MHMKC_BUILD_ID
#define MHMKC_BUILD_ID "unknown"
#endif
__attribute__((used)) static const char k_build_marker[] = "MHMKC_BUILD_ID=" MHMKC_BUILD_ID;
const char *mhmkc_build_id(void) { return k_build_marker + 15; }

int mhmkc_config_init(mhmkc_config *cfg) {
  if (!cfg) return MHMKC_EINVAL;
  memset(cfg, 0, sizeof *cfg);
  cfg->k = 21;
  cfg->n_longs = 0;
  cfg->qual_offset = 33;
  cfg->qual_cutoff = 20;
  cfg->dmin_thres = 2;
  cfg->dyn_min_depth = 0.9;
  cfg->device = -1;
  cfg->rank = 0;
  cfg->n_ranks = 1;
  cfg->comm_id = nullptr;
  cfg->stream = nullptr;
  cfg->output_owner = MHMKC_OWNER_HASH;
  cfg->minimizer_len = 0;
  return MHMKC_OK;
}

int mhmkc_comm_id(uint8_t out[MHMKC_COMM_ID_BYTES]) {
  if (!out) return MHMKC_EINVAL;
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) {
    g_create_error = std::string("ncclGetUniqueId: ") + ncclGetErrorString(r);
    return MHMKC_ERCCL;
  }
  static_assert(sizeof(ncclUniqueId) == MHMKC_COMM_ID_BYTES, "unique id size");
  memcpy(out, &id, MHMKC_COMM_ID_BYTES);
  return MHMKC_OK;
}

int mhmkc_create(mhmkc_t *out, const mhmkc_config *cfg) {
  if (!out || !cfg) {
    g_create_error = "null argument";
    return MHMKC_EINVAL;
  }
  *out = nullptr;
  const int k = cfg->k;
  if (k < 1 || k > 127) {
    g_create_error = "k must be in [1, 127]";
    return MHMKC_EINVAL;
  }
  if (k % 32 == 0) {
    g_create_error = "k % 32 == 0 is not supported (EMPTY-slot aliasing, see DESIGN.md)";
    return MHMKC_EUNSUPPORTED;
  }
  const int nl = k / 32 + 1;
  const int nlo = cfg->n_longs ? cfg->n_longs : nl;
  if (nlo < nl || nlo > 8) {
    g_create_error = "n_longs must be 0 or in [k/32+1, 8]";
    return MHMKC_EINVAL;
  }
  if (cfg->qual_cutoff < 0 || cfg->qual_cutoff > 32 || (cfg->qual_offset != 33 && cfg->qual_offset != 64)) {
    g_create_error = "qual_offset must be 33 or 64 and qual_cutoff in [0, 32]";
    return MHMKC_EINVAL;
  }
  if (cfg->dmin_thres < 0 || cfg->dmin_thres > 32768) {
    g_create_error = "dmin_thres must be in [0, 32768] (DESIGN.md §3.4)";
    return MHMKC_EUNSUPPORTED;
  }
  if (!(cfg->dyn_min_depth >= 0.0 && cfg->dyn_min_depth <= 1.0)) {
    g_create_error = "dyn_min_depth must be in [0, 1]";
    return MHMKC_EINVAL;
  }
  // up to 255 ranks: the coarse partition has at most 2^11 bins (what a scatter workgroup keeps in registers,
  // scatter_staged), so beyond 8 ranks a rank owns 2048 / n_ranks of them (equal hash ranges when n_ranks divides
  // 2048); the supermer exchange keeps owners in bytes
  if (cfg->n_ranks < 1 || cfg->n_ranks > 255 || cfg->rank < 0 || cfg->rank >= cfg->n_ranks) {
    g_create_error = "bad rank / n_ranks (1..255 ranks)";
    return MHMKC_EINVAL;
  }
  if (cfg->output_owner != MHMKC_OWNER_HASH && cfg->output_owner != MHMKC_OWNER_MINIMIZER) {
    g_create_error = "output_owner must be MHMKC_OWNER_HASH or MHMKC_OWNER_MINIMIZER";
    return MHMKC_EINVAL;
  }
  const int mlen = cfg->minimizer_len ? cfg->minimizer_len : mhm::minimizer_len_for(k);
  if (cfg->output_owner == MHMKC_OWNER_MINIMIZER && (mlen < 1 || mlen > 28 || mlen > k)) {
    g_create_error = "minimizer_len must be in [1, min(k, 28)] (Kmer::get_minimizer_fast)";
    return MHMKC_EINVAL;
  }
  mhmkc *h = new mhmkc();
  h->cfg = *cfg;
  h->k = k;
  h->nl = nl;
  h->nlo = nlo;
  h->mlen = mlen;
  h->dmin = cfg->dmin_thres;
  h->qcut_pending = cfg->qual_cutoff;
  h->packed = mhm::ext_packs(k, nl);
  h->hbits = mhm::stored_hash_bits(k, nl, h->packed);
  // supermer exchange: the reference's owner (MHMKC_OWNER_MINIMIZER) with keys of two or more
  // words is reached by shipping supermers, each rank then counting all of its k-mers over the whole hash range;
  // (the test knob smer = 0 keeps the record exchange + hand-off)
  h->smer = cfg->output_owner == MHMKC_OWNER_MINIMIZER && cfg->n_ranks > 1 && nl >= 2 && g_dbg.smer != 0;
  int extra = 0;
  while ((1 << extra) < cfg->n_ranks && extra < 3) extra++;
  if (h->smer) extra = 0;
  // coarse bits by key words: three- and four-word keys take 128 coarse buckets (half the extraction's cursor atomics
  // per record and runs twice as long at ~0.5 records per base; k = 99 38.9 -> 34.8 ms per C2 step, k = 77 31.4 -> 31.0).
  // (7 coarse bits for two-word keys: k = 63 23.00 -> 23.31 ms.) The test knobs cb0 / cb0_2 / cb0_3 override them,
  // checked below.
  const int cb_knob = (int)g_dbg.cb0[nl >= 3 ? 3 : nl];
  const int cb0 = cb_knob ? cb_knob : nl >= 3 ? 7 : 8;
  // A mixed record keeps the key bits below the coarse digit, shifted up by the 6-bit ext code, in its first 64-bit
  // word: three/four-word keys (64 bits of w0') need cb >= 7 (at cb = 6 with no fine bits the mask shift reaches 64
  // and a key bit is lost: a wrong table, not an error), two-word keys (k bits of L') cb >= k - 58. The coarse
  // partition has at most 2^11 bins (scatter_staged).
  const int cb_min = nl >= 3 ? 7 : nl == 2 ? std::max(1, k - 58) : 1;
  if (cb0 < cb_min || cb0 + extra > 11) {
    delete h;
    g_create_error = "coarse bits out of range: " + std::to_string(cb0) + " + " + std::to_string(extra) +
                     " rank bits for k = " + std::to_string(k) + " (at least " + std::to_string(cb_min) +
                     ", at most 11 with the rank bits)";
    return MHMKC_EUNSUPPORTED;
  }
  h->cb = cb0 + extra;
  // compact records for 10 <= k <= 21 (the test knob wide_records keeps the key-word records: the tests compare both)
  const bool wide = g_dbg.wide_records != 0;
  h->compact = mhm::compact_ok(k, nl) && 2 * k - h->cb <= 34 && !wide;
  if (h->compact) h->hbits = 0;
  // mixed two-word records for 33 <= k <= 63 (the same switch keeps the plain key words)
  h->mixed2 = mhm::mixed2_ok(k, nl) && !wide;
  if (h->mixed2) {
    h->packed = true;  // the ext code sits in w[0]
    h->hbits = 0;
  }
  // mixed three- and four-word records for 64 < k < 128
  h->mixed3 = mhm::mixed3_ok(k, nl) && !wide;
  if (h->mixed3) {
    h->packed = true;  // the ext code sits in w[0]
    h->hbits = 0;
  }
  h->nb = 1u << h->cb;
  h->own_lo = h->smer ? 0 : h->owner_lo(cfg->rank);
  h->own_hi = h->smer ? h->nb : h->owner_lo(cfg->rank + 1);
  hipError_t e;
  if (cfg->device >= 0) {
    if ((e = hipSetDevice(cfg->device)) != hipSuccess) {
      g_create_error = std::string("hipSetDevice: ") + hipGetErrorString(e);
      delete h;
      return MHMKC_EHIP;
    }
  }
  (void)hipGetDevice(&h->dev);
  if (hipDeviceGetAttribute(&h->n_cu, hipDeviceAttributeMultiprocessorCount, h->dev) != hipSuccess) h->n_cu = 0;
  if (cfg->stream) {
    h->stream = (hipStream_t)cfg->stream;
  } else {
    if ((e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking)) != hipSuccess) {
      g_create_error = std::string("hipStreamCreate: ") + hipGetErrorString(e);
      delete h;
      return MHMKC_EHIP;
    }
    h->own_stream = true;
  }
  if ((e = hipStreamCreateWithFlags(&h->copy_stream, hipStreamNonBlocking)) != hipSuccess ||
      (e = hipEventCreate(&h->ev_begin)) != hipSuccess || (e = hipEventCreate(&h->ev_end)) != hipSuccess ||
      (e = hipEventCreate(&h->ev_h2d0)) != hipSuccess || (e = hipEventCreate(&h->ev_h2d1)) != hipSuccess ||
      (e = h->d_err.ensure(16)) != hipSuccess || (e = h->d_stats.ensure(8 * mhm::STAT_ALLOC)) != hipSuccess ||
      (e = hipMemset(h->d_err.p, 0, 16)) != hipSuccess) {
    g_create_error = std::string("init: ") + hipGetErrorString(e);
    mhmkc_destroy(h);
    return MHMKC_EHIP;
  }
  // pipelined record exchange (MHMKC_XPIPE=1; MHMKC_XPIECES: slabs per device batch). Opt-in: its
  // rounds are collectives inside the mhmkc_add_* calls, so every rank must go from its adds to mhmkc_finish with no
  // other collective of the same ranks in between; without it the exchange runs once, in finish.
  const char *xp_env = getenv("MHMKC_XPIPE");
  h->xpipe = cfg->n_ranks > 1 && !h->smer && xp_env && atoi(xp_env);
  h->lrounds = cfg->n_ranks == 1 && !h->smer && g_dbg.local_rounds != 0;
  if (const char *env = getenv("MHMKC_XPIECES")) h->xpieces = std::max(1, std::min(64, atoi(env)));
  if ((e = hipEventCreate(&h->ev_tail0)) != hipSuccess ||
      (h->xpipe && ((e = hipStreamCreateWithFlags(&h->xstream, hipStreamNonBlocking)) != hipSuccess ||
                    (e = hipEventCreate(&h->ev_xdone)) != hipSuccess || (e = hipEventCreate(&h->ev_xext)) != hipSuccess)) ||
      ((h->xpipe || h->lrounds) && ((e = hipStreamCreateWithFlags(&h->pstream, hipStreamNonBlocking)) != hipSuccess ||
                                    (e = hipEventCreateWithFlags(&h->ev_pdone, hipEventDisableTiming)) != hipSuccess))) {
    g_create_error = std::string("exchange stream: ") + hipGetErrorString(e);
    mhmkc_destroy(h);
    return MHMKC_EHIP;
  }
  (void)mhm::preload_owner_kernels();  // (the hand-off's code object: loaded here, not in the first fetch)
  if (cfg->n_ranks > 1 && cfg->comm_id) {
    ncclUniqueId id;
    memcpy(&id, cfg->comm_id, sizeof id);
    ncclResult_t r = ncclCommInitRank(&h->comm, cfg->n_ranks, id, cfg->rank);
    if (r != ncclSuccess) {
      g_create_error = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
      h->comm = nullptr;
      mhmkc_destroy(h);
      return MHMKC_ERCCL;
    }
  }
  *out = h;
  return MHMKC_OK;
}

void mhmkc_destroy(mhmkc_t h) {
  if (!h) return;
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  if (h->copy_stream) (void)hipStreamSynchronize(h->copy_stream);
  if (h->xstream) (void)hipStreamSynchronize(h->xstream);
  if (h->pstream) (void)hipStreamSynchronize(h->pstream);
  if (h->comm) ncclCommDestroy(h->comm);
  for (IncRound *q : h->inc_pool) {
    q->chunks.release();
    q->srcs.release();
    q->pin.release();
    delete q;
  }
  if (h->pstream) (void)hipStreamDestroy(h->pstream);
  if (h->ev_pdone) (void)hipEventDestroy(h->ev_pdone);
  if (h->ev_tail0) (void)hipEventDestroy(h->ev_tail0);
  for (RecvPart *q : h->parts) {
    q->buf.release();
    delete q;
  }
  for (hipEvent_t ev : h->x_ev) (void)hipEventDestroy(ev);
  if (h->ev_xdone) (void)hipEventDestroy(h->ev_xdone);
  if (h->ev_xext) (void)hipEventDestroy(h->ev_xext);
  if (h->xstream) (void)hipStreamDestroy(h->xstream);
  if (h->smer_slab) h->slabs.push_back(h->smer_slab);
  for (Slab *s : h->slabs) {
    if (s->ev) (void)hipEventDestroy(s->ev);
    s->buf.release();
    s->meta.release();
    s->pin.release();
    delete s;
  }
  for (Arena *a : h->arenas) {
    a->bytes.release();
    a->offs.release();
    delete a;
  }
  DevBuf *bufs[] = {&h->d_hist,     &h->d_tiles,      &h->d_err,        &h->d_stats,      &h->d_fine_hist,
                    &h->d_fine_base, &h->d_fine_cursor, &h->d_chunks,    &h->d_srcs,       &h->d_r2,
                    &h->d_out_keys, &h->d_out_counts, &h->d_out_left,   &h->d_out_right,  &h->d_out_cursor,
                    &h->d_recv,     &h->d_xg,         &h->d_hll,        &h->d_dest,       &h->d_ohist,
                    &h->d_out2_keys, &h->d_out2_counts, &h->d_out2_left, &h->d_out2_right, &h->d_mh, &h->d_ord,
                    &h->d_spill,      &h->d_cfit,       &h->d_xsend,      &h->d_xsegs,
                    &h->d_owners, &h->d_rcodes, &h->d_rgood, &h->d_rdesc, &h->d_rnwin, &h->d_rwpre, &h->d_rtiles,
                    &h->d_rtmp,
                    &h->d_fqa_bytes, &h->d_fqa_offs,
                    &h->d_fq_text,  &h->d_fq_chunk,   &h->d_fq_lines,   &h->d_fq_len,     &h->d_fq_tmp,
                    &h->d_fq_bytes, &h->d_fq_offs,    &h->d_fq_err};
  for (DevBuf *b : bufs) b->release();
  DevBuf *cbufs[] = {&h->d_ctg_bytes, &h->d_ctg_offs, &h->d_ctg_win,   &h->d_ctg_depth, &h->d_ctg_scratch,
                     &h->d_ctg_state, &h->d_ctg_bucket, &h->d_ctg_done, &h->d_ctg_keys[0], &h->d_ctg_keys[1],
                     &h->d_ctg_keys[2], &h->d_ctg_keys[3]};
  for (DevBuf *b : cbufs) b->release();
  h->x_send.release();
  h->x_recv.release();
  h->fq_file_buf.release();
  for (auto &p : h->prof) {
    h->ev_pool.push_back(p.a);
    h->ev_pool.push_back(p.b);
  }
  for (hipEvent_t ev : h->ev_pool) (void)hipEventDestroy(ev);
  for (hipEvent_t ev : h->chunk_ev) (void)hipEventDestroy(ev);
  for (DevBuf &b : h->d_nib) b.release();
  hipEvent_t evs[] = {h->ev_begin,  h->ev_end,    h->ev_h2d0,    h->ev_h2d1,       h->nib_ev[0],
                      h->nib_ev[1], h->nib_ev[2], h->stage_ev[0], h->stage_ev[1]};
  for (hipEvent_t ev : evs)
    if (ev) (void)hipEventDestroy(ev);
  if (h->copy_stream) (void)hipStreamDestroy(h->copy_stream);
  if (h->own_stream && h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
}

int mhmkc_add_reads_device(mhmkc_t h, const uint8_t *d_bytes, const uint64_t *d_offs, uint64_t n_reads,
                           uint64_t n_bases) {
  if (!h) return MHMKC_EINVAL;
  if (n_reads && (!d_bytes || !d_offs)) return h->fail(MHMKC_EINVAL, "null device buffer");
  int rc = h->begin_round();  // (records the round's start event before the reads are counted)
  if (rc) return rc;
  h->st.reads += n_reads;
  h->st.bases += n_bases;
  if (n_reads == 0) return MHMKC_OK;
  if (n_reads >= 0xffffffffull) return h->fail(MHMKC_EINVAL, "at most 2^32-2 reads per batch");
  h->qcut_pending = h->cfg.qual_cutoff;
  const uint64_t P = (uint64_t)h->xpieces;
  if (h->xpipe && P > 1 && n_reads >= 64 * P) {
    // pipelined exchange: the batch as xpieces slabs of whole reads, so that each one's round overlaps the next
    // one's extraction (the cut points' offsets come from the device)
    std::vector<uint64_t> cut(P + 1);
    hipError_t e = hipSuccess;
    for (uint64_t i = 0; i <= P && e == hipSuccess; i++)
      e = hipMemcpyAsync(&cut[i], d_offs + n_reads * i / P, 8, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return h->hip_fail(e, "read offsets");
    // (the pieces' views start at their own cut, so the window kernel's offs[0] == obase + head check cannot see
    // a batch whose first offset is not 0: checked here, as the unsplit path checks it on the device)
    if (cut[0] != 0)
      return h->fail(MHMKC_EINVAL, "device read offsets are not a PackedReads CSR (offs[0] == 0, non-decreasing, reads "
                                   "<= 65535 bases, offs[n_reads] == n_bases)");
    std::vector<mhm::ReadsView> rvs(P);
    for (uint64_t i = 0; i < P; i++) {
      const uint64_t r0 = n_reads * i / P, r1 = n_reads * (i + 1) / P;
      if (cut[i + 1] < cut[i] || cut[P] != n_bases)
        return h->fail(MHMKC_EINVAL, "device read offsets are not a PackedReads CSR (offs[n_reads] == n_bases)");
      mhm::ReadsView &rv = rvs[i];
      rv = mhm::ReadsView{};
      rv.obase = cut[i] & ~15ull;
      rv.head = (uint32_t)(cut[i] - rv.obase);
      rv.bytes = d_bytes + rv.obase;
      rv.offs = d_offs + r0;
      rv.n_reads = r1 - r0;
      rv.n_bases = cut[i + 1] - rv.obase;
    }
    // every piece's windows (and the CSR checks) in one go: the batch's windows are announced to the other ranks by
    // the exchange rounds (the incremental partition's layout), then the pieces become slabs
    std::vector<uint64_t> wins(P, 0);
    unsigned int ef = 0;
    if ((e = h->grow(h->d_hist, (size_t)(h->nb + P) * 8 + 64)) != hipSuccess) return h->hip_fail(e, "histogram");
    unsigned long long *d_wins = h->d_hist.as<unsigned long long>() + h->nb;
    h->prof_begin(MHMKC_STAGE_TILEIDX);
    e = hipMemsetAsync(d_wins, 0, 8 * P, h->stream);
    for (uint64_t i = 0; i < P && e == hipSuccess; i++)
      e = mhm::launch_count_windows(rvs[i], h->k, d_wins + i, h->d_err.as<unsigned int>(), h->stream);
    h->prof_end();
    if (e == hipSuccess) e = hipMemcpyAsync(wins.data(), d_wins, 8 * P, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(&ef, h->d_err.p, 4, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return h->hip_fail(e, "window count");
    if (ef & 4u)
      return h->fail(MHMKC_EINVAL, "device read offsets are not a PackedReads CSR (offs[0] == 0, non-decreasing, reads "
                                   "<= 65535 bases, offs[n_reads] == n_bases)");
    uint64_t tot = 0;
    for (uint64_t w : wins) tot += w;
    h->inc_expect += tot;
    h->inc_announced += tot;
    for (uint64_t i = 0; i < P; i++)
      if ((rc = h->add_view(rvs[i], wins[i], true))) return rc;
    return MHMKC_OK;
  }
  mhm::ReadsView rv{d_bytes, d_offs, n_reads, n_bases, 0, 0, 0};
  return h->add_view(rv, 0, false);
}

int mhmkc_wait_stream(mhmkc_t h, void *stream) {
  if (!h) return MHMKC_EINVAL;
  hipEvent_t ev = h->take_event();
  hipError_t e = hipEventRecord(ev, (hipStream_t)stream);
  if (e == hipSuccess) e = hipStreamWaitEvent(h->stream, ev, 0);
  h->ev_pool.push_back(ev);  // reusable: a later record replaces the captured work, the wait is enqueued
  return e == hipSuccess ? MHMKC_OK : h->hip_fail(e, "wait_stream");
}

// FASTQ text on the device -> PackedReads in d_fq_bytes / d_fq_offs -> add_view (fastq.hip).
int mhmkc::add_fastq(const char *d_text, uint64_t n, bool pairs, uint64_t *consumed) {
  int rc = begin_round();
  if (rc) return rc;
  if (consumed) *consumed = 0;
  fq_reads = fq_bases = 0;
  if (pairs) st.fq_pairs = st.fq_merged = st.fq_ambiguous = st.fq_overlap_bases = 0;
  if (n == 0) return MHMKC_OK;
  if (n > mhm::FQ_LE_MASK) return fail(MHMKC_EINVAL, "FASTQ text larger than 2^40 bytes in one call");
  // the packed reads of an earlier add_fastq may still be read by a pending extraction: settle it first
  if ((rc = resolve_slabs())) return rc;
  hipError_t e;
  const uint64_t nch = (n + mhm::FQ_CHUNK - 1) / mhm::FQ_CHUNK;
  if ((e = grow(d_fq_chunk, (nch + 1) * 16)) != hipSuccess) return hip_fail(e, "fastq chunk counts");
  unsigned long long *cnt = d_fq_chunk.as<unsigned long long>(), *cbase = cnt + nch + 1;
  size_t tmp_bytes = mhm::fq_scan_tmp_bytes(nch + 1);
  if ((e = grow(d_fq_tmp, tmp_bytes)) != hipSuccess) return hip_fail(e, "fastq scan scratch");
  prof_begin(MHMKC_STAGE_OTHER);
  e = hipMemsetAsync(cnt + nch, 0, 8, stream);
  if (e == hipSuccess) e = mhm::launch_fq_count(d_text, n, cnt, stream);
  if (e == hipSuccess) e = mhm::fq_scan(d_fq_tmp.p, tmp_bytes, cnt, cbase, nch + 1, stream);
  prof_end();
  if (e != hipSuccess) return hip_fail(e, "fastq newline count");
  unsigned long long newlines = 0;
  char last = 0;
  if ((e = hipMemcpyAsync(&newlines, cbase + nch, 8, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
      (e = hipMemcpyAsync(&last, d_text + n - 1, 1, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
      (e = hipStreamSynchronize(stream)) != hipSuccess)
    return hip_fail(e, "fastq newline count D2H");
  // fgets returns a last line without its newline; a block's last line without one continues in the next block
  const uint64_t all_lines = newlines + (last != '\n' ? 1 : 0);
  const uint64_t lines = consumed ? (pairs ? newlines / 8 * 8 : newlines / 4 * 4) : all_lines;
  const uint64_t R = lines / 4;
  if (consumed && R == 0) return MHMKC_OK;  // no complete record (pair) yet: the caller reads more
  if ((e = grow(d_fq_lines, std::max<uint64_t>(all_lines, 1) * 8)) != hipSuccess) return hip_fail(e, "fastq lines");
  if ((e = grow(d_fq_len, (R + 1) * 8)) != hipSuccess || (e = grow(d_fq_offs, (R + 1) * 8)) != hipSuccess ||
      (e = grow(d_fq_err, 8)) != hipSuccess)
    return hip_fail(e, "fastq records");
  const size_t tmp2 = mhm::fq_scan_tmp_bytes(R + 1);
  if (tmp2 > tmp_bytes) {
    if ((e = grow(d_fq_tmp, tmp2)) != hipSuccess) return hip_fail(e, "fastq scan scratch");
    tmp_bytes = tmp2;
  }
  unsigned long long *lend = d_fq_lines.as<unsigned long long>(), *len = d_fq_len.as<unsigned long long>();
  unsigned long long *offs = d_fq_offs.as<unsigned long long>(), *err_d = d_fq_err.as<unsigned long long>();
  const unsigned long long n_end = n;
  prof_begin(MHMKC_STAGE_OTHER);
  e = mhm::launch_fq_lines(d_text, n, cbase, lend, stream);
  if (e == hipSuccess && !consumed && last != '\n')
    e = hipMemcpyAsync(lend + lines - 1, &n_end, 8, hipMemcpyHostToDevice, stream);
  if (e == hipSuccess) e = hipMemsetAsync(err_d, 0xff, 8, stream);
  if (e == hipSuccess && pairs) {  // the records' checks and the pairs' descriptors in one pass
    if ((e = grow(d_fq_desc, mhm::fq_pair_desc_bytes(R / 2))) == hipSuccess)
      e = mhm::launch_fq_pair_records(d_text, n, lend, R, len, err_d, d_fq_desc.p, stream);
  } else if (e == hipSuccess) {
    e = mhm::launch_fq_records(d_text, n, lend, R, len, err_d, stream);
  }
  if (e == hipSuccess) e = mhm::fq_scan(d_fq_tmp.p, tmp_bytes, len, offs, R + 1, stream);
  prof_end();
  if (e != hipSuccess) return hip_fail(e, "fastq records");
  unsigned long long n_bases = 0;
  if ((e = hipMemcpyAsync(&n_bases, offs + R, 8, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
      (e = hipStreamSynchronize(stream)) != hipSuccess)
    return hip_fail(e, "fastq records D2H");
  uint64_t R_out = R;  // reads added (pairs: two per pair)
  if (!pairs) {
    if ((e = grow(d_fq_bytes, std::max<uint64_t>(n_bases, 1) + 64)) != hipSuccess) return hip_fail(e, "fastq bytes");
    prof_begin(MHMKC_STAGE_OTHER);
    e = mhm::launch_fq_pack(d_text, lend, R, offs, cfg.qual_offset, d_fq_bytes.as<uint8_t>(), err_d, stream);
    prof_end();
  } else {
    // merge_reads: the record offsets lay out the quality scratch; the pair verdicts give the output lengths
    const uint64_t P = R / 2;
    R_out = 2 * P;
    if ((e = grow(d_fq_recoffs, (R + 1) * 8)) != hipSuccess ||
        (e = grow(d_fq_scratch, std::max<uint64_t>(n_bases, 1) + 64)) != hipSuccess ||
        (e = grow(d_fq_pairinfo, (P + 1) * 4)) != hipSuccess || (e = grow(d_fq_stats, 128)) != hipSuccess ||
        (e = grow(d_fq_desc, mhm::fq_pair_desc_bytes(P))) != hipSuccess ||
        (e = grow(d_fq_len, (2 * P + 1) * 8)) != hipSuccess)
      return hip_fail(e, "fastq pairs");
    const size_t tmp3 = mhm::fq_scan_tmp_bytes(2 * P + 1);
    if (tmp3 > tmp_bytes) {
      if ((e = grow(d_fq_tmp, tmp3)) != hipSuccess) return hip_fail(e, "fastq scan scratch");
      tmp_bytes = tmp3;
    }
    unsigned long long *roffs = d_fq_recoffs.as<unsigned long long>(), *fst = d_fq_stats.as<unsigned long long>();
    unsigned long long *len2 = d_fq_len.as<unsigned long long>();
    prof_begin(MHMKC_STAGE_OTHER);
    e = hipMemcpyAsync(roffs, offs, (R + 1) * 8, hipMemcpyDeviceToDevice, stream);
    if (e == hipSuccess) e = hipMemsetAsync(fst, 0, 128, stream);
    if (e == hipSuccess)
      e = mhm::launch_fq_merge(d_text, n, lend, P, roffs, cfg.qual_offset, d_fq_scratch.as<char>(), d_fq_desc.p,
                               d_fq_pairinfo.as<uint32_t>(), len2, err_d, fst, stream);
    if (e == hipSuccess) e = mhm::fq_scan(d_fq_tmp.p, tmp_bytes, len2, offs, 2 * P + 1, stream);
    prof_end();
    if (e != hipSuccess) return hip_fail(e, "fastq merge");
    unsigned long long hs[4] = {0, 0, 0, 0};
    if ((e = hipMemcpyAsync(&n_bases, offs + 2 * P, 8, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
        (e = hipMemcpyAsync(hs, fst, 32, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
        (e = hipStreamSynchronize(stream)) != hipSuccess)
      return hip_fail(e, "fastq merge D2H");
    st.fq_pairs = P;
    st.fq_merged = hs[1];
    st.fq_ambiguous = hs[2];
    st.fq_overlap_bases = hs[3];
    if ((e = grow(d_fq_bytes, std::max<uint64_t>(n_bases, 1) + 64)) != hipSuccess) return hip_fail(e, "fastq bytes");
    prof_begin(MHMKC_STAGE_OTHER);
    e = mhm::launch_fq_merge_pack(d_text, d_fq_desc.p, P, roffs, d_fq_scratch.as<char>(), d_fq_pairinfo.as<uint32_t>(),
                                  offs, cfg.qual_offset, d_fq_bytes.as<uint8_t>(), err_d, stream);
    prof_end();
  }
  unsigned long long first_err = ~0ull;
  if (e == hipSuccess) e = hipMemcpyAsync(&first_err, err_d, 8, hipMemcpyDeviceToHost, stream);
  if (e == hipSuccess) e = hipStreamSynchronize(stream);
  if (e != hipSuccess) return hip_fail(e, "fastq pack");
  if (lines % 4) first_err = std::min<unsigned long long>(first_err, ((unsigned long long)R << 4) | mhm::FQ_E_TRUNC);
  if (first_err != ~0ull) {
    unsigned long long rec = first_err >> 4;
    switch ((int)(first_err & 15)) {
      case mhm::FQ_E_PAIR_NAME:
        return fail(MHMKC_EINVAL, "FASTQ records %llu and %llu: mismatched pair names", rec - 1, rec);
      case mhm::FQ_E_PAIR_NUM:
        return fail(MHMKC_EINVAL, "FASTQ records %llu and %llu: mismatched pair numbers (not /1, /2)", rec - 1, rec);
      case mhm::FQ_E_CHAR2: return fail(MHMKC_EBADCHAR, "FASTQ record %llu: illegal base character", rec);
      case mhm::FQ_E_QUAL:
        return fail(MHMKC_EINVAL, "FASTQ records %llu and %llu: invalid quality score in the overlap", rec - 1, rec);
      case mhm::FQ_E_CHAR1: return fail(MHMKC_EBADCHAR, "FASTQ record %llu: illegal base character", rec - 1);
      case mhm::FQ_E_ID: return fail(MHMKC_EINVAL, "invalid FASTQ record %llu: expected read name (@)", rec);
      case mhm::FQ_E_PLUS: return fail(MHMKC_EINVAL, "invalid FASTQ record %llu: expected '+'", rec);
      case mhm::FQ_E_NAME: return fail(MHMKC_EINVAL, "invalid FASTQ record %llu: incorrect name format", rec);
      case mhm::FQ_E_LEN:
        return fail(MHMKC_EINVAL, "invalid FASTQ record %llu: sequence length != quals length", rec);
      case mhm::FQ_E_LONG:
        return fail(MHMKC_EUNSUPPORTED, "FASTQ record %llu: line longer than %llu characters", rec,
                    (unsigned long long)mhm::FQ_MAX_LINE);
      case mhm::FQ_E_CHAR: return fail(MHMKC_EBADCHAR, "FASTQ record %llu: illegal base character", rec);
      default: return fail(MHMKC_EINVAL, "FASTQ text ends inside record %llu", rec);
    }
  }
  if (consumed) {  // the text of the complete records: up to the newline of their last line
    unsigned long long le = 0;
    if ((e = hipMemcpy(&le, lend + lines - 1, 8, hipMemcpyDeviceToHost)) != hipSuccess) return hip_fail(e, "fastq block end");
    *consumed = std::min<uint64_t>(n, (uint64_t)(le & mhm::FQ_LE_MASK) + 1);
  }
  fq_reads = R_out;
  fq_bases = n_bases;
  st.reads += R_out;
  st.bases += n_bases;
  if (R_out == 0) return MHMKC_OK;
  qcut_pending = cfg.qual_cutoff;
  // the offsets were made here from checked records: the window count kernel re-checks them anyway
  mhm::ReadsView rv{d_fq_bytes.as<uint8_t>(), d_fq_offs.as<uint64_t>(), R_out, n_bases, 0, 0, 0};
  return add_view(rv, 0, false);
}

int mhmkc_add_reads(mhmkc_t h, const uint8_t *bytes, const uint64_t *offs, uint64_t n_reads) {
  if (!h) return MHMKC_EINVAL;
  if (!offs || (n_reads && !bytes)) return h->fail(MHMKC_EINVAL, "null host buffer");
  return h->add_host(bytes, offs, n_reads, h->cfg.qual_cutoff);
}

int mhmkc_add_fastq_device(mhmkc_t h, const char *d_text, uint64_t n_bytes) {
  if (!h) return MHMKC_EINVAL;
  if (n_bytes && !d_text) return h->fail(MHMKC_EINVAL, "null device buffer");
  return h->add_fastq(d_text, n_bytes);
}

int mhmkc_add_fastq_pairs_device(mhmkc_t h, const char *d_text, uint64_t n_bytes) {
  if (!h) return MHMKC_EINVAL;
  if (n_bytes && !d_text) return h->fail(MHMKC_EINVAL, "null device buffer");
  return h->add_fastq(d_text, n_bytes, true);
}

static int add_fastq_host(mhmkc_t h, const char *text, uint64_t n_bytes, bool pairs) {
  if (!h) return MHMKC_EINVAL;
  if (n_bytes && !text) return h->fail(MHMKC_EINVAL, "null host buffer");
  int rc = h->resolve_slabs();  // an earlier add_fastq's text may still be read
  if (rc) return rc;
  hipError_t e;
  if ((e = h->grow(h->d_fq_text, n_bytes + 16)) != hipSuccess) return h->hip_fail(e, "fastq staging");
  if (n_bytes && (e = hipMemcpyAsync(h->d_fq_text.p, text, n_bytes, hipMemcpyHostToDevice, h->stream)) != hipSuccess)
    return h->hip_fail(e, "fastq H2D");
  rc = h->add_fastq(h->d_fq_text.as<char>(), n_bytes, pairs);
  if (rc == MHMKC_OK && (e = hipStreamSynchronize(h->stream)) != hipSuccess) return h->hip_fail(e, "add_fastq");
  return rc;
}

int mhmkc_add_fastq(mhmkc_t h, const char *text, uint64_t n_bytes) { return add_fastq_host(h, text, n_bytes, false); }

// A FASTQ file (interleaved pairs with `pairs`) read in blocks of MHMKC_FQ_BLOCK bytes (default 256 MB) into two
// pinned buffers: while block i is copied to the device and parsed, block i + 1 is read by a reader thread (with
// MHMKC_FQ_THREADS parallel preads, default 8), and the extraction of block i runs on the device while block i + 1
// is parsed: file I/O overlapped with the count kernels (the reference reads its share of the
// file with FastqReader, src/fastq.cpp:504-551, and counts after the whole read). Each block's last, possibly cut,
// record (pair) is carried to the front of the next block (a reserve of FQ_CARRY bytes before its data).
constexpr uint64_t FQ_CARRY = 1ull << 20;
static int add_fastq_file(mhmkc_t h, const char *path, bool pairs) {
  if (!h) return MHMKC_EINVAL;
  if (!path) return h->fail(MHMKC_EINVAL, "null path");
  const int fd = open(path, O_RDONLY);
  if (fd < 0) return h->fail(MHMKC_EINVAL, "cannot open FASTQ file %s", path);
  struct stat sb;
  if (fstat(fd, &sb) != 0) {
    close(fd);
    return h->fail(MHMKC_EINVAL, "cannot stat FASTQ file %s", path);
  }
  const uint64_t size = (uint64_t)sb.st_size;
  uint64_t block = 256ull << 20;
  if (const char *env = getenv("MHMKC_FQ_BLOCK")) block = std::max<uint64_t>(64, strtoull(env, nullptr, 10));
  int nthr = 8;
  if (const char *env = getenv("MHMKC_FQ_THREADS")) nthr = std::max(1, std::min(64, atoi(env)));
  const uint64_t slot = FQ_CARRY + block + 64;  // one buffer: carry reserve | block data | padding
  hipError_t e;
  if ((e = h->fq_file_buf.ensure(2 * slot)) != hipSuccess) {
    close(fd);
    return h->hip_fail(e, "fastq file blocks");
  }
  char *buf[2] = {h->fq_file_buf.as<char>(), h->fq_file_buf.as<char>() + slot};
  bool added = false;  // some block's reads are in the round (a later failure leaves the round partial)
  // tests only: the read of block fq_read_fail fails (a file that shrinks or turns unreadable mid-call)
  const uint64_t fail_block = g_dbg.fq_read_fail >= 0 ? (uint64_t)g_dbg.fq_read_fail : ~0ull;
  // block i's data: file bytes [i * block, min(size, (i + 1) * block)), read in parallel pieces
  auto read_block = [&](uint64_t i, char *dst) -> bool {
    if (i == fail_block) return false;
    const uint64_t off = i * block, len = std::min(block, size - off);
    const uint64_t piece = (len + nthr - 1) / nthr;
    std::vector<std::thread> th;
    std::vector<char> ok(nthr, 1);
    for (int t = 0; t < nthr; t++) {
      const uint64_t a = std::min(len, t * piece), b = std::min(len, a + piece);
      if (a == b) continue;
      th.emplace_back([&, t, a, b] {
        for (uint64_t p = a; p < b;) {
          const ssize_t r = pread(fd, dst + p, (size_t)(b - p), (off_t)(off + p));
          if (r <= 0) {
            ok[t] = 0;
            return;
          }
          p += (uint64_t)r;
        }
      });
    }
    for (auto &x : th) x.join();
    for (char v : ok)
      if (!v) return false;
    return true;
  };
  const uint64_t n_blocks = (size + block - 1) / block;
  // the PackedReads of every block, appended on the device (the later k rounds count them again, as the
  // reference keeps packed_reads_list, src/main.cpp); a buffer that grows keeps its content
  uint64_t a_reads = 0, a_bases = 0;
  auto keep_grow = [&](DevBuf &b, size_t used, size_t need) -> hipError_t {
    if (need <= b.cap && b.p) return hipSuccess;
    hipError_t ge = hipStreamSynchronize(h->stream);
    if (ge != hipSuccess) return ge;
    DevBuf nb;
    if ((ge = nb.ensure(std::max(need, 2 * b.cap))) != hipSuccess) return ge;
    if (used && b.p && (ge = hipMemcpy(nb.p, b.p, std::min(used, b.cap), hipMemcpyDeviceToDevice)) != hipSuccess) {
      nb.release();
      return ge;
    }
    b.release();
    b = nb;
    return hipSuccess;
  };
  int rc = MHMKC_OK;
  uint64_t carry = 0, blocks = 0;
  uint64_t acc[4] = {0, 0, 0, 0};  // pair statistics summed over the blocks
  if (n_blocks && !read_block(0, buf[0] + FQ_CARRY)) rc = h->fail(MHMKC_EINVAL, "read error in FASTQ file %s", path);
  for (uint64_t i = 0; rc == MHMKC_OK && i < n_blocks; i++) {
    char *cur = buf[i & 1], *nxt = buf[(i + 1) & 1];
    const uint64_t len = std::min(block, size - i * block);
    char *text = cur + FQ_CARRY - carry;
    const uint64_t n = carry + len;
    const bool last = i + 1 == n_blocks;
    bool read_ok = true;
    std::thread reader;
    if (!last) reader = std::thread([&, i] { read_ok = read_block(i + 1, nxt + FQ_CARRY); });
    uint64_t used = 0;
    if ((rc = h->resolve_slabs()) == MHMKC_OK) {  // the previous block's text may still be read by its extraction
      if ((e = h->grow(h->d_fq_text, n + 16)) != hipSuccess ||
          (e = hipMemcpyAsync(h->d_fq_text.p, text, n, hipMemcpyHostToDevice, h->stream)) != hipSuccess)
        rc = h->hip_fail(e, "fastq block H2D");
      else
        rc = h->add_fastq(h->d_fq_text.as<char>(), n, pairs, last ? nullptr : &used);
      if (rc == MHMKC_OK) added = true;
    }
    if (reader.joinable()) reader.join();
    if (rc) {  // locate the bad record: the parser numbers records from the start of this block's text
      char where[160];
      snprintf(where, sizeof where, " (FASTQ file block %llu, whose text starts at file byte %llu)",
               (unsigned long long)i, (unsigned long long)(i * block - carry));
      h->err += where;
      break;
    }
    if (!read_ok) {
      rc = h->fail(MHMKC_EINVAL, "read error in FASTQ file %s", path);
      break;
    }
    blocks++;
    if (h->fq_reads) {
      const uint64_t r = h->fq_reads, nb = h->fq_bases;
      if ((e = keep_grow(h->d_fqa_bytes, a_bases, a_bases + nb + 64)) != hipSuccess ||
          (e = keep_grow(h->d_fqa_offs, (a_reads + 1) * 8, (a_reads + r + 1) * 8)) != hipSuccess ||
          (a_reads == 0 && (e = hipMemsetAsync(h->d_fqa_offs.p, 0, 8, h->stream)) != hipSuccess) ||
          (nb && (e = hipMemcpyAsync(h->d_fqa_bytes.as<char>() + a_bases, h->d_fq_bytes.p, nb, hipMemcpyDeviceToDevice,
                                     h->stream)) != hipSuccess) ||
          (e = mhm::launch_offs_rebase(h->d_fqa_offs.as<unsigned long long>() + a_reads + 1,
                                       h->d_fq_offs.as<unsigned long long>() + 1, r, a_bases, h->stream)) != hipSuccess) {
        rc = h->hip_fail(e, "fastq file packed reads");
        break;
      }
      a_reads += r;
      a_bases += nb;
    }
    if (pairs) {
      acc[0] += h->st.fq_pairs, acc[1] += h->st.fq_merged, acc[2] += h->st.fq_ambiguous, acc[3] += h->st.fq_overlap_bases;
    }
    if (last) break;
    carry = n - used;  // the cut record (pair), or the whole block if it held no complete one
    if (carry > FQ_CARRY) {
      rc = h->fail(MHMKC_EUNSUPPORTED, "FASTQ record longer than %llu bytes", (unsigned long long)FQ_CARRY);
      break;
    }
    memcpy(nxt + FQ_CARRY - carry, text + used, carry);
  }
  close(fd);
  // earlier blocks may already be in the round (counted reads, extractions enqueued): the handle refuses to
  // finish a round that holds part of a file until mhmkc_reset
  if (rc && added) h->partial = true;
  if (rc == MHMKC_OK) {  // mhmkc_fastq_packed / mhmkc_fastq_fetch now see every block's PackedReads
    if (a_reads == 0 && ((e = keep_grow(h->d_fqa_offs, 0, 8)) != hipSuccess ||
                         (e = hipMemsetAsync(h->d_fqa_offs.p, 0, 8, h->stream)) != hipSuccess))
      rc = h->hip_fail(e, "fastq file packed reads");
    std::swap(h->d_fq_bytes, h->d_fqa_bytes);  // (the last block's extraction may still read the old buffer:
    std::swap(h->d_fq_offs, h->d_fqa_offs);    //  both stay allocated)
    h->fq_reads = a_reads;
    h->fq_bases = a_bases;
  }
  if (pairs) h->st.fq_pairs = acc[0], h->st.fq_merged = acc[1], h->st.fq_ambiguous = acc[2], h->st.fq_overlap_bases = acc[3];
  h->st.fq_file_blocks = blocks;
  return rc;
}

int mhmkc_add_fastq_file(mhmkc_t h, const char *path) { return add_fastq_file(h, path, false); }
int mhmkc_add_fastq_pairs_file(mhmkc_t h, const char *path) { return add_fastq_file(h, path, true); }

int mhmkc_add_fastq_pairs(mhmkc_t h, const char *text, uint64_t n_bytes) {
  return add_fastq_host(h, text, n_bytes, true);
}

int mhmkc_fastq_packed(mhmkc_t h, const uint8_t **d_bytes, const uint64_t **d_offsets, uint64_t *n_reads,
                       uint64_t *n_bases) {
  if (!h) return MHMKC_EINVAL;
  if (d_bytes) *d_bytes = h->d_fq_bytes.as<uint8_t>();
  if (d_offsets) *d_offsets = h->d_fq_offs.as<uint64_t>();
  if (n_reads) *n_reads = h->fq_reads;
  if (n_bases) *n_bases = h->fq_bases;
  return MHMKC_OK;
}

int mhmkc_fastq_fetch(mhmkc_t h, uint8_t *bytes, uint64_t *offsets) {
  if (!h) return MHMKC_EINVAL;
  hipError_t e = hipSuccess;
  if (bytes && h->fq_bases) e = hipMemcpyAsync(bytes, h->d_fq_bytes.p, h->fq_bases, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess && offsets) {
    if (h->d_fq_offs.p && h->fq_reads)
      e = hipMemcpyAsync(offsets, h->d_fq_offs.p, (h->fq_reads + 1) * 8, hipMemcpyDeviceToHost, h->stream);
    else
      offsets[0] = 0;
  }
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  return e == hipSuccess ? MHMKC_OK : h->hip_fail(e, "fastq fetch");
}

// PackedRead code of a sequence character; case carries the quality (SeqBlockInserter::process_seq input,
// src/kcount/kcount.cpp:80-86; quals[i] = isupper, src/kcount/kcount_cpu.cpp:309-312). -1: not A/C/G/T/N
// (HashTableInserter::insert_supermer DIEs, src/kcount/kcount_cpu.cpp:452-458).
static int seq_byte(char c) {
  int code;
  switch (c) {
    case 'A': case 'a': code = 0; break;
    case 'C': case 'c': code = 1; break;
    case 'G': case 'g': code = 2; break;
    case 'T': case 't': code = 3; break;
    case 'N': case 'n': code = 4; break;
    default: return -1;
  }
  return code | ((c >= 'A' && c <= 'Z') ? (31 << 3) : 0);
}

int mhmkc_add_seqs(mhmkc_t h, const char *seqs, const uint64_t *offs, uint64_t n_seqs, uint16_t depth) {
  if (!h) return MHMKC_EINVAL;
  if (!offs || (n_seqs && !seqs)) return h->fail(MHMKC_EINVAL, "null host buffer");
  if (depth > 1) return h->fail(MHMKC_EUNSUPPORTED, "depth > 1 is a contig supermer: use mhmkc_add_ctgs");
  if (offs[0] != 0) return h->fail(MHMKC_EINVAL, "seq_offsets[0] must be 0");
  for (uint64_t i = 0; i < n_seqs; i++)
    if (offs[i + 1] < offs[i]) return h->fail(MHMKC_EINVAL, "seq_offsets must be non-decreasing");
  const uint64_t n = offs[n_seqs];
  // uppercase -> q 31, lowercase -> q 0, and the batch runs with cutoff 1
  std::vector<uint8_t> bytes(n);
  for (uint64_t i = 0; i < n; i++) {
    const int b = seq_byte(seqs[i]);
    if (b < 0) return h->fail(MHMKC_EBADCHAR, "bad char '%c' (%d) at position %llu", seqs[i], (int)seqs[i], (unsigned long long)i);
    bytes[i] = (uint8_t)b;
  }
  return h->add_host(bytes.data(), offs, n_seqs, 1);
}

int mhmkc_add_ctgs(mhmkc_t h, const char *seqs, const uint64_t *offs, const uint16_t *depths, uint64_t n_ctgs) {
  if (!h) return MHMKC_EINVAL;
  if (!offs || (n_ctgs && (!seqs || !depths))) return h->fail(MHMKC_EINVAL, "null host buffer");
  if (h->finished) return h->fail(MHMKC_ESTATE, "handle already finished; call mhmkc_reset first");
  if (offs[0] != 0) return h->fail(MHMKC_EINVAL, "seq_offsets[0] must be 0");
  const uint64_t k = (uint64_t)h->k;
  uint64_t W = h->ctg_win.back();
  for (uint64_t i = 0; i < n_ctgs; i++) {
    if (offs[i + 1] < offs[i]) return h->fail(MHMKC_EINVAL, "seq_offsets must be non-decreasing");
    const uint64_t L = offs[i + 1] - offs[i];
    W += L >= k + 2 ? L - k - 1 : 0;  // add_ctg_kmers skips contigs shorter than k + 2 (src/kcount/kcount.cpp:128)
  }
  if (W >= 0xffffffffull) return h->fail(MHMKC_EINVAL, "at most 2^32-1 contig k-mers per round");
  const uint64_t n = offs[n_ctgs];
  const size_t b0 = h->ctg_bytes.size();
  h->ctg_bytes.resize(b0 + n);
  // case carries the quality as for reads (get_kmers_and_exts: quals[i] = isupper, kcount_cpu.cpp:309-313);
  // contigs are uppercase. Characters other than ACGTN are fatal (insert_supermer DIE, :452-458).
  for (uint64_t i = 0; i < n; i++) {
    const int b = seq_byte(seqs[i]);
    if (b < 0) {
      h->ctg_bytes.resize(b0);
      return h->fail(MHMKC_EBADCHAR, "bad char '%c' (%d) in contig position %llu", seqs[i], (int)seqs[i],
                     (unsigned long long)i);
    }
    h->ctg_bytes[b0 + i] = (uint8_t)b;
  }
  for (uint64_t i = 0; i < n_ctgs; i++) {
    const uint64_t L = offs[i + 1] - offs[i];
    h->ctg_offs.push_back(b0 + offs[i + 1]);
    h->ctg_win.push_back(h->ctg_win.back() + (L >= k + 2 ? L - k - 1 : 0));  // interior windows only
    h->ctg_depth.push_back(depths[i]);
  }
  return MHMKC_OK;
}

int mhmkc_set_dmin_thres(mhmkc_t h, int32_t dmin_thres) {
  if (!h) return MHMKC_EINVAL;
  if (dmin_thres < 0 || dmin_thres > 32768)
    return h->fail(MHMKC_EUNSUPPORTED, "dmin_thres must be in [0, 32768] (DESIGN.md §3.4)");
  if (h->finished) return h->fail(MHMKC_ESTATE, "handle already finished; call mhmkc_reset first");
  h->dmin = dmin_thres;
  return MHMKC_OK;
}

int mhmkc_set_transport(mhmkc_t h, const mhmkc_transport *t) {
  if (!h) return MHMKC_EINVAL;
  if (!t || !t->allgather || !t->alltoallv) return h->fail(MHMKC_EINVAL, "transport needs allgather and alltoallv");
  if (h->comm) return h->fail(MHMKC_EINVAL, "the handle already has an RCCL communicator (comm_id)");
  h->xp = *t;
  h->has_xp = true;
  // A host-staged transport moves a few GB/s, so the last exchange round (the one no extraction overlaps) is
  // what a step waits for: cut the batch finer (2 ranks, C2: 252 -> 57 ms exposed for 4 % more bytes, DESIGN.md
  // §3.5e). RCCL over xGMI takes 8 (the sends carry no slack since round 5, §3.5f).
  if (!getenv("MHMKC_XPIECES")) h->xpieces = 16;
  return MHMKC_OK;
}

int mhmkc_minimizer_hashes(mhmkc_t h, const uint64_t *keys, uint64_t n, int32_t n_longs, int32_t m, uint64_t *hashes) {
  if (!h) return MHMKC_EINVAL;
  if (n && (!keys || !hashes)) return h->fail(MHMKC_EINVAL, "null host buffer");
  if (n_longs < h->nl || n_longs > 8) return h->fail(MHMKC_EINVAL, "n_longs must be in [k/32+1, 8]");
  const int mm = m ? m : mhm::minimizer_len_for(h->k);
  if (mm < 1 || mm > 28 || mm > h->k) return h->fail(MHMKC_EINVAL, "m must be in [1, min(k, 28)]");
  if (!n) return MHMKC_OK;
  hipError_t e;
  if ((e = h->grow(h->d_mh, n * 8 * ((size_t)n_longs + 1) + 64)) != hipSuccess) return h->hip_fail(e, "minimizer buffers");
  uint64_t *dk = h->d_mh.as<uint64_t>(), *dh = dk + n * n_longs;
  if ((e = hipMemcpyAsync(dk, keys, n * 8 * n_longs, hipMemcpyHostToDevice, h->stream)) != hipSuccess ||
      (e = mhm::launch_minimizer_hash(dk, n, n_longs, h->k, mm, dh, h->stream)) != hipSuccess ||
      (e = hipMemcpyAsync(hashes, dh, n * 8, hipMemcpyDeviceToHost, h->stream)) != hipSuccess ||
      (e = hipStreamSynchronize(h->stream)) != hipSuccess)
    return h->hip_fail(e, "minimizer hashes");
  return MHMKC_OK;
}

int mhmkc_finish(mhmkc_t h, uint64_t *n_out) {
  if (!h) return MHMKC_EINVAL;
  return h->finish(n_out);
}

int mhmkc_fetch(mhmkc_t h, uint64_t *keys, uint16_t *counts, char *left, char *right) {
  if (!h) return MHMKC_EINVAL;
  if (!h->finished) return h->fail(MHMKC_ESTATE, "fetch before finish");
  const uint64_t n = h->n_out;
  hipError_t e = hipSuccess;
  if (n && keys) e = h->d2h(keys, h->d_out_keys.p, n * 8 * h->nlo);
  if (e == hipSuccess && n && counts) e = h->d2h(counts, h->d_out_counts.p, n * 2);
  if (e == hipSuccess && n && left) e = h->d2h(left, h->d_out_left.p, n);
  if (e == hipSuccess && n && right) e = h->d2h(right, h->d_out_right.p, n);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  if (e != hipSuccess) return h->hip_fail(e, "fetch");
  return MHMKC_OK;
}

// The output rows ordered by the top 32 bits of mhmkc_map_hash, on the device (sorted once per finish, then kept for
// the range fetches).
int mhmkc::order_rows() {
  if (ord_ready) return MHMKC_OK;
  const uint64_t n = n_out;
  if (n >= 0xffffffffull) return fail(MHMKC_EUNSUPPORTED, "mhmkc_fetch_ordered: at most 2^32-1 rows");
  const size_t sb = mhm::map_order_scratch_bytes(n, nlo);
  const size_t ob = align_up(n * 8 * nlo + 64, 256) + align_up(n * 2 + 64, 256) + 2 * align_up(n + 64, 256);
  hipError_t e;
  // scratch and the ordered rows: the fine-record buffer of the finish (idle once the table is out, and larger
  // than both at every k: >= 4 B per counted occurrence against < 6 B per output row + the sort's 40-72 B), else
  // the handle's own buffers (a first hipMalloc of the sort's ~2 GB at C2 cost more than the sort)
  char *base = nullptr;
  if (d_r2.p && d_r2.cap >= sb + ob) {
    base = d_r2.as<char>();
  } else {
    if ((e = grow(d_ord, sb + ob)) != hipSuccess) return hip_fail(e, "fetch_ordered buffers");
    base = d_ord.as<char>();
  }
  char *ok = base + sb, *oc = ok + align_up(n * 8 * nlo + 64, 256), *ol = oc + align_up(n * 2 + 64, 256),
       *orr = ol + align_up(n + 64, 256);
  mhm::OutRows in{d_out_keys.as<uint64_t>(), d_out_counts.as<uint16_t>(), d_out_left.as<char>(), d_out_right.as<char>()};
  ord = mhm::OutRows{(uint64_t *)ok, (uint16_t *)oc, ol, orr};
  if (n && (e = mhm::launch_map_order(in, n, nlo, base, sb, ord, stream)) != hipSuccess)
    return hip_fail(e, "fetch_ordered sort");
  ord_ready = true;
  ord_scratch = base;
  ord_scratch_bytes = sb;
  map_cap = 0;
  return MHMKC_OK;
}

// The KmerMap slot and tag of every ordered row for a map of `cap` slots filled in this order from empty (a prefix
// maximum on the device, kcount_owner.hip k_map_slots), computed once per capacity.
int mhmkc::map_slots(uint64_t cap) {
  int rc = order_rows();
  if (rc) return rc;
  if (map_cap == cap) return MHMKC_OK;
  const uint64_t n = n_out;
  hipError_t e;
  if ((e = grow(d_mslot, n * 5 + 256)) != hipSuccess) return hip_fail(e, "map slots");
  // the scan runs in the ordering's scratch (>= 40 B per row, the scan needs 16 B per row + its own temporary)
  if (ord_scratch_bytes < mhm::map_slots_scratch_bytes(n)) return fail(MHMKC_EHIP, "internal: map slot scratch");
  uint32_t *slot = d_mslot.as<uint32_t>();
  uint8_t *tag = (uint8_t *)(slot + n);
  if (n && (e = mhm::launch_map_slots(ord.keys, n, nlo, cap, ord_scratch, ord_scratch_bytes, slot, tag, stream)) !=
               hipSuccess)
    return hip_fail(e, "map slots");
  map_cap = cap;
  return MHMKC_OK;
}

int mhmkc_fetch_ordered(mhmkc_t h, uint64_t *keys, uint16_t *counts, char *left, char *right) {
  if (!h) return MHMKC_EINVAL;
  return mhmkc_fetch_ordered_range(h, 0, h->finished ? h->n_out : 0, keys, counts, left, right);
}

int mhmkc_fetch_ordered_range(mhmkc_t h, uint64_t row0, uint64_t n_rows, uint64_t *keys, uint16_t *counts, char *left,
                              char *right) {
  if (!h) return MHMKC_EINVAL;
  if (!h->finished) return h->fail(MHMKC_ESTATE, "fetch before finish");
  if (row0 > h->n_out || n_rows > h->n_out - row0) return h->fail(MHMKC_EINVAL, "row range past the table's end");
  if (!n_rows) return MHMKC_OK;
  int rc = h->order_rows();
  if (rc) return rc;
  const int nlo = h->nlo;
  const mhm::OutRows &o = h->ord;
  hipError_t e = hipSuccess;
  if (keys) e = h->d2h(keys, o.keys + row0 * nlo, n_rows * 8 * nlo);
  if (e == hipSuccess && counts) e = h->d2h(counts, o.counts + row0, n_rows * 2);
  if (e == hipSuccess && left) e = h->d2h(left, o.left + row0, n_rows);
  if (e == hipSuccess && right) e = h->d2h(right, o.right + row0, n_rows);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  return e == hipSuccess ? MHMKC_OK : h->hip_fail(e, "fetch_ordered");
}

void *mhmkc_host_alloc(uint64_t bytes) {
  if (!bytes) bytes = 1;
  HostPool &hp = host_pool();
  {
    std::lock_guard<std::mutex> l(hp.mu);
    auto it = hp.free_.lower_bound(bytes);
    if (it != hp.free_.end() && it->first <= 2 * bytes) {
      void *p = it->second;
      hp.live[p] = it->first;
      hp.free_bytes -= it->first;
      hp.free_.erase(it);
      return p;
    }
  }
  void *p = nullptr;
  if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  std::lock_guard<std::mutex> l(hp.mu);
  hp.live[p] = bytes;
  return p;
}

void mhmkc_host_free(void *p) {
  if (!p) return;
  HostPool &hp = host_pool();
  std::lock_guard<std::mutex> l(hp.mu);
  auto it = hp.live.find(p);
  if (it == hp.live.end()) return;  // (not a block of mhmkc_host_alloc)
  const size_t b = it->second;
  hp.live.erase(it);
  if (hp.free_bytes + b <= HOST_POOL_KEEP) {
    hp.free_.emplace(b, p);
    hp.free_bytes += b;
  } else {
    (void)hipHostFree(p);
  }
}

int mhmkc_fetch_map_range(mhmkc_t h, uint64_t capacity, uint64_t row0, uint64_t n_rows, uint64_t *keys,
                          uint16_t *counts, char *left, char *right, uint32_t *slots, uint8_t *tags) {
  if (!h) return MHMKC_EINVAL;
  if (!h->finished) return h->fail(MHMKC_ESTATE, "fetch before finish");
  if (capacity < 16 || (capacity & (capacity - 1)) || capacity > (1ull << 32))
    return h->fail(MHMKC_EINVAL, "capacity must be a power of two in [16, 2^32]");
  if (row0 > h->n_out || n_rows > h->n_out - row0) return h->fail(MHMKC_EINVAL, "row range past the table's end");
  if (!n_rows) return MHMKC_OK;
  int rc = h->map_slots(capacity);
  if (rc) return rc;
  const uint32_t *slot = h->d_mslot.as<uint32_t>();
  const uint8_t *tag = (const uint8_t *)(slot + h->n_out);
  hipError_t e = hipSuccess;
  if (slots) e = h->d2h(slots, slot + row0, n_rows * 4);
  if (e == hipSuccess && tags) e = h->d2h(tags, tag + row0, n_rows);
  if (e != hipSuccess) return h->hip_fail(e, "fetch_map");
  return mhmkc_fetch_ordered_range(h, row0, n_rows, keys, counts, left, right);
}

int mhmkc_device_output(mhmkc_t h, const uint64_t **d_keys, const uint16_t **d_counts, const char **d_left,
                        const char **d_right, uint64_t *n_out) {
  if (!h) return MHMKC_EINVAL;
  if (!h->finished) return h->fail(MHMKC_ESTATE, "device_output before finish");
  if (d_keys) *d_keys = h->d_out_keys.as<uint64_t>();
  if (d_counts) *d_counts = h->d_out_counts.as<uint16_t>();
  if (d_left) *d_left = h->d_out_left.as<char>();
  if (d_right) *d_right = h->d_out_right.as<char>();
  if (n_out) *n_out = h->n_out;
  return MHMKC_OK;
}

int mhmkc_get_stats(mhmkc_t h, mhmkc_stats *s) {
  if (!h || !s) return MHMKC_EINVAL;
  *s = h->st;
  return MHMKC_OK;
}

int mhmkc_reset(mhmkc_t h) {
  if (!h) return MHMKC_EINVAL;
  hipError_t e = hipStreamSynchronize(h->stream);
  if (e == hipSuccess && h->xstream) e = hipStreamSynchronize(h->xstream);
  if (e == hipSuccess && h->pstream) e = hipStreamSynchronize(h->pstream);
  if (e != hipSuccess) return h->hip_fail(e, "reset");
  h->inc = h->inc_tried = false;
  h->inc_parted = 0;
  h->inc_expect = h->inc_announced = h->x_expect_all = h->x_r0_total = 0;
  h->x_r0_coarse.clear();
  h->x_round_slab.clear();
  h->lq = 0;
  h->inc_distinct = h->inc_ext_per_rec = 0;
  h->prof_collect();
  h->n_slabs = 0;
  h->n_parts = 0;
  h->xq = 0;
  h->x_rounds = 0;
  h->x_all_done = false;
  h->n_arenas = 0;
  h->ctg_bytes.clear();
  h->ctg_offs.assign(1, 0);
  h->ctg_win.assign(1, 0);
  h->ctg_depth.clear();
  h->ctg_n = 0;
  h->fq_reads = h->fq_bases = 0;
  h->finished = false;
  h->began = false;
  h->partial = false;
  h->n_out = 0;
  h->ord_ready = false;
  memset(&h->st, 0, sizeof h->st);
  if ((e = hipMemsetAsync(h->d_err.p, 0, 16, h->stream)) != hipSuccess) return h->hip_fail(e, "reset");
  return MHMKC_OK;
}

int mhmkc_set_profiling(mhmkc_t h, int on) {
  if (!h) return MHMKC_EINVAL;
  h->profiling = on != 0;
  h->prof_heavy_only = on == 2;
  return MHMKC_OK;
}

const char *mhmkc_last_error(mhmkc_t h) { return h ? h->err.c_str() : g_create_error.c_str(); }

int mhmkc_debug_set(const char *knob, int64_t value) {
  if (!knob) return MHMKC_EINVAL;
  const std::string k = knob;
  if (k == "exact") g_dbg.exact = value;
  else if (k == "cap") g_dbg.cap = value;
  else if (k == "fine_bits") g_dbg.fine_bits = value;
  else if (k == "out_cap") g_dbg.out_cap = value;
  else if (k == "fq_read_fail") g_dbg.fq_read_fail = value;
  else if (k == "wide_records") g_dbg.wide_records = value;
  else if (k == "smer") g_dbg.smer = value;
  else if (k == "chunk_bytes") g_dbg.chunk_bytes = value;
  else if (k == "d2h_chunk") g_dbg.d2h_chunk = value;
  else if (k == "h2d_nib") g_dbg.h2d_nib = value;
  else if (k == "local_rounds") g_dbg.local_rounds = value;
  else if (k == "h2d_threads") g_dbg.h2d_threads = value;
  else if (k == "h2d_nt") g_dbg.h2d_nt = value;
  else if (k == "h2d_adapt") g_dbg.h2d_adapt = value;
  else if (k == "cb0") g_dbg.cb0[1] = value;
  else if (k == "cb0_2") g_dbg.cb0[2] = value;
  else if (k == "cb0_3") g_dbg.cb0[3] = value;
  else return MHMKC_EINVAL;
  return MHMKC_OK;
}

void mhmkc_debug_reset(void) { g_dbg = DebugKnobs(); }

int mhmkc_debug_nib_pack(const uint8_t *src, uint64_t n, uint8_t *dst, int qcut, int mode) {
  if ((!src || !dst) && n) return MHMKC_EINVAL;
  if (mode == 0) {
    nib_pack(src, n, dst, qcut);
  } else if (mode == 1) {
    nib_pack_swar(src, n, dst, qcut);
  } else if (mode == 2) {
    if (!__builtin_cpu_supports("avx2")) return MHMKC_EUNSUPPORTED;
    nib_pack_avx2(src, n, dst, qcut, false);
  } else {
    return MHMKC_EINVAL;
  }
  return MHMKC_OK;
}

}  // extern "C"
