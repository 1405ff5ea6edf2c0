// Host side of libmhmkc: handle lifetime, device memory arena, stage orchestration, the RCCL
// exchange and the C ABI declared in include/mhmkc.h.
//
// One handle = one GPU = one rank. The reference's per-rank state (KmerDHT + HashTableInserter,
// src/kcount/kmer_dht.hpp:95-172) maps onto this struct; its UPC++ supermer store
// (src/kcount/kmer_dht.cpp:133-149,222-224) maps onto the hash-range exchange in exchange().
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mhmkc.h"
#include "kcount_launch.hpp"
#include "kmer_ops.hpp"

namespace {

thread_local std::string g_create_error;

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
    return hipSuccess;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T *as() const {
    return (T *)p;
  }
};

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Records of one add_reads batch, partitioned by coarse bucket (hash range). Every coarse bucket b is
// E_NSUB segments i = b * E_NSUB + s (one per group of blocks sharing an XCD in the capped layout; in
// the exact layout segment s = 0 holds the whole bucket and the others are empty). Segments are in
// bucket order, so a range of buckets is one contiguous span (with gaps in the capped layout).
constexpr uint32_t NSUB = mhm::E_NSUB;
struct Slab {
  DevBuf buf;
  mhm::PlaneSet planes{};
  uint64_t n = 0;
  std::vector<uint64_t> counts;  // [nb * NSUB]
  std::vector<uint64_t> bases;   // [nb * NSUB + 1] segment starts, bases[nb * NSUB] = end of the slab
};

// A source of owned records for the fine partition: per owned coarse bucket (local index) and segment.
struct Source {
  mhm::PlaneSet planes{};
  std::vector<uint64_t> start;  // [n_owned * NSUB]
  std::vector<uint64_t> count;  // [n_owned * NSUB]
};

struct Prof {
  int stage;
  hipEvent_t a, b;
};

}  // namespace

struct mhmkc {
  mhmkc_config cfg{};
  int k = 0, nl = 1, nlo = 1;
  bool packed = true;
  bool compact = false;  // compact records (kmer_ops.hpp cmix): 5 B per coarse record, 4 B per fine record
  int cb = 8, fb = 8, hbits = 0;
  uint32_t nb = 256, nf = 256;
  uint32_t own_lo = 0, own_hi = 256;  // owned coarse range [own_lo, own_hi)
  int dev = 0;
  int n_cu = 0;  // compute units: persistent k_count workgroups
  hipStream_t stream = nullptr;
  bool own_stream = false;
  ncclComm_t comm = nullptr;

  std::vector<Slab *> slabs;  // pool; first n_slabs are in use
  size_t n_slabs = 0;
  DevBuf d_hist, d_cursor, d_tiles, d_err, d_stats, d_fine_hist, d_fine_base, d_fine_cursor, d_chunks, d_srcs;
  DevBuf d_r2, d_out_keys, d_out_counts, d_out_left, d_out_right, d_out_cursor, d_recv, d_xcounts;
  DevBuf d_in_bytes, d_in_offs, d_hll;
  // FASTQ ingest (fastq.hip): text staging, chunk counts, newline positions, record lengths, scan scratch,
  // the packed reads of the last batch, first error
  DevBuf d_fq_text, d_fq_chunk, d_fq_lines, d_fq_len, d_fq_tmp, d_fq_bytes, d_fq_offs, d_fq_err;
  uint64_t fq_reads = 0, fq_bases = 0;
  int add_fastq(const char *d_text, uint64_t n);
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
  uint64_t n_out = 0;
  mhmkc_stats st{};
  bool profiling = false;
  std::vector<Prof> prof;
  std::vector<hipEvent_t> ev_pool;
  hipEvent_t ev_begin = nullptr, ev_end = nullptr;

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
  void prof_begin(int stage) {
    if (!profiling) return;
    Prof p{stage, take_event(), take_event()};
    (void)hipEventRecord(p.a, stream);
    prof.push_back(p);
  }
  void prof_end() {
    if (!profiling || prof.empty()) return;
    (void)hipEventRecord(prof.back().b, stream);
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
    return slabs[n_slabs++];
  }

  // Record planes for n records: NL u64 word planes (+ a byte plane when the ext code is not packed);
  // compact: a u32 plane (w[0]) + a byte plane for coarse-bucketed records, the u32 plane alone for fine.
  int set_planes(DevBuf &buf, uint64_t n, mhm::PlaneSet &ps, bool fine = false) {
    const uint64_t m = std::max<uint64_t>(n, 1);
    const size_t plane = align_up(m * (compact ? 4 : 8), 256);
    const size_t extb = (compact ? !fine : !packed) ? align_up(m, 256) : 0;
    const int np = compact ? 1 : nl;
    hipError_t e = buf.ensure(plane * np + extb);
    if (e != hipSuccess) return hip_fail(e, "allocating record planes");
    char *b = buf.as<char>();
    for (int w = 0; w < 4; w++) ps.w[w] = w < np ? (uint64_t *)(b + plane * w) : nullptr;
    ps.ext = extb ? (uint8_t *)(b + plane * np) : nullptr;
    return MHMKC_OK;
  }

  int add_device(const uint8_t *bytes, const uint64_t *offs, uint64_t n_reads, uint64_t n_bases, int qcut);
  int exchange(std::vector<Source> &srcs);
  int finish(uint64_t *n_out_ret);
};

// Fine partition target: distinct keys per fine bucket <= FINE_LOAD x LDS table slots.
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
// extract one batch of reads into a coarse-bucketed slab

// Coarse buckets are sized from the exact window count (+4 % and 4096 records of slack each), which lets
// one extract pass write the records. A bucket that would overflow (only skewed inputs: very repetitive
// reads) makes the pass redo itself with an exact histogram first (extract_hist).
int mhmkc::add_device(const uint8_t *bytes, const uint64_t *offs, uint64_t n_reads, uint64_t n_bases, int qcut) {
  int rc = begin_round();
  if (rc) return rc;
  st.reads += n_reads;
  st.bases += n_bases;
  if (n_reads == 0 || n_bases == 0) return MHMKC_OK;
  if (n_reads >= 0xffffffffull) return fail(MHMKC_EINVAL, "at most 2^32-2 reads per batch");
  const int T = mhm::tile_bases(nl);
  const uint64_t tiles64 = (n_bases + T - 1) / T;
  if (tiles64 >= 0x7fffffffull) return fail(MHMKC_EINVAL, "batch too large");
  const uint32_t tiles = (uint32_t)tiles64;
  hipError_t e;
  if ((e = d_tiles.ensure((size_t)tiles * 4)) != hipSuccess) return hip_fail(e, "tile index");
  if ((e = d_hist.ensure((size_t)nb * 8 + 8)) != hipSuccess) return hip_fail(e, "histogram");
  if ((e = d_cursor.ensure((size_t)nb * NSUB * mhm::CPAD * 8)) != hipSuccess) return hip_fail(e, "cursor");
  unsigned long long *d_wins = d_hist.as<unsigned long long>() + nb;

  mhm::ExtractParams p{};
  p.reads = {bytes, offs, n_reads, n_bases};
  p.tile_first_read = d_tiles.as<uint32_t>();
  p.n_tiles = tiles;
  p.k = k;
  p.qual_cutoff = qcut;
  p.coarse_bits = cb;
  p.n_bins = nb;
  p.hbits = hbits;
  p.compact = compact;
  p.hist = d_hist.as<unsigned long long>();
  p.cursor = d_cursor.as<unsigned long long>();
  p.err = d_err.as<unsigned int>();

  prof_begin(MHMKC_STAGE_TILEIDX);
  e = mhm::launch_tile_first_read(p.reads, d_tiles.as<uint32_t>(), tiles, T, stream);
  if (e == hipSuccess) e = hipMemsetAsync(d_wins, 0, 8, stream);
  if (e == hipSuccess) e = mhm::launch_count_windows(p.reads, k, d_wins, stream);
  prof_end();
  if (e != hipSuccess) return hip_fail(e, "tile index / window count");
  uint64_t wins = 0;
  if ((e = hipMemcpyAsync(&wins, d_wins, 8, hipMemcpyDeviceToHost, stream)) != hipSuccess)
    return hip_fail(e, "window count D2H");
  if ((e = hipStreamSynchronize(stream)) != hipSuccess) return hip_fail(e, "window count");
  if (wins == 0) return MHMKC_OK;

  Slab *sl = new_slab();
  const uint32_t nseg = nb * NSUB;
  sl->counts.assign(nseg, 0);
  sl->bases.assign(nseg + 1, 0);
  // device cursors are sub-major (cursor[s * nb + b]): the 64 lanes of one atomic instruction then hit 64
  // consecutive words, which the memory-side atomic unit serves as whole lines
  std::vector<uint64_t> cur((size_t)nseg), hist(nb);
  auto cidx = [&](uint32_t i) { return (size_t)(i % NSUB) * nb + i / NSUB; };
  const uint64_t expect = wins / nseg;
  const uint64_t cap = align_up(expect + expect / 25 + 1024, 64);
  bool exact = getenv("MHMKC_DEBUG_EXACT") != nullptr;  // tests only
  for (int attempt = 0; attempt < 2; attempt++) {
    if (exact) {
      prof_begin(MHMKC_STAGE_OTHER);
      e = hipMemsetAsync(d_hist.p, 0, (size_t)nb * 8, stream);
      prof_end();
      if (e != hipSuccess) return hip_fail(e, "memset");
      prof_begin(MHMKC_STAGE_EHIST);
      e = mhm::launch_extract_hist(p, nl, packed, stream);
      prof_end();
      if (e != hipSuccess) return hip_fail(e, "extract_hist");
      if ((e = hipMemcpyAsync(hist.data(), d_hist.p, (size_t)nb * 8, hipMemcpyDeviceToHost, stream)) != hipSuccess)
        return hip_fail(e, "histogram D2H");
      if ((e = hipStreamSynchronize(stream)) != hipSuccess) return hip_fail(e, "extract_hist");
      uint64_t tot = 0;
      for (uint32_t b = 0; b < nb; b++) {
        sl->bases[b * NSUB] = tot;
        tot += hist[b];
        for (uint32_t q = 1; q < NSUB; q++) sl->bases[b * NSUB + q] = tot;  // empty segments
      }
      sl->bases[nseg] = tot;
      p.bin_cap = 0;
    } else {
      for (uint32_t i = 0; i <= nseg; i++) sl->bases[i] = (uint64_t)i * cap;
      p.bin_cap = cap;
    }
    if ((rc = set_planes(sl->buf, sl->bases[nseg], sl->planes))) return rc;
    for (uint32_t i = 0; i < nseg; i++) cur[cidx(i)] = sl->bases[i];
    if ((e = hipMemcpyAsync(d_cursor.p, cur.data(), cur.size() * 8, hipMemcpyHostToDevice, stream)) != hipSuccess)
      return hip_fail(e, "cursor H2D");
    p.out = sl->planes;
    prof_begin(MHMKC_STAGE_ESCAT);
    e = mhm::launch_extract_scatter(p, nl, packed, stream);
    prof_end();
    if (e != hipSuccess) return hip_fail(e, "extract_scatter");
    unsigned int errf = 0;
    if ((e = hipMemcpyAsync(cur.data(), d_cursor.p, cur.size() * 8, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
        (e = hipMemcpyAsync(&errf, d_err.p, 4, hipMemcpyDeviceToHost, stream)) != hipSuccess)
      return hip_fail(e, "cursor D2H");
    if ((e = hipStreamSynchronize(stream)) != hipSuccess) return hip_fail(e, "extract_scatter");
    if (!(errf & 2u)) break;
    // a capped bucket overflowed: clear the flag (keep the bad-input bit) and redo with exact sizes
    errf &= ~2u;
    if ((e = hipMemcpy(d_err.p, &errf, 4, hipMemcpyHostToDevice)) != hipSuccess) return hip_fail(e, "flag reset");
    exact = true;
    st.exact_reruns++;
  }
  uint64_t tot = 0;
  for (uint32_t i = 0; i < nseg; i++) {
    sl->counts[i] = cur[cidx(i)] - sl->bases[i];
    tot += sl->counts[i];
  }
  sl->n = tot;
  st.occurrences += tot;
  return MHMKC_OK;
}

// ------------------------------------------------------------------------------------------------
// hash-range exchange between ranks (replaces the UPC++ ThreeTierAggrStore<Supermer> traffic,
// src/kcount/kmer_dht.cpp:133-149,222-224, and its flush/barrier, kmer_dht.cpp:227-231)

int mhmkc::exchange(std::vector<Source> &srcs) {
  const int G = cfg.n_ranks, me = cfg.rank;
  const uint32_t no = n_owned();
  hipError_t e;
  ncclResult_t nr;
  // 1. number of slabs of every rank
  uint64_t my_slabs = n_slabs;
  if ((e = d_xcounts.ensure(8 * (size_t)G * 2)) != hipSuccess) return hip_fail(e, "exchange counts");
  if ((e = hipMemcpyAsync(d_xcounts.p, &my_slabs, 8, hipMemcpyHostToDevice, stream)) != hipSuccess)
    return hip_fail(e, "exchange H2D");
  uint64_t *dx = d_xcounts.as<uint64_t>();
  if ((nr = ncclAllGather(dx, dx + G, 1, ncclUint64, comm, stream)) != ncclSuccess)
    return fail(MHMKC_ERCCL, "ncclAllGather: %s", ncclGetErrorString(nr));
  std::vector<uint64_t> slabs_of(G);
  if ((e = hipMemcpyAsync(slabs_of.data(), dx + G, 8 * (size_t)G, hipMemcpyDeviceToHost, stream)) != hipSuccess)
    return hip_fail(e, "exchange D2H");
  if ((e = hipStreamSynchronize(stream)) != hipSuccess) return hip_fail(e, "exchange sync");
  const uint64_t ms = std::max<uint64_t>(1, *std::max_element(slabs_of.begin(), slabs_of.end()));
  // 2. per slab: segment counts [nseg] and segment starts [nseg + 1] (capped slabs have gaps), of every rank
  const uint32_t nseg = nb * NSUB;
  const size_t per = 2 * (size_t)nseg + 1;
  std::vector<uint64_t> mine(ms * per, 0), all((size_t)G * ms * per, 0);
  for (size_t s = 0; s < n_slabs; s++) {
    std::copy(slabs[s]->counts.begin(), slabs[s]->counts.end(), mine.begin() + s * per);
    std::copy(slabs[s]->bases.begin(), slabs[s]->bases.end(), mine.begin() + s * per + nseg);
  }
  if ((e = d_xcounts.ensure(8 * (size_t)(G + 1) * ms * per)) != hipSuccess) return hip_fail(e, "exchange counts");
  dx = d_xcounts.as<uint64_t>();
  if ((e = hipMemcpyAsync(dx, mine.data(), 8 * ms * per, hipMemcpyHostToDevice, stream)) != hipSuccess)
    return hip_fail(e, "exchange H2D");
  if ((nr = ncclAllGather(dx, dx + ms * per, ms * per, ncclUint64, comm, stream)) != ncclSuccess)
    return fail(MHMKC_ERCCL, "ncclAllGather: %s", ncclGetErrorString(nr));
  if ((e = hipMemcpyAsync(all.data(), dx + ms * per, 8 * (size_t)G * ms * per, hipMemcpyDeviceToHost, stream)) !=
      hipSuccess)
    return hip_fail(e, "exchange D2H");
  if ((e = hipStreamSynchronize(stream)) != hipSuccess) return hip_fail(e, "exchange sync");
  auto cnt = [&](int r, uint64_t s, uint32_t i) { return all[((size_t)r * ms + s) * per + i]; };
  auto bas = [&](int r, uint64_t s, uint32_t i) { return all[((size_t)r * ms + s) * per + nseg + i]; };
  // 3. receive layout: for each peer p != me, for each of its slabs s, the span of my owned range
  uint64_t recv_total = 0;
  struct Seg {
    int peer;
    uint64_t slab, off, n;
  };
  std::vector<Seg> rsegs;
  for (int p = 0; p < G; p++) {
    if (p == me) continue;
    for (uint64_t s = 0; s < slabs_of[p]; s++) {
      const uint64_t n = bas(p, s, own_hi * NSUB) - bas(p, s, own_lo * NSUB);
      rsegs.push_back({p, s, recv_total, n});
      recv_total += n;
    }
  }
  mhm::PlaneSet rps{};
  int rc;
  if ((rc = set_planes(d_recv, recv_total, rps))) return rc;
  // 4. grouped send/recv (per pair the calls are issued in the same slab/plane order on both sides)
  prof_begin(MHMKC_STAGE_XCHG);
  if ((nr = ncclGroupStart()) != ncclSuccess) return fail(MHMKC_ERCCL, "ncclGroupStart: %s", ncclGetErrorString(nr));
  uint64_t sent = 0;
  for (int p = 0; p < G; p++) {
    if (p == me) continue;
    const uint32_t lo = owner_lo(p), hi = owner_lo(p + 1);
    for (size_t s = 0; s < n_slabs; s++) {
      const Slab *sl = slabs[s];
      const uint64_t a = sl->bases[lo * NSUB], b = sl->bases[hi * NSUB];
      if (b == a) continue;
      if (compact) {
        ncclSend((uint32_t *)sl->planes.w[0] + a, b - a, ncclUint32, p, comm, stream);
      } else {
        for (int w = 0; w < nl; w++) ncclSend(sl->planes.w[w] + a, b - a, ncclUint64, p, comm, stream);
      }
      if (sl->planes.ext) ncclSend(sl->planes.ext + a, b - a, ncclUint8, p, comm, stream);
      sent += (b - a) * rec_bytes();
    }
  }
  for (const Seg &g : rsegs) {
    if (!g.n) continue;
    if (compact) {
      ncclRecv((uint32_t *)rps.w[0] + g.off, g.n, ncclUint32, g.peer, comm, stream);
    } else {
      for (int w = 0; w < nl; w++) ncclRecv(rps.w[w] + g.off, g.n, ncclUint64, g.peer, comm, stream);
    }
    if (rps.ext) ncclRecv(rps.ext + g.off, g.n, ncclUint8, g.peer, comm, stream);
  }
  if ((nr = ncclGroupEnd()) != ncclSuccess) return fail(MHMKC_ERCCL, "ncclGroupEnd: %s", ncclGetErrorString(nr));
  prof_end();
  st.bytes_sent += sent;
  // 5. sources: local slabs (owned range in place) + received segments
  for (size_t s = 0; s < n_slabs; s++) {
    Source src;
    src.planes = slabs[s]->planes;
    src.start.assign(slabs[s]->bases.begin() + own_lo * NSUB, slabs[s]->bases.begin() + own_hi * NSUB);
    src.count.assign(slabs[s]->counts.begin() + own_lo * NSUB, slabs[s]->counts.begin() + own_hi * NSUB);
    srcs.push_back(std::move(src));
  }
  for (const Seg &g : rsegs) {
    Source src;
    src.planes = rps;
    src.start.resize((size_t)no * NSUB);
    src.count.resize((size_t)no * NSUB);
    for (uint32_t i = 0; i < no * NSUB; i++) {
      src.start[i] = g.off + (bas(g.peer, g.slab, own_lo * NSUB + i) - bas(g.peer, g.slab, own_lo * NSUB));
      src.count[i] = cnt(g.peer, g.slab, own_lo * NSUB + i);
    }
    srcs.push_back(std::move(src));
  }
  return MHMKC_OK;
}

// ------------------------------------------------------------------------------------------------
// contig pass: extract, fold and bucket the contig k-mers (kcount_ctg.hip); k_count applies them

int mhmkc::prepare_ctgs() {
  ctg_n = 0;
  const uint64_t W = ctg_win.back();
  if (!W) return MHMKC_OK;
  if (cfg.n_ranks > 1) return fail(MHMKC_EUNSUPPORTED, "the contig pass is single-rank in this version");
  hipError_t e;
  const uint64_t nc = ctg_depth.size();
  if ((e = d_ctg_bytes.ensure(ctg_bytes.size() + 64)) != hipSuccess ||
      (e = d_ctg_offs.ensure((nc + 1) * 8)) != hipSuccess || (e = d_ctg_win.ensure((nc + 1) * 8)) != hipSuccess ||
      (e = d_ctg_depth.ensure(nc * 2 + 2)) != hipSuccess)
    return hip_fail(e, "contig staging");
  if ((e = hipMemcpyAsync(d_ctg_bytes.p, ctg_bytes.data(), ctg_bytes.size(), hipMemcpyHostToDevice, stream)) !=
          hipSuccess ||
      (e = hipMemcpyAsync(d_ctg_offs.p, ctg_offs.data(), (nc + 1) * 8, hipMemcpyHostToDevice, stream)) != hipSuccess ||
      (e = hipMemcpyAsync(d_ctg_win.p, ctg_win.data(), (nc + 1) * 8, hipMemcpyHostToDevice, stream)) != hipSuccess ||
      (e = hipMemcpyAsync(d_ctg_depth.p, ctg_depth.data(), nc * 2, hipMemcpyHostToDevice, stream)) != hipSuccess)
    return hip_fail(e, "contig H2D");
  const size_t sb = mhm::ctg_scratch_bytes(W, nl);
  if ((e = d_ctg_scratch.ensure(sb)) != hipSuccess) return hip_fail(e, "contig scratch");
  uint64_t *keys[4] = {nullptr, nullptr, nullptr, nullptr};
  for (int w = 0; w < nl; w++) {
    if ((e = d_ctg_keys[w].ensure(W * 8)) != hipSuccess) return hip_fail(e, "contig keys");
    keys[w] = d_ctg_keys[w].as<uint64_t>();
  }
  if ((e = d_ctg_state.ensure(W * 4)) != hipSuccess || (e = d_ctg_bucket.ensure(W * 4)) != hipSuccess ||
      (e = d_ctg_done.ensure(W)) != hipSuccess)
    return hip_fail(e, "contig entries");
  mhm::CtgView cv{d_ctg_bytes.as<uint8_t>(), d_ctg_offs.as<uint64_t>(), d_ctg_depth.as<uint16_t>(),
                  d_ctg_win.as<uint64_t>(), nc, W};
  prof_begin(MHMKC_STAGE_OTHER);
  e = mhm::ctg_prepare(cv, k, nl, compact, 1, cfg.dmin_thres, 1.0 - cfg.dyn_min_depth, cb, fb, own_lo, d_ctg_scratch.p, sb, keys,
                       d_ctg_state.as<uint32_t>(), d_ctg_bucket.as<uint32_t>(), &ctg_n, d_err.as<unsigned int>(),
                       stream);
  prof_end();
  if (e != hipSuccess) return hip_fail(e, "contig pass");
  st.ctg_kmers = ctg_n;
  return MHMKC_OK;
}

// ------------------------------------------------------------------------------------------------
// fine partition + LDS count + finalize

// Fine buckets are capped at 1.25x their expected size (+256): a single scatter pass, no histogram. If a
// bucket overflows, the count kernel's results are discarded and the pass is redone with part_hist + scan.
int mhmkc::finish(uint64_t *n_out_ret) {
  int rc = begin_round();
  if (rc) return rc;
  hipError_t e;
  const uint32_t no = n_owned();
  std::vector<Source> srcs;
  if (cfg.n_ranks > 1) {
    if ((rc = exchange(srcs))) return rc;
  } else {
    for (size_t s = 0; s < n_slabs; s++) {
      Source src;
      src.planes = slabs[s]->planes;
      src.start.assign(slabs[s]->bases.begin(), slabs[s]->bases.begin() + (size_t)nb * NSUB);
      src.count = slabs[s]->counts;
      srcs.push_back(std::move(src));
    }
  }
  std::vector<uint64_t> per_coarse(no, 0);
  uint64_t owned = 0;
  for (auto &s : srcs)
    for (uint32_t i = 0; i < no * NSUB; i++) {
      per_coarse[i / NSUB] += s.count[i];
      owned += s.count[i];
    }
  st.owned_records = owned;
  st.coarse_record_bytes = rec_bytes();
  st.fine_record_bytes = compact ? 4 : rec_bytes();
  for (uint32_t c = 0; c < no; c++)  // k_count indexes a bucket with 32 bits
    if (per_coarse[c] >= 0xffffffffull)
      return fail(MHMKC_EUNSUPPORTED, "more than 2^32 records in one hash bucket (split the input into batches of ranks)");

  // run table: one entry per non-empty (source, segment) span; the device expands it into chunks
  const int T = mhm::tile_bases(nl);
  std::vector<mhm::SRun> runs;
  std::vector<mhm::PlaneSet> ps;
  uint64_t n_chunks = 0, n_c0 = 0;  // n_c0: chunks of the first owned coarse bucket (they come first)
  uint64_t xcd_start[9] = {0};
  for (size_t s = 0; s < srcs.size(); s++) ps.push_back(srcs[s].planes);
  // ordered by XCD class (coarse % 8), then coarse bucket, segment, source (see xcd_chunk)
  for (uint32_t x = 0; x < 8; x++) {
    xcd_start[x] = n_chunks;
    for (uint32_t c = x; c < no; c += 8) {
      for (uint32_t q = 0; q < NSUB; q++)
        for (size_t s = 0; s < srcs.size(); s++) {
          const uint32_t i = c * NSUB + q;
          const uint64_t cnt = srcs[s].count[i];
          if (!cnt) continue;
          runs.push_back({srcs[s].start[i], cnt, (uint32_t)s, c, (uint32_t)n_chunks, 0});
          n_chunks += (cnt + T - 1) / T;
        }
      if (c == 0) n_c0 = n_chunks;
    }
  }
  xcd_start[8] = n_chunks;
  if (n_chunks >= 0x7fffffffull) return fail(MHMKC_EINVAL, "too many chunks");
  uint64_t xcd_max = 0;
  for (int x = 0; x < 8; x++) xcd_max = std::max(xcd_max, xcd_start[x + 1] - xcd_start[x]);
  if ((e = d_chunks.ensure(std::max<size_t>(1, runs.size()) * sizeof(mhm::SRun) + 4 * (n_chunks + 1) + 256)) !=
      hipSuccess)
    return hip_fail(e, "chunk table");
  mhm::SRun *d_runs = d_chunks.as<mhm::SRun>();
  uint32_t *d_chunk_run = (uint32_t *)(d_chunks.as<char>() + align_up(runs.size() * sizeof(mhm::SRun), 256));
  if ((e = d_srcs.ensure(std::max<size_t>(1, ps.size()) * sizeof(mhm::PlaneSet) + 16 * (size_t)no)) != hipSuccess)
    return hip_fail(e, "source table");
  unsigned long long *d_cfit = (unsigned long long *)(d_srcs.as<char>() + align_up(ps.size() * sizeof(mhm::PlaneSet), 16));
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

  // fine bits: at most FINE_LOAD x the LDS table slots of distinct keys per fine bucket,
  // with the distinct keys of the first owned coarse bucket estimated by a HyperLogLog sketch (the ratio
  // of distinct keys to records grows with k and the error rate, so the record count alone misjudges it)
  const uint32_t cap_slots = (uint32_t)mhm::count_cap(nl, compact);
  fb = 4;
  if (n_c0) {
    mhm::PartitionParams sp{};
    sp.runs = d_runs;
    sp.chunk_run = d_chunk_run;
    sp.n_runs = (uint32_t)runs.size();
    sp.n_chunks = (uint32_t)n_chunks;
    sp.srcs = d_srcs.as<mhm::PlaneSet>();
    sp.k = k;
    sp.coarse_bits = cb;
    sp.hbits = hbits;
    sp.compact = compact;
    std::vector<uint32_t> reg(mhm::SKETCH_M);
    prof_begin(MHMKC_STAGE_OTHER);
    if ((e = d_hll.ensure(4 * mhm::SKETCH_M)) != hipSuccess ||
        (e = hipMemsetAsync(d_hll.p, 0, 4 * mhm::SKETCH_M, stream)) != hipSuccess ||
        (e = mhm::launch_sketch(sp, (uint32_t)n_c0, d_hll.as<unsigned int>(), nl, packed, stream)) != hipSuccess)
      return hip_fail(e, "distinct sketch");
    prof_end();
    if ((e = hipMemcpyAsync(reg.data(), d_hll.p, 4 * mhm::SKETCH_M, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
        (e = hipStreamSynchronize(stream)) != hipSuccess)
      return hip_fail(e, "sketch D2H");
    const double est = hll_estimate(reg);
    st.distinct_estimate = (uint64_t)(est * no);
    while (fb < 11 && est / (double)(1u << fb) > FINE_LOAD * cap_slots) fb++;
  } else {  // no records in the first coarse bucket: ~4 records per slot
    const uint64_t avg_coarse = owned / std::max<uint32_t>(no, 1);
    while (fb < 11 && (avg_coarse >> fb) > (uint64_t)cap_slots * 4) fb++;
  }
  if (const char *env = getenv("MHMKC_DEBUG_FINE_BITS")) fb = std::min(11, std::max(0, atoi(env)));  // tests only
  fb = std::max(fb, min_fine_bits());
  nf = 1u << fb;
  const uint32_t n_fine = no * nf;
  st.fine_buckets = n_fine;
  if ((rc = prepare_ctgs())) return rc;

  // capped fine layout
  std::vector<uint64_t> cfit(2 * (size_t)no);  // [coarse_base | coarse_fcap]
  uint64_t r2_size = 0;
  for (uint32_t c = 0; c < no; c++) {
    const uint64_t ex = per_coarse[c] >> fb;
    const uint64_t fcap = align_up(ex + ex / 4 + 256, 16);
    cfit[c] = r2_size;
    cfit[no + c] = fcap;
    r2_size += fcap << fb;
  }
  if (no && (e = hipMemcpyAsync(d_cfit, cfit.data(), 16 * (size_t)no, hipMemcpyHostToDevice, stream)) != hipSuccess)
    return hip_fail(e, "layout H2D");
  if ((e = d_fine_hist.ensure((size_t)n_fine * 8)) != hipSuccess) return hip_fail(e, "fine histogram");
  if ((e = d_fine_base.ensure((size_t)n_fine * 8)) != hipSuccess) return hip_fail(e, "fine bases");
  if ((e = d_fine_cursor.ensure((size_t)n_fine * 8)) != hipSuccess) return hip_fail(e, "fine cursor");
  const uint64_t out_cap = owned / 2 + ctg_n + 1;
  if ((e = d_out_keys.ensure(out_cap * 8 * nlo)) != hipSuccess) return hip_fail(e, "output keys");
  if ((e = d_out_counts.ensure(out_cap * 2)) != hipSuccess) return hip_fail(e, "output counts");
  if ((e = d_out_left.ensure(out_cap)) != hipSuccess) return hip_fail(e, "output left");
  if ((e = d_out_right.ensure(out_cap)) != hipSuccess) return hip_fail(e, "output right");
  if ((e = d_out_cursor.ensure(8)) != hipSuccess) return hip_fail(e, "output cursor");

  mhm::PartitionParams pp{};
  pp.runs = d_runs;
  pp.chunk_run = d_chunk_run;
  pp.n_runs = (uint32_t)runs.size();
  pp.n_chunks = (uint32_t)n_chunks;
  for (int x = 0; x < 9; x++) pp.xcd_start[x] = (uint32_t)xcd_start[x];
  pp.grid = (uint32_t)(8 * xcd_max);
  pp.srcs = d_srcs.as<mhm::PlaneSet>();
  pp.k = k;
  pp.coarse_bits = cb;
  pp.fine_bits = fb;
  pp.hbits = hbits;
  pp.compact = compact;
  pp.fine_hist = d_fine_hist.as<unsigned long long>();
  pp.fine_cursor = d_fine_cursor.as<unsigned long long>();
  pp.err = d_err.as<unsigned int>();

  mhm::CountParams cp{};
  cp.bucket_base = d_fine_base.as<unsigned long long>();
  cp.bucket_end = d_fine_cursor.as<unsigned long long>();
  cp.hbits = hbits;
  cp.compact = compact;
  cp.coarse_bits = cb;
  cp.fine_bits = fb;
  cp.bucket0 = own_lo << fb;
  cp.n_buckets = n_fine;
  cp.grid = (uint32_t)std::max(0, n_cu);  // one persistent workgroup per CU (k_count needs ~160 KB of LDS)
  cp.k = k;
  cp.cap = mhm::count_cap(nl, compact);
  if (const char *env = getenv("MHMKC_DEBUG_CAP")) cp.cap = std::min(cp.cap, std::max(64, atoi(env)) & ~3);  // tests only
  cp.dmin_thres = cfg.dmin_thres;
  cp.dyn_mult = 1.0 - cfg.dyn_min_depth;
  cp.nlo = nlo;
  cp.out_keys = d_out_keys.as<uint64_t>();
  cp.out_counts = d_out_counts.as<uint16_t>();
  cp.out_left = d_out_left.as<char>();
  cp.out_right = d_out_right.as<char>();
  cp.out_cursor = d_out_cursor.as<unsigned long long>();
  cp.stats = d_stats.as<unsigned long long>();
  cp.ctg_n = ctg_n;
  for (int w = 0; w < 4; w++) cp.ctg_keys[w] = w < nl ? d_ctg_keys[w].as<uint64_t>() : nullptr;
  cp.ctg_state = d_ctg_state.as<uint32_t>();
  cp.ctg_bucket = d_ctg_bucket.as<uint32_t>();
  cp.ctg_done = d_ctg_done.as<uint8_t>();

  bool exact = getenv("MHMKC_DEBUG_EXACT") != nullptr;  // tests only
  unsigned long long stats[mhm::STAT_ALLOC];
  unsigned int errf = 0;
  for (int attempt = 0; attempt < 2; attempt++) {
    mhm::PlaneSet r2{};
    prof_begin(MHMKC_STAGE_OTHER);
    e = hipMemsetAsync(d_out_cursor.p, 0, 8, stream);
    if (e == hipSuccess) e = hipMemsetAsync(d_stats.p, 0, 8 * mhm::STAT_ALLOC, stream);
    if (e == hipSuccess && ctg_n) e = hipMemsetAsync(d_ctg_done.p, 0, ctg_n, stream);
    if (e == hipSuccess && exact) e = hipMemsetAsync(d_fine_hist.p, 0, (size_t)n_fine * 8, stream);
    if (e == hipSuccess && !exact)
      e = mhm::launch_init_fine(d_cfit, d_cfit + no, no, fb, d_fine_base.as<unsigned long long>(),
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
      if ((rc = set_planes(d_r2, owned, r2, true))) return rc;
    } else {
      pp.coarse_base = d_cfit;
      pp.coarse_fcap = d_cfit + no;
      if ((rc = set_planes(d_r2, r2_size, r2, true))) return rc;
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
    if ((e = hipMemcpyAsync(stats, d_stats.p, sizeof stats, hipMemcpyDeviceToHost, stream)) != hipSuccess)
      return hip_fail(e, "stats D2H");
    if ((e = hipMemcpyAsync(&errf, d_err.p, 4, hipMemcpyDeviceToHost, stream)) != hipSuccess)
      return hip_fail(e, "error flag D2H");
    if ((e = hipStreamSynchronize(stream)) != hipSuccess) return hip_fail(e, "finish");
    if (!(errf & 2u)) break;
    errf &= ~2u;
    if ((e = hipMemcpy(d_err.p, &errf, 4, hipMemcpyHostToDevice)) != hipSuccess) return hip_fail(e, "flag reset");
    exact = true;
    st.exact_reruns++;
  }
  float ms = 0;
  if (hipEventElapsedTime(&ms, ev_begin, ev_end) == hipSuccess) st.ms_total = ms;
  prof_collect();
  finished = true;
  if (errf & 1u) return fail(MHMKC_EBADCHAR, "input byte with a base code > 4 (not A,C,G,T,N)");
  if (stats[mhm::STAT_N - 1]) return fail(MHMKC_EHIP, "internal: LDS probe bound exceeded");
  if (getenv("MHMKC_PRINT_STAMPS")) {  // k_count phase cycles of an MHMKC_STAMP build (diagnostics)
    const char *names[6] = {"clear", "loadwait", "insert", "barrier", "overflow", "finalize"};
    double tot = 0;
    for (int i = 0; i < 6; i++) tot += (double)stats[8 + i];
    fprintf(stderr, "k_count stamps:");
    for (int i = 0; i < 6; i++) fprintf(stderr, " %s %.1f%%", names[i], tot > 0 ? 100.0 * stats[8 + i] / tot : 0.0);
    fprintf(stderr, " (total %.3g wave-cycles)\n", tot);
  }
  st.distinct = stats[mhm::STAT_DISTINCT];
  st.n_out = stats[mhm::STAT_NOUT];
  st.purged = stats[mhm::STAT_PURGED];
  st.count_sum = stats[mhm::STAT_COUNTSUM];
  st.overflow_sweeps = stats[mhm::STAT_SWEEPS];
  st.max_bucket = stats[mhm::STAT_MAXBUCKET];
  st.dropped = 0;
  n_out = st.n_out;
  if (n_out > out_cap) return fail(MHMKC_EHIP, "internal: output overflow");
  if (n_out_ret) *n_out_ret = n_out;
  return MHMKC_OK;
}

// ------------------------------------------------------------------------------------------------
// C ABI

extern "C" {

int mhmkc_abi_version(void) { return MHMKC_ABI_VERSION; }

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
  // up to 8 ranks (one node): the coarse partition then has <= 2^11 bins, what a scatter workgroup keeps
  // in registers (scatter_staged)
  if (cfg->n_ranks < 1 || cfg->n_ranks > 8 || cfg->rank < 0 || cfg->rank >= cfg->n_ranks) {
    g_create_error = "bad rank / n_ranks (1..8 ranks, one per GPU of a node)";
    return MHMKC_EINVAL;
  }
  if (cfg->n_ranks > 1 && !cfg->comm_id) {
    g_create_error = "comm_id required when n_ranks > 1";
    return MHMKC_EINVAL;
  }
  mhmkc *h = new mhmkc();
  h->cfg = *cfg;
  h->k = k;
  h->nl = nl;
  h->nlo = nlo;
  h->packed = mhm::ext_packs(k, nl);
  h->hbits = mhm::stored_hash_bits(k, nl, h->packed);
  int extra = 0;
  while ((1 << extra) < cfg->n_ranks) extra++;
#ifndef MHMKC_CB0
#define MHMKC_CB0 8
#endif
  h->cb = MHMKC_CB0 + extra;
  // compact records for 10 <= k <= 21 (MHMKC_WIDE_RECORDS=1 keeps the 8-byte records: A/B and tests)
  const char *wide = getenv("MHMKC_WIDE_RECORDS");
  h->compact = mhm::compact_ok(k, nl) && 2 * k - h->cb <= 34 && !(wide && atoi(wide));
  if (h->compact) h->hbits = 0;
  h->nb = 1u << h->cb;
  h->own_lo = h->owner_lo(cfg->rank);
  h->own_hi = h->owner_lo(cfg->rank + 1);
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
  if ((e = hipEventCreate(&h->ev_begin)) != hipSuccess || (e = hipEventCreate(&h->ev_end)) != hipSuccess ||
      (e = h->d_err.ensure(16)) != hipSuccess || (e = h->d_stats.ensure(8 * mhm::STAT_ALLOC)) != hipSuccess ||
      (e = hipMemset(h->d_err.p, 0, 16)) != hipSuccess) {
    g_create_error = std::string("init: ") + hipGetErrorString(e);
    mhmkc_destroy(h);
    return MHMKC_EHIP;
  }
  if (cfg->n_ranks > 1) {
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
  if (h->comm) ncclCommDestroy(h->comm);
  for (Slab *s : h->slabs) {
    s->buf.release();
    delete s;
  }
  DevBuf *bufs[] = {&h->d_hist,     &h->d_cursor,    &h->d_tiles,     &h->d_err,       &h->d_stats,
                    &h->d_fine_hist, &h->d_fine_base, &h->d_fine_cursor, &h->d_chunks,  &h->d_srcs,
                    &h->d_r2,       &h->d_out_keys,  &h->d_out_counts, &h->d_out_left, &h->d_out_right,
                    &h->d_out_cursor, &h->d_recv,    &h->d_xcounts,   &h->d_in_bytes,  &h->d_in_offs,
                    &h->d_hll,       &h->d_fq_text,   &h->d_fq_chunk,  &h->d_fq_lines,  &h->d_fq_len,
                    &h->d_fq_tmp,    &h->d_fq_bytes,  &h->d_fq_offs,   &h->d_fq_err};
  for (DevBuf *b : bufs) b->release();
  DevBuf *cbufs[] = {&h->d_ctg_bytes, &h->d_ctg_offs, &h->d_ctg_win,   &h->d_ctg_depth, &h->d_ctg_scratch,
                     &h->d_ctg_state, &h->d_ctg_bucket, &h->d_ctg_done, &h->d_ctg_keys[0], &h->d_ctg_keys[1],
                     &h->d_ctg_keys[2], &h->d_ctg_keys[3]};
  for (DevBuf *b : cbufs) b->release();
  for (auto &p : h->prof) {
    h->ev_pool.push_back(p.a);
    h->ev_pool.push_back(p.b);
  }
  for (hipEvent_t ev : h->ev_pool) (void)hipEventDestroy(ev);
  if (h->ev_begin) (void)hipEventDestroy(h->ev_begin);
  if (h->ev_end) (void)hipEventDestroy(h->ev_end);
  if (h->own_stream && h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
}

int mhmkc_add_reads_device(mhmkc_t h, const uint8_t *d_bytes, const uint64_t *d_offs, uint64_t n_reads,
                           uint64_t n_bases) {
  if (!h) return MHMKC_EINVAL;
  if (n_reads && (!d_bytes || !d_offs)) return h->fail(MHMKC_EINVAL, "null device buffer");
  return h->add_device(d_bytes, d_offs, n_reads, n_bases, h->cfg.qual_cutoff);
}

// FASTQ text on the device -> PackedReads in d_fq_bytes / d_fq_offs -> add_device (fastq.hip).
int mhmkc::add_fastq(const char *d_text, uint64_t n) {
  int rc = begin_round();
  if (rc) return rc;
  fq_reads = fq_bases = 0;
  if (n == 0) return MHMKC_OK;
  if (n > mhm::FQ_LE_MASK) return fail(MHMKC_EINVAL, "FASTQ text larger than 2^40 bytes in one call");
  hipError_t e;
  const uint64_t nch = (n + mhm::FQ_CHUNK - 1) / mhm::FQ_CHUNK;
  if ((e = d_fq_chunk.ensure((nch + 1) * 16)) != hipSuccess) return hip_fail(e, "fastq chunk counts");
  unsigned long long *cnt = d_fq_chunk.as<unsigned long long>(), *cbase = cnt + nch + 1;
  size_t tmp_bytes = mhm::fq_scan_tmp_bytes(nch + 1);
  if ((e = d_fq_tmp.ensure(tmp_bytes)) != hipSuccess) return hip_fail(e, "fastq scan scratch");
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
  // fgets returns a last line without its newline
  const uint64_t lines = newlines + (last != '\n' ? 1 : 0);
  const uint64_t R = lines / 4;
  if ((e = d_fq_lines.ensure(std::max<uint64_t>(lines, 1) * 8)) != hipSuccess) return hip_fail(e, "fastq lines");
  if ((e = d_fq_len.ensure((R + 1) * 8)) != hipSuccess || (e = d_fq_offs.ensure((R + 1) * 8)) != hipSuccess ||
      (e = d_fq_err.ensure(8)) != hipSuccess)
    return hip_fail(e, "fastq records");
  const size_t tmp2 = mhm::fq_scan_tmp_bytes(R + 1);
  if (tmp2 > tmp_bytes) {
    if ((e = d_fq_tmp.ensure(tmp2)) != hipSuccess) return hip_fail(e, "fastq scan scratch");
    tmp_bytes = tmp2;
  }
  unsigned long long *lend = d_fq_lines.as<unsigned long long>(), *len = d_fq_len.as<unsigned long long>();
  unsigned long long *offs = d_fq_offs.as<unsigned long long>(), *err_d = d_fq_err.as<unsigned long long>();
  const unsigned long long n_end = n;
  prof_begin(MHMKC_STAGE_OTHER);
  e = mhm::launch_fq_lines(d_text, n, cbase, lend, stream);
  if (e == hipSuccess && last != '\n') e = hipMemcpyAsync(lend + lines - 1, &n_end, 8, hipMemcpyHostToDevice, stream);
  if (e == hipSuccess) e = hipMemsetAsync(err_d, 0xff, 8, stream);
  if (e == hipSuccess) e = mhm::launch_fq_records(d_text, n, lend, R, len, err_d, stream);
  if (e == hipSuccess) e = mhm::fq_scan(d_fq_tmp.p, tmp_bytes, len, offs, R + 1, stream);
  prof_end();
  if (e != hipSuccess) return hip_fail(e, "fastq records");
  unsigned long long n_bases = 0;
  if ((e = hipMemcpyAsync(&n_bases, offs + R, 8, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
      (e = hipStreamSynchronize(stream)) != hipSuccess)
    return hip_fail(e, "fastq records D2H");
  if ((e = d_fq_bytes.ensure(std::max<uint64_t>(n_bases, 1) + 64)) != hipSuccess) return hip_fail(e, "fastq bytes");
  prof_begin(MHMKC_STAGE_OTHER);
  e = mhm::launch_fq_pack(d_text, lend, R, offs, cfg.qual_offset, d_fq_bytes.as<uint8_t>(), err_d, stream);
  prof_end();
  unsigned long long first_err = ~0ull;
  if (e == hipSuccess) e = hipMemcpyAsync(&first_err, err_d, 8, hipMemcpyDeviceToHost, stream);
  if (e == hipSuccess) e = hipStreamSynchronize(stream);
  if (e != hipSuccess) return hip_fail(e, "fastq pack");
  if (lines % 4) first_err = std::min<unsigned long long>(first_err, ((unsigned long long)R << 4) | mhm::FQ_E_TRUNC);
  if (first_err != ~0ull) {
    const unsigned long long rec = first_err >> 4;
    switch ((int)(first_err & 15)) {
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
  fq_reads = R;
  fq_bases = n_bases;
  return add_device(d_fq_bytes.as<uint8_t>(), d_fq_offs.as<uint64_t>(), R, n_bases, cfg.qual_cutoff);
}

static int add_host(mhmkc_t h, const uint8_t *bytes, const uint64_t *offs, uint64_t n_reads, int qcut) {
  const uint64_t n_bases = offs[n_reads];
  hipError_t e;
  if ((e = h->d_in_bytes.ensure(std::max<uint64_t>(n_bases, 1) + 64)) != hipSuccess)
    return h->hip_fail(e, "input staging");
  if ((e = h->d_in_offs.ensure((n_reads + 1) * 8)) != hipSuccess) return h->hip_fail(e, "input staging");
  if (n_bases && (e = hipMemcpyAsync(h->d_in_bytes.p, bytes, n_bases, hipMemcpyHostToDevice, h->stream)) != hipSuccess)
    return h->hip_fail(e, "input H2D");
  if ((e = hipMemcpyAsync(h->d_in_offs.p, offs, (n_reads + 1) * 8, hipMemcpyHostToDevice, h->stream)) != hipSuccess)
    return h->hip_fail(e, "input H2D");
  int rc = h->add_device(h->d_in_bytes.as<uint8_t>(), h->d_in_offs.as<uint64_t>(), n_reads, n_bases, qcut);
  if (rc == MHMKC_OK) {
    if ((e = hipStreamSynchronize(h->stream)) != hipSuccess) return h->hip_fail(e, "add_reads");
  }
  return rc;
}

static int check_offsets(mhmkc_t h, const uint64_t *offs, uint64_t n_reads) {
  if (offs[0] != 0) return h->fail(MHMKC_EINVAL, "read_offsets[0] must be 0");
  for (uint64_t i = 0; i < n_reads; i++) {
    if (offs[i + 1] < offs[i]) return h->fail(MHMKC_EINVAL, "read_offsets must be non-decreasing (read %llu)",
                                              (unsigned long long)i);
    if (offs[i + 1] - offs[i] > 65535)
      return h->fail(MHMKC_EINVAL, "read %llu longer than 65535 (PackedRead read_len is uint16)",
                     (unsigned long long)i);
  }
  return MHMKC_OK;
}

int mhmkc_add_reads(mhmkc_t h, const uint8_t *bytes, const uint64_t *offs, uint64_t n_reads) {
  if (!h) return MHMKC_EINVAL;
  if (!offs || (n_reads && !bytes)) return h->fail(MHMKC_EINVAL, "null host buffer");
  int rc = check_offsets(h, offs, n_reads);
  if (rc) return rc;
  return add_host(h, bytes, offs, n_reads, h->cfg.qual_cutoff);
}

int mhmkc_add_fastq_device(mhmkc_t h, const char *d_text, uint64_t n_bytes) {
  if (!h) return MHMKC_EINVAL;
  if (n_bytes && !d_text) return h->fail(MHMKC_EINVAL, "null device buffer");
  return h->add_fastq(d_text, n_bytes);
}

int mhmkc_add_fastq(mhmkc_t h, const char *text, uint64_t n_bytes) {
  if (!h) return MHMKC_EINVAL;
  if (n_bytes && !text) return h->fail(MHMKC_EINVAL, "null host buffer");
  hipError_t e;
  if ((e = h->d_fq_text.ensure(n_bytes + 16)) != hipSuccess) return h->hip_fail(e, "fastq staging");
  if (n_bytes && (e = hipMemcpyAsync(h->d_fq_text.p, text, n_bytes, hipMemcpyHostToDevice, h->stream)) != hipSuccess)
    return h->hip_fail(e, "fastq H2D");
  int rc = h->add_fastq(h->d_fq_text.as<char>(), n_bytes);
  if (rc == MHMKC_OK && (e = hipStreamSynchronize(h->stream)) != hipSuccess) return h->hip_fail(e, "add_fastq");
  return rc;
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

int mhmkc_add_seqs(mhmkc_t h, const char *seqs, const uint64_t *offs, uint64_t n_seqs, uint16_t depth) {
  if (!h) return MHMKC_EINVAL;
  if (!offs || (n_seqs && !seqs)) return h->fail(MHMKC_EINVAL, "null host buffer");
  if (depth > 1) return h->fail(MHMKC_EUNSUPPORTED, "contig pass (depth > 1) is not supported in this version");
  if (offs[0] != 0) return h->fail(MHMKC_EINVAL, "seq_offsets[0] must be 0");
  for (uint64_t i = 0; i < n_seqs; i++)
    if (offs[i + 1] < offs[i]) return h->fail(MHMKC_EINVAL, "seq_offsets must be non-decreasing");
  const uint64_t n = offs[n_seqs];
  // Case carries the quality (SeqBlockInserter::process_seq input, src/kcount/kcount.cpp:80-86;
  // quals[i] = isupper, src/kcount/kcount_cpu.cpp:309-312): uppercase -> q 31, lowercase -> q 0, and the
  // batch runs with cutoff 1. Characters other than ACGTN are fatal in the reference
  // (HashTableInserter::insert_supermer DIE, src/kcount/kcount_cpu.cpp:452-458).
  std::vector<uint8_t> bytes(n);
  for (uint64_t i = 0; i < n; i++) {
    const char c = seqs[i];
    uint8_t code;
    switch (c) {
      case 'A': case 'a': code = 0; break;
      case 'C': case 'c': code = 1; break;
      case 'G': case 'g': code = 2; break;
      case 'T': case 't': code = 3; break;
      case 'N': case 'n': code = 4; break;
      default:
        return h->fail(MHMKC_EBADCHAR, "bad char '%c' (%d) at position %llu", c, (int)c, (unsigned long long)i);
    }
    const bool upper = (c >= 'A' && c <= 'Z');
    bytes[i] = (uint8_t)(code | (upper ? (31u << 3) : 0u));
  }
  return add_host(h, bytes.data(), offs, n_seqs, 1);
}

int mhmkc_add_ctgs(mhmkc_t h, const char *seqs, const uint64_t *offs, const uint16_t *depths, uint64_t n_ctgs) {
  if (!h) return MHMKC_EINVAL;
  if (!offs || (n_ctgs && (!seqs || !depths))) return h->fail(MHMKC_EINVAL, "null host buffer");
  if (h->finished) return h->fail(MHMKC_ESTATE, "handle already finished; call mhmkc_reset first");
  if (offs[0] != 0) return h->fail(MHMKC_EINVAL, "seq_offsets[0] must be 0");
  for (uint64_t i = 0; i < n_ctgs; i++)
    if (offs[i + 1] < offs[i]) return h->fail(MHMKC_EINVAL, "seq_offsets must be non-decreasing");
  const uint64_t n = offs[n_ctgs];
  const size_t b0 = h->ctg_bytes.size();
  h->ctg_bytes.resize(b0 + n);
  // case carries the quality as for reads (get_kmers_and_exts: quals[i] = isupper, kcount_cpu.cpp:309-313);
  // contigs are uppercase. Characters other than ACGTN are fatal (insert_supermer DIE, :452-458).
  for (uint64_t i = 0; i < n; i++) {
    const char c = seqs[i];
    uint8_t code;
    switch (c) {
      case 'A': case 'a': code = 0; break;
      case 'C': case 'c': code = 1; break;
      case 'G': case 'g': code = 2; break;
      case 'T': case 't': code = 3; break;
      case 'N': case 'n': code = 4; break;
      default:
        h->ctg_bytes.resize(b0);
        return h->fail(MHMKC_EBADCHAR, "bad char '%c' (%d) in contig position %llu", c, (int)c, (unsigned long long)i);
    }
    h->ctg_bytes[b0 + i] = (uint8_t)(code | ((c >= 'A' && c <= 'Z') ? (31u << 3) : 0u));
  }
  const uint64_t k = (uint64_t)h->k;
  for (uint64_t i = 0; i < n_ctgs; i++) {
    const uint64_t L = offs[i + 1] - offs[i];
    h->ctg_offs.push_back(b0 + offs[i + 1]);
    // add_ctg_kmers skips contigs shorter than k + 2 (src/kcount/kcount.cpp:128); interior windows only
    h->ctg_win.push_back(h->ctg_win.back() + (L >= k + 2 ? L - k - 1 : 0));
    h->ctg_depth.push_back(depths[i]);
  }
  if (h->ctg_win.back() >= 0xffffffffull) return h->fail(MHMKC_EINVAL, "at most 2^32-1 contig k-mers per round");
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
  if (n && keys) e = hipMemcpyAsync(keys, h->d_out_keys.p, n * 8 * h->nlo, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess && n && counts) e = hipMemcpyAsync(counts, h->d_out_counts.p, n * 2, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess && n && left) e = hipMemcpyAsync(left, h->d_out_left.p, n, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess && n && right) e = hipMemcpyAsync(right, h->d_out_right.p, n, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  if (e != hipSuccess) return h->hip_fail(e, "fetch");
  return MHMKC_OK;
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
  if (e != hipSuccess) return h->hip_fail(e, "reset");
  h->prof_collect();
  h->n_slabs = 0;
  h->ctg_bytes.clear();
  h->ctg_offs.assign(1, 0);
  h->ctg_win.assign(1, 0);
  h->ctg_depth.clear();
  h->ctg_n = 0;
  h->fq_reads = h->fq_bases = 0;
  h->finished = false;
  h->began = false;
  h->n_out = 0;
  memset(&h->st, 0, sizeof h->st);
  if ((e = hipMemsetAsync(h->d_err.p, 0, 16, h->stream)) != hipSuccess) return h->hip_fail(e, "reset");
  return MHMKC_OK;
}

int mhmkc_set_profiling(mhmkc_t h, int on) {
  if (!h) return MHMKC_EINVAL;
  h->profiling = on != 0;
  return MHMKC_OK;
}

const char *mhmkc_last_error(mhmkc_t h) { return h ? h->err.c_str() : g_create_error.c_str(); }

}  // extern "C"
