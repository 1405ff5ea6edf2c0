// Launch interface between the host orchestration (mhmkc_host.cpp) and the gfx950 kernels
// (kcount_kernels.hip). Plain structs of device pointers; no torch types anywhere.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mhm {

// Read stream in the PackedRead byte layout (src/packed_reads.cpp:73-109) + CSR offsets.
// A view may be a slice of a larger batch (one H2D chunk, mhmkc_add_reads): its offsets are then the
// batch's, and obase (<= offs[0], 16-byte aligned in the batch) is subtracted from them; bytes points
// at batch byte obase. Positions [0, head) belong to the previous slice's last read and hold no window.
struct ReadsView {
  const uint8_t *bytes;   // n_bases bytes: code (bits 0-2) | min(q-off,31) << 3
  const uint64_t *offs;   // n_reads+1 offsets, offs[n_reads] - obase = n_bases
  uint64_t n_reads;
  uint64_t n_bases;
  uint64_t obase;         // subtracted from every offset (0 for a whole batch)
  uint32_t head;          // offs[0] - obase (< 16)
  uint32_t pad;
};

// Record planes of one slab: word planes (SoA) + optional ext byte plane.
struct PlaneSet {
  uint64_t *w[4];
  uint8_t *ext;  // nullptr when the ext code is packed into the last key word
};

struct ExtractParams {
  ReadsView reads;
  const uint32_t *tile_first_read;  // per tile: first read r with offs[r] >= tile_lo
  uint32_t n_tiles;
  int k;
  int qual_cutoff;
  int coarse_bits;                  // coarse digit = h1 >> (64 - coarse_bits)
  uint32_t n_bins;                  // 1 << coarse_bits
  int hbits;                        // hash bits stored in the record after the ext code (0: none)
  int compact;                      // mixed records: compact (NL = 1, kmer_ops.hpp cmix): out = u32 plane w[0] +
                                    // byte plane ext; NL = 2: m2_mix records, two u64 planes
  unsigned long long *hist;         // [n_bins] (E-hist)
  unsigned long long *cursor;       // [E_NSUB * n_bins] (E-scatter): cursor of segment (b, s) at s * n_bins + b
  uint64_t bin_cap;                 // capped mode: segment (b, s) owns [i*bin_cap, (i+1)*bin_cap), i = b*E_NSUB+s,
                                    // s = blockIdx % E_NSUB; 0 = exact bases, everything in segment (b, 0)
  PlaneSet out;                     // (E-scatter)
  unsigned int *err;                // bit 0: input byte with code > 4
  unsigned int *ovf;                // bit 1: a capped bin of this slab overflowed (per slab)
  const uint32_t *tile_starts;      // the batch's flat read-start bits (k_read_start_bits; tile t's groups are words
                                    // [t tile / 32, t tile / 32 + kGroups)), or nullptr:
                                    // load_tile builds it from the offsets
  uint32_t bin_lo, bin_hi;          // k_smer_extract: only records of coarse bins [bin_lo, bin_hi) are kept (a finish
                                    // pass over part of the hash range); 0, n_bins = all
};

constexpr int SMER_SLICES = 64;  // counter slices per destination (spread the workgroups' atomics)
// Supermer exchange (kcount_kernels.hip). Sender side, per read slab: owners and per-destination
// counts (k_smer_owner), then the supermers packed into exact per-destination spans (k_smer_pack).
struct SmerParams {
  ReadsView reads;
  const uint32_t *tile_first_read;
  uint32_t n_tiles;
  int k, m, n_ranks, qual_cutoff;
  uint8_t *owners;              // [n_tiles * tile]: owner of the window at each tile position, 0xFF: not counted
  unsigned long long *hist;     // [n_ranks][SMER_SLICES][2]: words, supermers per destination and slice of tiles
                                // (tile % SMER_SLICES; k_smer_owner adds)
  unsigned long long *cursor;   // the same layout: word and supermer cursors (k_smer_pack)
  uint64_t *codes;              // supermer bases, 2-bit codes, 32 per word (MSB first)
  uint32_t *good;               // their "extension countable" bits, 32 per word
  uint64_t *desc;               // per supermer: first word << 16 | windows
  uint64_t n_words, n_smer;     // the planes' sizes (k_smer_pack writes nothing past them: err bit 3)
  unsigned int *err;
};
// Receiver side: the received supermers of every peer back to back (descriptors rebased), their window prefix
// wpre[n_smer + 1], and per tile of window indices the supermer holding its first window.
struct SmerSource {
  const uint64_t *codes;
  const uint32_t *good;
  const uint64_t *desc;
  const uint64_t *wpre;
  const uint64_t *tile_first;   // [n_tiles + 1]
  uint64_t n_smer, n_windows;
  uint64_t n_words;             // code / good words (a window reaching past them is not read: err bit 3)
};
hipError_t launch_smer_owner(const SmerParams &p, int nl, hipStream_t s);
hipError_t launch_smer_pack(const SmerParams &p, int nl, hipStream_t s);
// records of the received supermers into a coarse slab (p.out / p.cursor as launch_extract_scatter), or (hist) the
// exact bin histogram into p.hist
hipError_t launch_smer_extract(const ExtractParams &p, const SmerSource &src, int nl, bool packed, bool hist,
                               hipStream_t s);
// descriptors of a received span: word offsets += delta (mod 2^64), nwin[i] = windows of supermer i
hipError_t launch_smer_rebase(uint64_t *desc, uint64_t n, uint64_t delta, unsigned long long *nwin, hipStream_t s);
hipError_t launch_smer_tiles(const uint64_t *wpre, uint64_t n_smer, uint64_t *tile_first, uint32_t n_tiles, int tile,
                             hipStream_t s);

// One chunk of S work: <= tile records of one (source, coarse bucket) segment.
struct SChunk {
  uint64_t start;        // first record index in the source planes
  uint32_t count;        // records in the chunk
  uint32_t src;          // index into the source plane-set table
  uint32_t coarse_local; // coarse bucket index relative to this rank's first owned bucket
  uint32_t pad;
};

// A run = one non-empty (source, segment) span, cut into tile-sized chunks; chunk0 = its first chunk.
struct SRun {
  uint64_t start, count;
  uint32_t src, coarse_local;
  uint32_t chunk0, pad;
};

struct PartitionParams {
  const SRun *runs;                 // [n_runs]
  const SChunk *chunks;             // [n_chunks]: each chunk's span (launch_chunk_runs expands the runs into them)
  uint32_t n_runs;
  uint32_t n_chunks;
  // XCD-aware launch: the chunks are ordered by XCD class (coarse bucket % 8); class x holds chunks
  // [xcd_start[x], xcd_start[x + 1]) and is served by the workgroups b with b % 8 == x (grid = 8 * largest)
  uint32_t xcd_start[9];
  uint32_t grid;
  const PlaneSet *srcs;           // device table of source plane sets
  int k;
  int coarse_bits;
  int fine_bits;
  int hbits;                        // hash bits stored in the records (fine digit read from them if >= fine_bits)
  int compact;                      // mixed records (see ExtractParams): compact sources u32 + byte planes, out
                                    // one u32 plane; NL = 2: two u64 planes in and out
  unsigned long long *fine_hist;    // [n_coarse_local << fine_bits]
  unsigned long long *fine_cursor;  // [n_coarse_local << fine_bits]
  const unsigned long long *coarse_base;  // capped mode: first fine bucket of coarse bucket c starts here
  const unsigned long long *coarse_fcap;  // capped mode: capacity of every fine bucket of c; nullptr = exact
  unsigned int *err;                      // bit 1: a capped fine bucket overflowed
  PlaneSet out;
};

struct CountParams {
  PlaneSet recs;                      // fine-bucketed records (overwritten in place by overflow)
  const unsigned long long *bucket_base;
  const unsigned long long *bucket_end;  // == the fine cursors after the scatter
  int hbits;                           // stored hash bits to strip from the last key word
  int compact;                         // mixed records (compact u32 plane w[0], or NL = 2 m2_mix words); the key
                                       // is rebuilt from the bucket digits
  int coarse_bits, fine_bits;
  uint32_t bucket0;                    // global index of local fine bucket 0 (own_lo << fine_bits)
  uint32_t n_buckets;
  uint32_t grid;                      // persistent workgroups (one per CU); 0 = one per bucket
  int k;
  int cap;                            // LDS table slots
  int dmin_thres;
  double dyn_mult;                    // 1.0 - DYN_MIN_DEPTH, computed in double on the host
  int nlo;                            // output words per key
  uint64_t *out_keys;                 // [out_cap * nlo]
  uint16_t *out_counts;
  char *out_left;
  char *out_right;
  unsigned long long *out_cursor;
  unsigned long long out_cap;         // output rows allocated: a reservation past it sets err bit 4 (16) and writes
                                      // nothing (the cursor still counts, so the host learns the size and redoes the pass)
  unsigned long long *stats;          // [STAT_*]
  unsigned int *err;                  // k_part_scatter's flag word: bit 1 set = a capped fine bucket overflowed,
                                      // its cursor ran past the bucket, so the launch is void (returns at once)
  // contig pass (kcount_ctg.hip): folded contig k-mers sorted by bucket; 0 entries = no contig pass
  uint64_t ctg_n;
  const uint64_t *ctg_keys[4];        // [NL][ctg_n] canonical key words
  const uint32_t *ctg_state;          // count (16 bits) | left code << 16 | right code << 19
  const uint32_t *ctg_bucket;         // local fine bucket of each entry (sorted ascending)
  uint32_t ctg_base;                  // local fine bucket of this launch's bucket 0 (a finish pass over part of the
                                      // owned range: its first coarse bucket << fine_bits)
  PlaneSet spill;                     // deferred records of cold sweeps: SPILL_RECORDS per workgroup (fine record
                                      // layout; planes of grid * SPILL_RECORDS entries); w[0] == nullptr: none
  uint8_t *ctg_done;                  // [ctg_n] applied (zeroed before the launch)
  const uint8_t *coarse_skip;         // [n_buckets >> fine_bits] or null: a local coarse bucket whose fine buckets are
                                      // counted by a later launch (k_inc_fixup emptied them): no contig k-mers here
};

// Contig pass state word of one folded contig k-mer (kcount_ctg.hip).
__host__ __device__ inline uint32_t ctg_state_word(uint32_t count, uint32_t l, uint32_t r) {
  return (count & 0xffffu) | (l << 16) | (r << 19);
}

// Input of the contig-pass extraction: contigs in the PackedRead byte layout (case -> quality 31 / 0).
struct CtgView {
  const uint8_t *bytes;
  const uint64_t *offs;        // [n_ctgs + 1]
  const uint16_t *depth;       // [n_ctgs]: Contig::get_uint16_t_depth() (0 counts as 1)
  const uint64_t *win_prefix;  // [n_ctgs + 1]: counted windows before each contig
  uint64_t n_ctgs;
  uint64_t n_windows;
};

// Owner filter of the contig pass with the supermer exchange: keep the k-mers whose get_kmer_target_rank
// (quick_hash(minimizer_fast(m)) % n_ranks) is `rank`; n_ranks = 0: no filter.
struct CtgOwner {
  int n_ranks, rank, m;
};

// Contig pass (kcount_ctg.hip). Scratch sizes come from ctg_scratch_bytes.
size_t ctg_scratch_bytes(uint64_t n_windows, int nl);
// Extract, sort by key (stable: contig order kept within a key), fold every key's contig occurrences in
// order (insert_supermer_from_ctg) and sort the folded k-mers by local fine bucket. Outputs (n_out of them)
// go to out_keys[NL] (SoA, each out_cap long), out_state, out_bucket.
// Only k-mers whose coarse bucket is in [own_lo, own_hi) (this rank's hash range) are kept.
hipError_t ctg_prepare(const CtgView &cv, int k, int nl, bool mixed, int qual_cutoff, int dmin_thres,
                       double dyn_mult, int coarse_bits, int fine_bits, uint32_t own_lo, uint32_t own_hi,
                       const CtgOwner &ow, void *scratch, size_t scratch_bytes,
                       uint64_t *const out_keys[4], uint32_t *out_state, uint32_t *out_bucket, uint64_t *n_out,
                       unsigned int *err, hipStream_t s);

enum {
  STAT_DISTINCT = 0,
  STAT_NOUT = 1,
  STAT_PURGED = 2,
  STAT_COUNTSUM = 3,
  STAT_SWEEPS = 4,
  STAT_MAXBUCKET = 5,
  STAT_MISSES = 6,    // records worked off in phase B (not in their home group)
  STAT_N = 8,         // stats[STAT_N - 1]: internal error flag
};
constexpr int STAT_ALLOC = 16;
// k_count's cold sweeps (< 0xC000 records) hand their waves the rounds' record slots dynamically; their deferred
// records go to a per-workgroup spill area of this many records (and from there back to the bucket's own region)
constexpr uint32_t SPILL_RECORDS = 0xC000;  // stats[8..13]: k_count phase stamps in MHMKC_STAMP builds
// ... for keys of at most this many words (with three and four key words the dynamic instantiation spilled 20-40 VGPRs
// and made k_count 10-22 % slower): the host allocates the spill area only for them
constexpr int DYN_SWEEP_MAX_NL = 2;

// Workgroup shapes (each measured against its neighbours on MI355X).
constexpr int E_THREADS = 256;  // default threads of the extract / partition workgroups
constexpr int E_NSUB = 8;       // segments per coarse bucket: one per group of workgroups sharing an XCD
// k_count: one persistent 1024-thread workgroup per CU with all 160 KB of LDS (two 512-thread workgroups with half
// the LDS each measured slower once the fine partition's cost is counted, §4.2). MHMKC_CSPLIT=2 builds (A/B variants
// only) run that split: C_SPLIT workgroups per CU, each with 1/C_SPLIT of the threads, the LDS and the table.
#ifndef MHMKC_CSPLIT
#define MHMKC_CSPLIT 1
#endif
constexpr int C_SPLIT = MHMKC_CSPLIT;
constexpr int C_THREADS = 1024 / C_SPLIT;
constexpr size_t C_LDS = 163840 / C_SPLIT;

// Hash bits stored in a packed record next to the ext code (bits [6, 6 + hbits) of the last word).
inline int stored_hash_bits(int k, int nl, bool packed) {
  if (!packed) return 0;
  const int room = 64 - 2 * (k - 32 * (nl - 1)) - 6;
  return room >= 16 ? 16 : (room >= 8 ? room : 0);
}

// Bases per extract tile, by key words. Two-word keys: 4096-base tiles of 16 windows per thread (78 KB of LDS before
// the capped stage, two workgroups per CU) measured faster than 2048 (k = 63 extract 9.29 -> 8.52 ms). Three-word
// keys: 1536-base tiles, so that the staged 24-byte records of three workgroups fit a CU's LDS (2048: k = 77 14.70 ->
// 13.05 ms); four-word keys keep 2048 (1536: 16.08 -> 19.09 ms).
constexpr int TILE_BASES[5] = {0, 4096, 4096, 1536, 2048};
inline int tile_bases(int nl) { return TILE_BASES[nl]; }
// threads of an extract workgroup (tile_bases / threads windows each); four-word keys: 8 windows per thread at 256
// threads and 128 VGPRs fit four workgroups per CU (512 threads: 13.23 ms, 256: 10.04 ms at k = 99)
constexpr int E_THREADS_NL[5] = {0, 256, 256, 256, 256};
// records per partition chunk and threads per partition workgroup; two-, three- and four-word keys take longer chunks
// over more threads (the chunk's runs per fine bucket grow, the LDS per wave stays; four-word: the staged chunk + 2048
// bins' counters fit 160 KB; two-word 3072 over 512: k = 63 5.59 -> 5.50 ms, k = 33 7.49 -> 7.33)
constexpr int P_TILE[5] = {0, 4096, 3072, 4096, 3072};
constexpr int P_THREADS[5] = {0, 256, 512, 512, 512};
inline int chunk_records(int nl) { return P_TILE[nl]; }
// LDS hash-table slots of the count kernel for NL words per key (~143 KB of LDS); compact records keep
// 32-bit keys (the stored bits of the mixed key), 24 bytes per slot instead of 28.
// k_count LDS: table (keys, count, 4 extension words per slot) + 192 B of scalars + the miss queues of the waves
// (key words + ext code per entry); together <= 160 KiB. Two-word keys: 3800 / 4200 slots measured slower than 4000,
// three / four-word keys 2880 / 2400 slower than 3264 / 2752 (§4.2).
constexpr int COUNT_CAP[5] = {0, 5120, 4000, 3264, 2752};
__host__ __device__ constexpr int count_key_bytes(bool cmp) { return cmp ? 4 : 8; }
__host__ __device__ constexpr int count_cap(int nl, bool cmp = false) {
  return ((cmp ? 6144 : COUNT_CAP[nl]) / C_SPLIT) & ~3;
}
__host__ __device__ constexpr size_t count_table_bytes(int nl, bool cmp = false) {
  return (size_t)count_cap(nl, cmp) * (count_key_bytes(cmp) * nl + 4 + 16) + 256;  // + k_count's scalars
}
__host__ __device__ constexpr int miss_cap(int nl, bool cmp = false) {
  return (int)(((C_LDS - count_table_bytes(nl, cmp)) / (count_key_bytes(cmp) * nl + 4)) & ~(size_t)63);
}
__host__ __device__ constexpr size_t count_lds_bytes(int nl, bool cmp = false) {
  return count_table_bytes(nl, cmp) + (size_t)miss_cap(nl, cmp) * (count_key_bytes(cmp) * nl + 4);
}
static_assert(count_lds_bytes(1) <= C_LDS && count_lds_bytes(2) <= C_LDS && count_lds_bytes(3) <= C_LDS &&
                  count_lds_bytes(4) <= C_LDS && count_lds_bytes(1, true) <= C_LDS,
              "k_count LDS budget");

hipError_t launch_tile_first_read(const ReadsView &r, uint32_t *out, uint32_t n_tiles, int tile, hipStream_t s);
// the batch's read-start bits for the extraction (read_start_words(n_tiles, nl) u32, every word written):
// ExtractParams tile_starts
hipError_t launch_read_start_bits(const ReadsView &r, uint32_t *bits, uint64_t n_words, hipStream_t s);
uint64_t read_start_words(uint64_t n_tiles, int nl);
// total counted windows sum(max(0, L - k - 1)) of a batch, added to *out; err bit 2 (4) when the offsets are
// not a valid PackedReads CSR (offs[0] != 0, decreasing, a read longer than 65535, offs[n] != n_bases)
hipError_t launch_count_windows(const ReadsView &r, int k, unsigned long long *out, unsigned int *err, hipStream_t s);
// one H2D chunk of a host batch sent as nibbles (code | (q >= qcut) << 3, two per byte): arena[b0, b0 + n) as PackedRead
// bytes again (code | (q >= qcut ? 31 : 0) << 3)
hipError_t launch_expand_nibbles(const uint8_t *nib, uint8_t *arena, uint64_t b0, uint64_t n, hipStream_t s);
// offs[i] = b0 + d[i], i < n: a chunk's offsets from the u32 distances the nibble H2D sends
hipError_t launch_offs_from_deltas(const uint32_t *d, uint64_t *offs, uint64_t n, uint64_t b0, hipStream_t s);
// capped fine layout: base/cursor of bucket (c, d) = coarse_base[c] + d * coarse_fcap[c]
// The incremental layout after its last round: a coarse bucket with a fine bucket past its capped
// segment (k_part_scatter wrote none of that bucket's overflowing runs) gets skip[c] = 1 and all its fine buckets
// emptied (cursor = base), so k_count counts the others and the host redoes just the skipped coarse buckets; err bit 1
// (the overflow flag, which would void the k_count launch) is cleared.
hipError_t launch_inc_fixup(const unsigned long long *coarse_base, const unsigned long long *coarse_fcap,
                            uint32_t n_coarse, int fine_bits, unsigned long long *cursor, uint8_t *skip,
                            unsigned int *err, hipStream_t s);
hipError_t launch_init_fine(const unsigned long long *coarse_base, const unsigned long long *coarse_fcap,
                            uint32_t n_coarse, int fine_bits, unsigned long long *base, unsigned long long *cursor,
                            hipStream_t s);
hipError_t launch_extract_hist(const ExtractParams &p, int nl, bool packed, hipStream_t s);
hipError_t launch_extract_scatter(const ExtractParams &p, int nl, bool packed, hipStream_t s);
// chunk_run[c] for every chunk of the runs (one workgroup per run)
hipError_t launch_chunk_runs(const SRun *runs, uint32_t n_runs, SChunk *chunks, int tile, hipStream_t s);
hipError_t launch_part_hist(const PartitionParams &p, int nl, bool packed, hipStream_t s);
hipError_t launch_part_scatter(const PartitionParams &p, int nl, bool packed, hipStream_t s);
// HyperLogLog sketch of the distinct keys in chunks [0, n_chunks) of p's chunk table (one coarse bucket):
// hll[SKETCH_M] registers, max-merged, and hll[SKETCH_M] += the records' extension adds; hll[SKETCH_M + 1 ..
// 2 SKETCH_M + 1) the registers of the even-numbered chunks alone (a second sample point for the growth of the distinct
// keys with the records). Zero all 2 SKETCH_M + 1 words first. fine_hist (p.fine_bits =
// SKETCH_FB): also the records per fine digit, hll[SKETCH_WORDS ..) (SKETCH_FH more words, zeroed too), from which the
// incremental layout learns how unevenly the records fall on fine buckets (a key's copies all land in one).
constexpr int SKETCH_M = 1024;
constexpr int SKETCH_WORDS = 2 * SKETCH_M + 1;
constexpr int SKETCH_FB = 11, SKETCH_FH = 1 << SKETCH_FB;
hipError_t launch_sketch(const PartitionParams &p, uint32_t n_chunks, unsigned int *hll, int nl, bool packed,
                         hipStream_t s, bool fine_hist = false);
hipError_t launch_scan(const unsigned long long *in, unsigned long long *base, unsigned long long *cursor,
                       uint32_t n, hipStream_t s);
hipError_t launch_count(const CountParams &p, int nl, bool packed, hipStream_t s);
// The exchange's send side: the filled part of every capped segment a peer owns, copied back to back into a dense
// send plane (a slab's owned range has up to the capped slack between its segments, which the wire need not carry).
// Elements of elem_bytes (1, 4, 8 or 16); segs in elements.
struct SegCopy {
  uint64_t src, dst, n;
};
hipError_t launch_seg_gather(const SegCopy *segs, uint32_t n_segs, const void *src, void *dst, int elem_bytes,
                             hipStream_t s);

// FASTQ ingest (fastq.hip): text -> PackedRead bytes. FQ_CHUNK bytes of text per count / lines block.
constexpr int FQ_CHUNK = 4096;
// longest line (without its newline) that the reference's fgets buffer reads whole (BUF_SIZE 2047,
// src/fastq.hpp:61)
constexpr uint64_t FQ_MAX_LINE = 2045;
// error kinds, in the order the reference checks them (src/fastq.cpp:525-547, packed_reads.cpp:104)
enum { FQ_E_ID = 1, FQ_E_PLUS = 2, FQ_E_NAME = 3, FQ_E_LEN = 4, FQ_E_LONG = 5, FQ_E_CHAR = 6, FQ_E_TRUNC = 7 };
// read-pair merging (merge_reads.cpp), reported at the pair's second record so that both records' own checks
// come first, in the reference's order: names, pair numbers, mate 2's revcomp, an overlap quality, mate 1's
// (or the merged read's) PackedRead
enum { FQ_E_PAIR_NAME = 8, FQ_E_PAIR_NUM = 9, FQ_E_CHAR2 = 10, FQ_E_QUAL = 11, FQ_E_CHAR1 = 12 };
size_t fq_scan_tmp_bytes(uint64_t n_items);
hipError_t fq_scan(void *tmp, size_t tmp_bytes, const unsigned long long *in, unsigned long long *out,
                   uint64_t n_items, hipStream_t s);
// newlines per FQ_CHUNK chunk -> chunk[ceil(n / FQ_CHUNK)]
hipError_t launch_fq_count(const char *text, uint64_t n, unsigned long long *chunk, hipStream_t s);
hipError_t launch_offs_rebase(unsigned long long *dst, const unsigned long long *src, uint64_t n, unsigned long long delta,
                              hipStream_t s);
// every newline, in order, from the scanned chunk counts, as one word per line: position (bits 0-39),
// trailing whitespace count of the line it ends (bits 40-55), first character of the next line (56-63)
constexpr int FQ_LE_BITS = 40;
constexpr uint64_t FQ_LE_MASK = (1ull << FQ_LE_BITS) - 1;
hipError_t launch_fq_lines(const char *text, uint64_t n, const unsigned long long *chunk_base,
                           unsigned long long *line_end, hipStream_t s);
// per record: sequence length (len[n_rec] = 0 for the scan) and format checks (err: atomicMin of
// record << 4 | FQ_E_*)
// paired input: k_fq_records' checks and the pair descriptors in one pass (launch_fq_merge reads the descriptors)
hipError_t launch_fq_pair_records(const char *text, uint64_t n, const unsigned long long *line_end, uint64_t n_rec,
                                  unsigned long long *len, unsigned long long *err, void *desc_buf, hipStream_t s);
hipError_t launch_fq_records(const char *text, uint64_t n, const unsigned long long *line_end, uint64_t n_rec,
                             unsigned long long *len, unsigned long long *err, hipStream_t s);
// pair p = records 2p, 2p+1: verdict in pair_info, output read lengths (merged + 1, or L1, L2) in out_len
// [2 n_pairs + 1]; stats[1..3] += merged pairs, ambiguous events, overlap bases. scratch: rec_offs[2 n_pairs]
// bytes (quality copies of pairs with an N).
// bytes of the per-pair line descriptors (desc_buf) of launch_fq_merge / launch_fq_merge_pack
size_t fq_pair_desc_bytes(uint64_t n_pairs);
hipError_t launch_fq_merge(const char *text, uint64_t n, const unsigned long long *line_end, uint64_t n_pairs,
                           const unsigned long long *rec_offs, int qual_offset, char *scratch, void *desc_buf,
                           uint32_t *pair_info, unsigned long long *out_len, unsigned long long *err,
                           unsigned long long *stats, hipStream_t s);
hipError_t launch_fq_merge_pack(const char *text, const void *desc_buf, uint64_t n_pairs,
                                const unsigned long long *rec_offs, const char *scratch, const uint32_t *pair_info,
                                const unsigned long long *out_offs, int qual_offset, uint8_t *out,
                                unsigned long long *err, hipStream_t s);
hipError_t launch_fq_pack(const char *text, const unsigned long long *line_end, uint64_t n_rec,
                          const unsigned long long *offs, int qual_offset, uint8_t *out, unsigned long long *err,
                          hipStream_t s);

// Output hand-off to the reference's owner rank (kcount_owner.hip): get_kmer_target_rank =
// minimizer_hash_fast(minimizer_len) % rank_n (src/kcount/kmer_dht.cpp:193-196, src/kmer.cpp:344-393,454-463).
struct OutRows {
  uint64_t *keys;  // [n * nlo] Kmer::longs layout
  uint16_t *counts;
  char *left, *right;
};
// KmerDHT minimizer length for k (src/kcount/kmer_dht.cpp:114-116)
inline int minimizer_len_for(int k) { return k * 2 / 3 + 1 < 15 ? 15 : (k * 2 / 3 + 1 > 27 ? 27 : k * 2 / 3 + 1); }
// mhmkc_fetch_ordered: the output rows in the order of the top 32 bits of mhmkc_map_hash (kcount_owner.hip)
size_t map_order_scratch_bytes(uint64_t n, int nlo);
hipError_t preload_owner_kernels();
// mhmkc_fetch_map_range: each of the n ordered rows' slot in a KmerMap of cap (a power of two) slots filled in this
// order from empty (0xFFFFFFFF: past the last slot) and its tag byte
size_t map_slots_scratch_bytes(uint64_t n);
hipError_t launch_map_slots(const uint64_t *keys, uint64_t n, int nlo, uint64_t cap, void *scratch, size_t scratch_bytes,
                            uint32_t *slot, uint8_t *tag, hipStream_t s);
hipError_t launch_map_order(const OutRows &in, uint64_t n, int nlo, void *scratch, size_t scratch_bytes, const OutRows &out,
                            hipStream_t s);
// minimizer_hash_fast of n keys (nlo words each, the first k/32+1 used)
hipError_t launch_minimizer_hash(const uint64_t *keys, uint64_t n, int nlo, int k, int m, uint64_t *out, hipStream_t s);
// dest[i] = owner rank of row i; hist[r] += rows owned by rank r (zero hist first)
hipError_t launch_owner_hist(const uint64_t *keys, uint64_t n, int nlo, int k, int m, int n_ranks, uint8_t *dest,
                             unsigned long long *hist, hipStream_t s);
// rows grouped by owner: row i goes to out at cursor[dest[i]]++ (cursor = per-owner start offsets)
hipError_t launch_owner_scatter(const OutRows &in, uint64_t n, int nlo, const uint8_t *dest, int n_ranks,
                                unsigned long long *cursor, const OutRows &out, hipStream_t s);

}  // namespace mhm
