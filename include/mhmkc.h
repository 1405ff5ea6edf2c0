/*
 * mhmkc.h — C ABI of the MI355X-native k-mer counting stage (libmhmkc.so).
 *
 * This is the drop-in boundary for the MetaHipMer2 kcount hot path of ajpowelsnl/mhm2_proxy
 * (reference: src/kcount/). The reference has no C ABI; its backend seam is two pimpl classes,
 * SeqBlockInserter<MAX_K> (src/kcount/kcount.hpp:57-69) and HashTableInserter<MAX_K>
 * (src/kcount/kmer_dht.hpp:95-116), linked either from kcount_cpu.cpp or kcount_gpu.cpp
 * (src/kcount/CMakeLists.txt:23-43). Every entry point below names the reference interface it
 * replaces. include/mhmkc_kcount.hpp rebuilds those C++ shapes (Kmer<MAX_K>, KmerCounts, KmerMap,
 * analyze_kmers) on top of this ABI; INTEGRATION.md shows the binding.
 *
 * Semantics are bit-exact with the reference CPU kcount (kcount_cpu.cpp), not with its CUDA
 * backend (which drops N-k-mers, caps extension counts at 10000 and uses an approximate filter).
 *
 * Conventions (mirroring the reference's error behaviour, which DIEs on bad input):
 *   - every function returns MHMKC_OK (0) or a negative MHMKC_E* code; mhmkc_last_error() holds the
 *     message; the C++ adapter turns a failure into a fatal error like the reference's DIE;
 *   - host input buffers are borrowed only for the duration of the call;
 *   - device input buffers passed to *_device functions must stay valid until mhmkc_finish returns, and
 *     are read on the handle's stream: data written on another stream must be ordered first with
 *     mhmkc_wait_stream (or by creating the handle on that stream, mhmkc_config.stream);
 *   - a handle drives exactly one GPU and is not thread-safe. Multi-GPU = one process (rank) per
 *     GPU, all ranks calling the same sequence; the k-mer exchange is an all-to-all inside mhmkc_finish
 *     (replacing the UPC++ supermer store, src/kcount/kmer_dht.cpp:133-149,222-224): RCCL over xGMI
 *     (mhmkc_config.comm_id), or a host-staged transport the caller provides (mhmkc_set_transport: a
 *     UPC++/MPI/gloo host, several nodes, or several ranks sharing one GPU).
 */
#ifndef MHMKC_H
#define MHMKC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MHMKC_ABI_VERSION 14
#define MHMKC_COMM_ID_BYTES 128

enum {
  MHMKC_OK = 0,
  MHMKC_EINVAL = -1,      /* bad argument or configuration */
  MHMKC_ENOMEM = -2,      /* device or host allocation failed */
  MHMKC_EHIP = -3,        /* HIP runtime error */
  MHMKC_ERCCL = -4,       /* RCCL error */
  MHMKC_ESTATE = -5,      /* call out of order (e.g. fetch before finish) */
  MHMKC_EBADCHAR = -6,    /* input byte outside the PackedRead code range (reference DIE, kcount_cpu.cpp:453-458) */
  MHMKC_EUNSUPPORTED = -7, /* valid for the reference but not supported here */
  MHMKC_ETRANSPORT = -8    /* a mhmkc_set_transport callback failed, or none was set where needed */
};

typedef struct mhmkc *mhmkc_t;

/* Configuration of one counting round (one k). Replaces the KmerDHT constructor arguments
 * (src/kcount/kmer_dht.cpp:106-154) and the analyze_kmers parameters (src/kcount/kcount.hpp:71-73). */
typedef struct {
  int32_t k;              /* k-mer length; 1 <= k <= 127, k % 32 != 0 */
  int32_t n_longs;        /* output words per key; 0 = k/32+1 (= MAX_K/32, src/main.cpp:170) */
  int32_t qual_offset;    /* 33 or 64 (only used by mhmkc_add_seqs' PackedRead-free path) */
  int32_t qual_cutoff;    /* KCOUNT_QUAL_CUTOFF (CMakeDefinitions.txt:46), default 20 */
  int32_t dmin_thres;     /* --min-depth-thres (src/options.cpp:289-290), default 2; <= 32768 */
  double dyn_min_depth;   /* DYN_MIN_DEPTH (CMakeDefinitions.txt:60), default 0.9 */
  int32_t device;         /* HIP device ordinal; -1 = current device */
  int32_t rank;           /* this rank, 0 <= rank < n_ranks */
  int32_t n_ranks;        /* number of GPUs (ranks) sharing the k-mer space */
  const uint8_t *comm_id; /* MHMKC_COMM_ID_BYTES from mhmkc_comm_id() on rank 0; NULL if n_ranks==1 or
                             the exchange goes through mhmkc_set_transport */
  void *stream;           /* hipStream_t to run on; NULL = the library creates its own */
  int32_t output_owner;   /* MHMKC_OWNER_*: where a finished k-mer lives when n_ranks > 1 */
  int32_t minimizer_len;  /* m of get_kmer_target_rank; 0 = the KmerDHT rule clamp(2k/3+1, 15, 27)
                             (src/kcount/kmer_dht.cpp:114-116) */
} mhmkc_config;

enum {
  MHMKC_OWNER_HASH = 0,      /* the counting partition (hash range): no extra exchange */
  MHMKC_OWNER_MINIMIZER = 1  /* the reference's owner, KmerDHT::get_kmer_target_rank =
                                minimizer_hash_fast(minimizer_len) % n_ranks (src/kcount/kmer_dht.cpp:193-196),
                                which dbjg_traversal.cpp looks k-mers up on (:232-234,264-274) */
};

/* Statistics; replaces the SLOG lines of flush_inserts / insert_into_local_hashtable
 * (src/kcount/kcount_cpu.cpp:465-488,525-527). Counters are for this rank. */
typedef struct {
  uint64_t reads;          /* reads submitted */
  uint64_t bases;          /* bases submitted */
  uint64_t occurrences;    /* counted windows i in [1, L-k-1] (records produced by this rank) */
  uint64_t owned_records;  /* records counted on this rank after the exchange */
  uint64_t distinct;       /* distinct canonical k-mers owned by this rank */
  uint64_t purged;         /* dropped at finish: count < 2 or both extensions 'X' */
  uint64_t n_out;          /* k-mers in the output table (== distinct - purged) */
  uint64_t dropped;        /* always 0: the table never drops (reference num_dropped) */
  uint64_t count_sum;      /* sum over distinct k-mers of the unsaturated count (== owned_records) */
  uint64_t overflow_sweeps;/* extra LDS sweeps needed by over-full fine buckets */
  uint64_t max_bucket;     /* largest fine bucket, records */
  uint64_t fine_buckets;   /* number of fine buckets on this rank */
  uint64_t bytes_sent;     /* bytes sent to other ranks in the exchange */
  uint64_t exact_reruns;   /* capped partition passes redone with exact bucket sizes (skewed input) */
  uint64_t ctg_kmers;      /* distinct contig k-mers of the contig pass (0 without contigs) */
  uint64_t coarse_record_bytes; /* HBM bytes per k-mer record after extraction (5 for compact records) */
  uint64_t fine_record_bytes;   /* HBM bytes per k-mer record after the fine partition (4 when compact) */
  uint64_t distinct_estimate;   /* sketch estimate of this rank's distinct k-mers (sizes the fine partition) */
  double ms_total;         /* wall time of the last add_reads..finish sequence (device events) */
  double ms_kernel[8];     /* per-stage device time when profiling is on: see MHMKC_STAGE_* */
  uint64_t launches[8];    /* per-stage launch count when profiling is on */
  uint64_t bytes_recv;     /* bytes received from other ranks in the exchange */
  uint64_t handoff_sent;   /* finished k-mers moved to their MHMKC_OWNER_MINIMIZER owner (other ranks) */
  uint64_t handoff_recv;   /* finished k-mers received from other ranks at the hand-off */
  uint64_t h2d_bytes;      /* host bytes copied to the device by mhmkc_add_reads (PackedRead bytes + offsets) */
  uint64_t h2d_chunks;     /* H2D chunks of mhmkc_add_reads, each extracted as soon as it has landed */
  uint64_t slabs;          /* extracted record slabs (one per device batch or H2D chunk) */
  double ms_h2d;           /* device time of the H2D copies of the last mhmkc_add_reads (copy-stream events) */
  uint64_t lds_misses;     /* count kernel: records not found in their home slot group (LDS slow path) */
  uint64_t lds_ext_adds;   /* count kernel: extension-counter increments (from the sampled first coarse bucket,
                              scaled to all records) */
  uint64_t fq_pairs;       /* mhmkc_add_fastq_pairs: read pairs of the last call */
  uint64_t fq_merged;      /* ... of which merged (merge_reads num_merged) */
  uint64_t fq_ambiguous;   /* ... merge_reads' num_ambiguous increments */
  uint64_t fq_overlap_bases; /* ... overlap bases of the merged pairs (merge_reads overlap_len) */
  uint64_t table_slots;    /* count kernel: LDS table slots used per fine bucket (fitted to the sketch estimate) */
  uint64_t fq_file_blocks; /* mhmkc_add_fastq[_pairs]_file: blocks of the last call */
  uint64_t smer_count;     /* supermer exchange: supermers this rank built (all destinations, itself included) */
  uint64_t smer_words;     /* ... their 32-base words (each a u64 of 2-bit codes + a u32 of extension bits) */
  uint64_t xchg_rounds;    /* pipelined record exchange: rounds (one per slab of the rank with the most slabs) */
  double ms_xchg;          /* ... device time of the rounds' transfers (exchange stream events, summed) */
  double ms_xchg_exposed;  /* ... of it after the last extraction ended (what the overlap did not hide) */
  uint64_t finish_passes;  /* finish: parts of the owned hash range counted one after the other (memory: MHMKC_PASSES,
                              or as many as free device memory asks for) */
  uint64_t out_reruns;     /* finish passes redone because the output (sized from the distinct-key sketch) was full */
  uint64_t device_bytes;   /* device memory held by this process's handles after the finish */
  uint64_t device_bytes_peak; /* ... the most it held at any time */
  uint64_t inc_rounds;     /* pipelined record exchange: rounds fine-partitioned as they landed (0: all at finish) */
  uint64_t inc_fallbacks;  /* ... finishes whose incremental count failed and were redone from the sources */
  double ms_finish_tail;   /* device time from the last transfer's end (or finish's start) to the finished table */
  uint64_t inc_redone_coarse; /* ... coarse buckets whose capped fine layout overflowed (skew), counted again exactly */
  double inc_slack;           /* ... the capped fine buckets' slack over their expected records (0.25 .. 2) */
  double ms_h2d_pack;         /* last mhmkc_add_reads: host wall time packing its chunks for the wire (nibble H2D) */
  double ms_h2d_wait;         /* ... host wall time waiting for a pinned staging slot's previous copy */
  double ms_h2d_rounds;       /* ... host wall time enqueueing local rounds between its chunks (mhmkc_debug.h) */
  uint64_t h2d_raw_chunks;    /* ... its chunks sent as PackedRead bytes (the wire had drained while the host packed) */
} mhmkc_stats;

enum {
  MHMKC_STAGE_TILEIDX = 0, /* per-tile first-read index */
  MHMKC_STAGE_EHIST = 1,   /* extract + coarse histogram */
  MHMKC_STAGE_ESCAT = 2,   /* extract + coarse scatter */
  MHMKC_STAGE_XCHG = 3,    /* RCCL all-to-all exchange */
  MHMKC_STAGE_SHIST = 4,   /* fine histogram */
  MHMKC_STAGE_SSCAT = 5,   /* fine scatter */
  MHMKC_STAGE_COUNT = 6,   /* LDS hash-table count + finalize + compaction */
  MHMKC_STAGE_OTHER = 7    /* scans, memsets */
};

/* Fill *cfg with the reference defaults (k=21, qual 33/20, dmin 2, dyn 0.9, one rank). */
int mhmkc_config_init(mhmkc_config *cfg);

/* Create a counter. Replaces KmerDHT<MAX_K>::KmerDHT + HashTableInserter::init
 * (src/kcount/kmer_dht.cpp:106-154, src/kcount/kcount_cpu.cpp:425-443). With n_ranks > 1 every rank
 * must call this collectively with the same comm_id. */
int mhmkc_create(mhmkc_t *h, const mhmkc_config *cfg);

/* Release all device memory and the communicator (HashTableInserter::~HashTableInserter,
 * src/kcount/kcount_cpu.cpp:420-423). NULL is allowed. */
void mhmkc_destroy(mhmkc_t h);

/* RCCL unique id for mhmkc_config.comm_id (rank 0 calls it and broadcasts the bytes). */
int mhmkc_comm_id(uint8_t out[MHMKC_COMM_ID_BYTES]);

/* Add reads in the PackedRead byte layout (src/packed_reads.cpp:73-109): one byte per base,
 * bits 0-2 = A,C,G,T,N -> 0..4, bits 3-7 = min(q - qual_offset, 31). read_offsets has n_reads+1
 * entries, read_offsets[0] == 0, read i = bytes[read_offsets[i], read_offsets[i+1]).
 * Replaces the count_kmers read loop + SeqBlockInserter::process_seq
 * (src/kcount/kcount.cpp:54-98, src/kcount/kcount_cpu.cpp:73-103). Host buffers: copied to the device in
 * chunks on a copy stream, each chunk extracted as soon as it has landed (pinned host memory, e.g. from
 * hipHostMalloc, lets the copies run without the CPU). Returns once the copies are done. */
int mhmkc_add_reads(mhmkc_t h, const uint8_t *packed_bytes, const uint64_t *read_offsets, uint64_t n_reads);

/* Same, with device-resident buffers (no copy; must stay valid until mhmkc_finish returns). n_bases must be
 * d_read_offsets[n_reads]; the offsets are checked on the device (MHMKC_EINVAL: not a PackedReads CSR). */
int mhmkc_add_reads_device(mhmkc_t h, const uint8_t *d_packed_bytes, const uint64_t *d_read_offsets,
                           uint64_t n_reads, uint64_t n_bases);

/* Order the handle's later device work after everything enqueued so far on `stream` (a hipStream_t; NULL =
 * the legacy default stream): call it before passing buffers that another stream (e.g. torch's current
 * stream) has just written. */
int mhmkc_wait_stream(mhmkc_t h, void *stream);

/* Add sequences given as characters, lowercase = quality below the cutoff — the string that
 * SeqBlockInserter::process_seq receives (src/kcount/kcount.cpp:80-86). Host buffers. depth is the
 * per-sequence count (reads: 1). Only depth == 1 (the read pass) is supported in this version. */
int mhmkc_add_seqs(mhmkc_t h, const char *seqs, const uint64_t *seq_offsets, uint64_t n_seqs, uint16_t depth);

/* Add reads given as FASTQ text: parsed and packed on the device, then counted as mhmkc_add_reads.
 * Replaces FastqReader::get_next_fq_record (src/fastq.cpp:504-551: 4 lines per record, rtrim, the '@' and
 * '+' checks, get_fq_name :73-122, equal sequence and quality lengths) + the PackedRead constructor
 * (src/packed_reads.cpp:73-109: N and IUPAC codes -> 4, quality min(q - qual_offset, 31)) for reads that
 * reach kcount unchanged (single-end input; paired input goes through mhmkc_add_fastq_pairs, which merges
 * the pairs first). Where the reference DIEs the call fails:
 * MHMKC_EINVAL for a malformed record (the message names the first bad record, 0-based),
 * MHMKC_EBADCHAR for a base outside A C G T N U R Y K M S W B D H V, MHMKC_EUNSUPPORTED for a line
 * longer than 2045 characters (the reference's fgets buffer, src/fastq.hpp:61, would split it).
 * Host text of n_bytes bytes (no terminator needed). */
int mhmkc_add_fastq(mhmkc_t h, const char *text, uint64_t n_bytes);

/* Same, with device-resident text (only read during the call). The buffer must extend at least 4 bytes
 * past n_bytes (the parser reads whole aligned dwords; the padding bytes are never interpreted). */
int mhmkc_add_fastq_device(mhmkc_t h, const char *d_text, uint64_t n_bytes);

/* Add read pairs given as interleaved FASTQ text (records 2p and 2p+1 are the mates /1 and /2 of pair p, the
 * order FastqReader gives a pair of files, src/fastq.cpp:509-516): parsed on the device as mhmkc_add_fastq,
 * then merged as merge_reads does (src/merge_reads.cpp:237-588: mate 2 reverse-complemented, offsets scanned
 * with the mismatch, N and differential-quality rules, an unambiguous overlap merged base by base by quality),
 * and the resulting PackedReads counted: for each pair the merged read and a dummy mate "N", or both mates
 * unmerged (packed_reads_list of merge_reads). A last record without its mate is not added (the reference's
 * loop stops there). Fails where the reference DIEs: the mhmkc_add_fastq errors, MHMKC_EINVAL for mates whose
 * names differ or are not /1 and /2 ("Mismatched pairs"), for an overlap quality outside the Q2Perror table,
 * MHMKC_EBADCHAR for an illegal base. Statistics: fq_pairs, fq_merged, fq_ambiguous, fq_overlap_bases. */
int mhmkc_add_fastq_pairs(mhmkc_t h, const char *text, uint64_t n_bytes);
/* Same, with device-resident text (only read during the call; 4 bytes of padding as for mhmkc_add_fastq_device). */
int mhmkc_add_fastq_pairs_device(mhmkc_t h, const char *d_text, uint64_t n_bytes);

/* FASTQ file ingest with the file I/O overlapped: the file at `path` is read in blocks of
 * MHMKC_FQ_BLOCK bytes (environment; default 256 MB) into pinned memory, each block copied to the device and parsed
 * (as mhmkc_add_fastq / mhmkc_add_fastq_pairs) as soon as it is read, its cut last record (pair) carried into the
 * next block; a block's extraction runs on the device while the next block is read. Errors as for the text entry
 * points (record indices in messages count from the start of the failing block; the message names the block and
 * the file byte its text starts at); MHMKC_EINVAL if the file cannot be opened or read. A failure after the first
 * block leaves the earlier blocks' reads in the round: mhmkc_finish then fails with MHMKC_ESTATE until
 * mhmkc_reset. mhmkc_fastq_packed / mhmkc_fastq_fetch then hold the PackedReads of the whole file (every
 * block's, appended on the device: the later k rounds count them with mhmkc_add_reads_device). */
int mhmkc_add_fastq_file(mhmkc_t h, const char *path);
int mhmkc_add_fastq_pairs_file(mhmkc_t h, const char *path);

/* The PackedReads of the last mhmkc_add_fastq[_pairs][_device] call on the device: d_bytes[n_bases] in the
 * PackedRead layout, d_offsets[n_reads + 1]. Valid until the next add_fastq, reset or destroy. Any
 * pointer may be NULL. */
int mhmkc_fastq_packed(mhmkc_t h, const uint8_t **d_bytes, const uint64_t **d_offsets, uint64_t *n_reads,
                       uint64_t *n_bases);

/* Copy the PackedReads of the last mhmkc_add_fastq[_device] call to host arrays (either may be NULL):
 * bytes[n_bases], offsets[n_reads + 1] (sizes from mhmkc_fastq_packed). */
int mhmkc_fastq_fetch(mhmkc_t h, uint8_t *bytes, uint64_t *offsets);

/* Add contigs for the contig pass of rounds after the first k (add_ctg_kmers, src/kcount/kcount.cpp:100-138;
 * insert_supermer_from_ctg, src/kcount/kcount_cpu.cpp:356-406). seqs: contig sequences back to back (case
 * = quality as for reads; contigs are uppercase), seq_offsets: n_ctgs+1 offsets, depths:
 * Contig::get_uint16_t_depth() (src/contigs.hpp:65), 0 counting as 1. The contig pass runs inside
 * mhmkc_finish after every read, over the contigs in the order they were added (the reference's order,
 * which its rules depend on). Contigs shorter than k+2 contribute nothing. Host buffers. With several ranks
 * every rank passes its own contigs (possibly none) and the contigs of all ranks are applied in rank order
 * (rank 0's first), one serialisation the reference's concurrent supermer stores can produce; the result
 * equals a single rank given the concatenation. */
int mhmkc_add_ctgs(mhmkc_t h, const char *seqs, const uint64_t *seq_offsets, const uint16_t *depths, uint64_t n_ctgs);

/* The depth threshold of the finish: the reference's global _dmin_thres (src/kcount/kmer_dht.hpp:57), which
 * analyze_kmers sets (src/kcount/kcount.cpp:145) after the KmerDHT was built and get_ext reads at finish
 * (src/kcount/kcount_cpu.cpp:178). Starts as mhmkc_config.dmin_thres; takes effect at the next finish. */
int mhmkc_set_dmin_thres(mhmkc_t h, int32_t dmin_thres);

/* Exchange (multi-GPU), count and finalize: purge count < 2 and X/X, choose extensions; with
 * MHMKC_OWNER_MINIMIZER, then move every finished k-mer to its get_kmer_target_rank owner.
 * Replaces KmerDHT::flush_updates + finish_updates -> HashTableInserter::insert_into_local_hashtable
 * (src/kcount/kmer_dht.cpp:227-236, src/kcount/kcount_cpu.cpp:490-528). *n_out may be NULL. */
int mhmkc_finish(mhmkc_t h, uint64_t *n_out);

/* Copy the finished table to host arrays (any may be NULL): keys[n_out*n_longs] in Kmer::longs layout,
 * counts[n_out], left[n_out], right[n_out] ('A','C','G','T','F' or 'X'). Order is unspecified, as the
 * reference's KmerMap iteration order is. Replaces the KmerMap fill (kcount_cpu.cpp:503-522). */
int mhmkc_fetch(mhmkc_t h, uint64_t *keys, uint16_t *counts, char *left, char *right);

/* The hash the C++ adapter's KmerMap (include/mhmkc_kcount.hpp) places a key with: a multiply-xorshift mix of its
 * n_longs words; the map's home slot for a key is the top log2(capacity) bits. */
#ifdef __HIPCC__
__host__ __device__
#endif
static inline uint64_t mhmkc_map_hash(const uint64_t *w, int n_longs) {
  uint64_t h = 0x9E3779B97F4A7C15ull;
  for (int i = 0; i < n_longs; i++) {
    h = (h ^ w[i]) * 0xBF58476D1CE4E5B9ull;
    h ^= h >> 31;
  }
  h *= 0x94D049BB133111EBull;
  return h ^ (h >> 29);
}

/* mhmkc_fetch with the rows ordered by the top 32 bits of mhmkc_map_hash (a radix sort on the device): filling a
 * KmerMap in that order walks its slot array once from front to back instead of touching a random slot per row
 * (insert_into_local_hashtable's loop, src/kcount/kcount_cpu.cpp:503-522). At most 2^32-1 rows. */
int mhmkc_fetch_ordered(mhmkc_t h, uint64_t *keys, uint16_t *counts, char *left, char *right);

/* Rows [row0, row0 + n_rows) of mhmkc_fetch_ordered's order (the device sorts once per finish and keeps the ordered
 * rows until the next reset): a host that fills its KmerMap chunk by chunk while the next chunk is on the wire (the C++
 * adapter's insert_into_local_hashtable) never holds the whole table twice. */
int mhmkc_fetch_ordered_range(mhmkc_t h, uint64_t row0, uint64_t n_rows, uint64_t *keys, uint16_t *counts, char *left,
                              char *right);

/* Rows [row0, row0 + n_rows) of mhmkc_fetch_ordered's order, each with the slot it takes in a KmerMap of `capacity`
 * slots (a power of two, 16 .. 2^32; home slot = the top log2(capacity) bits of mhmkc_map_hash) filled with the rows
 * in this order from empty by linear probing, and its tag byte (0x80 | the low 7 bits of mhmkc_map_hash): slot i =
 * max(home i, slot i-1 + 1), computed on the device (a prefix maximum), or 0xFFFFFFFF past the last slot (the map
 * places that row itself). The C++ adapter's KmerMap then writes each row straight to its slot, with no hashing or
 * probing on the host (insert_into_local_hashtable, src/kcount/kcount_cpu.cpp:503-522). slots / tags may be NULL. */
int mhmkc_fetch_map_range(mhmkc_t h, uint64_t capacity, uint64_t row0, uint64_t n_rows, uint64_t *keys,
                          uint16_t *counts, char *left, char *right, uint32_t *slots, uint8_t *tags);

/* Pinned (page-locked) host memory for a caller's fetch buffers: a fetch into it is one DMA per array, with no copy
 * through the library's staging buffers (mhmkc_fetch copies into pageable memory chunk by chunk). Freed blocks are
 * kept by the library for the next mhmkc_host_alloc (up to 2 GiB), since pinning costs more than one copy. NULL when
 * the allocation fails; mhmkc_host_free ignores pointers it did not hand out. */
void *mhmkc_host_alloc(uint64_t bytes);
void mhmkc_host_free(void *p);

/* Device pointers of the finished table (valid until the next reset/destroy). */
int mhmkc_device_output(mhmkc_t h, const uint64_t **d_keys, const uint16_t **d_counts, const char **d_left,
                        const char **d_right, uint64_t *n_out);

/* Host-staged exchange between ranks (instead of RCCL): for n_ranks > 1 with comm_id == NULL, set before
 * the first mhmkc_finish. Every rank's callbacks are called collectively, in the same order on all ranks, with
 * host buffers; a callback returns 0 on success.
 *   allgather: every rank contributes `bytes` bytes from send; recv receives n_ranks * bytes, rank order;
 *   alltoallv: send holds, back to back in rank order, send_bytes[p] bytes for every rank p (0 for itself);
 *              recv receives recv_bytes[p] bytes from every rank p, back to back in rank order.
 * This is the seam a UPC++ / MPI host (several nodes, or several ranks sharing one GPU) plugs into; the
 * reference's own transport is UPC++ RPC (src/kcount/kmer_dht.cpp:133-149,222-231). */
typedef struct {
  void *ctx;
  int (*allgather)(void *ctx, const void *send, void *recv, uint64_t bytes);
  int (*alltoallv)(void *ctx, const void *send, const uint64_t *send_bytes, void *recv, const uint64_t *recv_bytes);
} mhmkc_transport;
int mhmkc_set_transport(mhmkc_t h, const mhmkc_transport *t);

/* Kmer::minimizer_hash_fast(m) of n k-mers of the handle's k (src/kmer.cpp:344-393,454-463), computed on the
 * handle's GPU: keys[n * n_longs] in Kmer::longs layout (host), hashes[n] (host). get_kmer_target_rank is
 * hashes[i] % rank_n (src/kcount/kmer_dht.cpp:193-196). m = 0: the KmerDHT minimizer length for k. */
int mhmkc_minimizer_hashes(mhmkc_t h, const uint64_t *keys, uint64_t n, int32_t n_longs, int32_t m, uint64_t *hashes);

/* Statistics of the last round. */
int mhmkc_get_stats(mhmkc_t h, mhmkc_stats *s);

/* Forget all k-mers (keep allocations) so the handle can count the next batch/round
 * (KmerDHT::clear_stores + a fresh HashTableInserter, src/kcount/kcount.cpp:156). */
int mhmkc_reset(mhmkc_t h);

/* Per-stage HIP-event timing (mhmkc_stats.ms_kernel). Off by default (0); 1: every stage; 2: the heavy stages only
 * (extraction scatter, fine scatter, exchange, count), whose events cost the step less. */
int mhmkc_set_profiling(mhmkc_t h, int on);

/* Last error message of the handle (or of the last failed mhmkc_create when h is NULL). */
const char *mhmkc_last_error(mhmkc_t h);

/* Library ABI version (MHMKC_ABI_VERSION). */
int mhmkc_abi_version(void);

/* Build id of this library: the first 16 hex digits of the SHA-256 of the sources it was compiled from
 * (mhm2_proxy_amd/build.py: LIB_DEPS, paths and contents), fixed at compile time. A loader compares it with the id
 * of the tree it runs from to know that the binary it mapped is the one those sources make ("unknown": built
 * without build.py). Not part of the reference (provenance of the prebuilt library only). */
const char *mhmkc_build_id(void);

#ifdef __cplusplus
}
#endif

#endif /* MHMKC_H */
