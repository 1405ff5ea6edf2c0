/* mhmkc_debug.h — the test-only entry point of libmhmkc.so.
 *
 * Not part of the product interface (include/mhmkc.h): process-wide switches with which the parity tests force the
 * rare paths of the counter (exact histogram layouts instead of capped ones, tiny LDS tables, a fixed fine partition,
 * an output too small for the table, a failing file read, the key-word records the mixed ones are compared with, ...).
 * A production caller never sets them; the library reads no environment variable for them.
 */
#ifndef MHMKC_DEBUG_H
#define MHMKC_DEBUG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Set one knob (returns MHMKC_OK, or MHMKC_EINVAL for an unknown name). Knobs read at mhmkc_create (wide_records,
 * smer, local_rounds, cb0, cb0_2, cb0_3) apply to handles created afterwards, the others to the next call that uses them:
 *   exact         1: exact (histogram) layouts for every slab and finish pass
 *   cap           k_count's LDS table slots (>= 64; 0: the kernel's own)
 *   fine_bits     fine bits of the partition (-1: from the distinct-key sketch)
 *   out_cap       output rows of the first finish pass (-1: from the sketch)
 *   fq_read_fail  mhmkc_add_fastq_file: the read of this block fails (-1: none)
 *   wide_records  1: key-word records instead of the compact / mixed ones
 *   smer          0: MHMKC_OWNER_MINIMIZER at k >= 33 takes the record exchange + hand-off, not supermers
 *   chunk_bytes   H2D chunk of a host batch (0: 128 MB)
 *   d2h_chunk     staging chunk of a fetch into pageable host memory (0: 8 MB)
 *   h2d_nib       H2D of a host batch (mhmkc_add_reads): 1 the bases as nibbles and the offsets as u32 distances, 2
 *                 nibbles and u64 offsets, 0 PackedRead bytes and u64 offsets, -1 (default) 1 when the process has at
 *                 least 4 host threads, else 0
 *   h2d_threads   nibble H2D: host worker threads that pack the bases (0: all of them)
 *   h2d_nt        nibble H2D: 0 ordinary stores into the pinned staging instead of streaming stores
 *   h2d_adapt     nibble H2D from pinned memory: 1 (default) some chunks go as PackedRead bytes when the host packs
 *                 much slower than the wire runs, 0 never, 2 every other chunk
 *   local_rounds  0: one rank's host batches are fine-partitioned at finish, not chunk by chunk as they land (created
 *                 handles)
 *   cb0, cb0_2, cb0_3  coarse bits for one-, two-, three/four-word keys (0: 8, 8, 7) */
int mhmkc_debug_set(const char *knob, int64_t value);
/* Every knob back to its default. */
void mhmkc_debug_reset(void);
/* The nibble H2D's host packing (no GPU): n PackedRead bytes of src as (n + 1) / 2 bytes of nibbles
 * code | (q >= qcut) << 3 into dst, the first in the low half; mode 0 as mhmkc_add_reads packs (AVX2 when the CPU has
 * it, streaming stores into a 32-byte aligned dst), 1 the portable 8-bytes-at-a-time path, 2 AVX2 with ordinary stores
 * (MHMKC_EUNSUPPORTED without AVX2). */
int mhmkc_debug_nib_pack(const uint8_t *src, uint64_t n, uint8_t *dst, int qcut, int mode);

#ifdef __cplusplus
}
#endif

#endif
