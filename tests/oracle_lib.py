"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY (the CPU checker).

Also binds oracle/_ref/libhashref.so, the reference's own src/hash_funcs.c compiled unmodified
(oracle/Makefile), when it has been built.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
ORACLE = ROOT / "oracle" / "liboracle.so"
HASHREF = ROOT / "oracle" / "_ref" / "libhashref.so"

_o = None


def oracle() -> C.CDLL:
    global _o
    if _o is None:
        if not ORACLE.exists():
            raise ImportError(f"{ORACLE} missing: run `make -C oracle`")
        L = C.CDLL(str(ORACLE))
        U64, VP, I = C.c_uint64, C.c_void_p, C.c_int
        L.orc_murmur3_x64_64.argtypes = [VP, C.c_uint32]
        L.orc_murmur3_x64_64.restype = U64
        L.orc_murmur3_x64_128.argtypes = [VP, C.c_uint32, C.c_uint32, VP]
        L.orc_murmur3_x64_128.restype = None
        L.orc_quick_hash.argtypes = [U64]
        L.orc_quick_hash.restype = U64
        L.orc_kmer_from_string.argtypes = [C.c_char_p, I, I, VP]
        L.orc_kmer_from_string.restype = None
        L.orc_kmer_to_string.argtypes = [VP, I, C.c_char_p]
        L.orc_kmer_to_string.restype = None
        L.orc_kmer_revcomp.argtypes = [VP, I, I, VP]
        L.orc_kmer_revcomp.restype = None
        L.orc_kmer_hash.argtypes = [VP, I]
        L.orc_kmer_hash.restype = U64
        L.orc_get_minimizer_fast.argtypes = [VP, I, I, I, I]
        L.orc_get_minimizer_fast.restype = U64
        L.orc_minimizer_hash_fast.argtypes = [VP, I, I, I]
        L.orc_minimizer_hash_fast.restype = U64
        L.orc_minimizer_len.argtypes = [I]
        L.orc_kmer_target_rank.argtypes = [VP, I, I, I]
        L.orc_kcount.argtypes = [VP, VP, U64, I, I, I, I, C.c_double]
        L.orc_kcount.restype = VP
        L.orc_kcount_mt.argtypes = [VP, VP, U64, I, I, I, I, C.c_double, I]
        L.orc_kcount_mt.restype = VP
        L.orc_kcount_mt_range.argtypes = [VP, VP, U64, I, I, I, I, C.c_double, I, I, I]
        L.orc_kcount_mt_range.restype = VP
        L.orc_kcount_mt_ctgs_range.argtypes = [VP, VP, U64, C.c_char_p, VP, VP, U64, I, I, I, I, C.c_double, I, I, I]
        L.orc_kcount_mt_ctgs_range.restype = VP
        L.orc_kcount_mt_digests.argtypes = [VP, VP, U64, I, I, I, C.c_double, I, I, I, I, VP]
        L.orc_kcount_mt_digests.restype = I
        L.orc_fp_digests.argtypes = [VP, VP, U64, I, VP]
        L.orc_fp_digests.restype = None
        L.orc_mt_ranges.argtypes = [VP, U64, I, I, I, VP]
        L.orc_mt_ranges.restype = None
        L.orc_row_fingerprints.argtypes = [VP, VP, VP, VP, U64, I, I, VP]
        L.orc_row_fingerprints.restype = None
        L.orc_kmer_target_ranks.argtypes = [VP, U64, I, I, I, I, VP]
        L.orc_kmer_target_ranks.restype = None
        L.orc_kcount_ctgs.argtypes = [VP, VP, U64, VP, VP, VP, U64, I, I, I, I, C.c_double]
        L.orc_kcount_ctgs.restype = VP
        L.orc_extract.argtypes = [VP, VP, U64, I, I, I, VP, VP, U64]
        L.orc_extract.restype = C.c_int64
        L.orc_count_records.argtypes = [VP, VP, U64, I, I, C.c_double]
        L.orc_count_records.restype = VP
        L.orc_fastq_pack.argtypes = [C.c_char_p, U64, I, VP, VP, VP]
        L.orc_fastq_pack.restype = C.c_int64
        L.orc_merge_fastq.argtypes = [C.c_char_p, U64, I, VP, VP, VP, VP]
        L.orc_merge_fastq.restype = C.c_int64
        L.orc_table_size.argtypes = [VP]
        L.orc_table_size.restype = U64
        L.orc_table_fetch.argtypes = [VP, VP, VP, VP, VP]
        L.orc_table_fetch.restype = None
        L.orc_table_stats.argtypes = [VP, VP]
        L.orc_table_stats.restype = None
        L.orc_table_free.argtypes = [VP]
        L.orc_table_free.restype = None
        _o = L
    return _o


def hashref():
    """The reference's compiled hash_funcs.c, or None when oracle/_ref was not built."""
    if not HASHREF.exists():
        return None
    L = C.CDLL(str(HASHREF))
    L.MurmurHash3_x64_64.argtypes = [C.c_void_p, C.c_uint32]
    L.MurmurHash3_x64_64.restype = C.c_uint64
    L.MurmurHash3_x64_128.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p]
    L.MurmurHash3_x64_128.restype = None
    L.quick_hash.argtypes = [C.c_uint64]
    L.quick_hash.restype = C.c_uint64
    return L


class OracleTable:
    def __init__(self, ptr, n_longs, k):
        if not ptr:
            raise ValueError("oracle rejected the input (the reference would DIE)")
        self.ptr, self.n_longs, self.k = ptr, n_longs, k

    def fetch(self):
        L = oracle()
        n = L.orc_table_size(self.ptr)
        keys = np.empty((n, self.n_longs), dtype=np.uint64)
        counts = np.empty(n, dtype=np.uint16)
        left = np.empty(n, dtype=np.uint8)
        right = np.empty(n, dtype=np.uint8)
        L.orc_table_fetch(self.ptr, keys.ctypes.data, counts.ctypes.data, left.ctypes.data, right.ctypes.data)
        return keys, counts, left, right

    def stats(self) -> dict:
        s = np.zeros(5, dtype=np.uint64)
        oracle().orc_table_stats(self.ptr, s.ctypes.data)
        return dict(occurrences=int(s[0]), distinct=int(s[1]), purged=int(s[2]), n_out=int(s[3]), reads=int(s[4]))

    def __del__(self):
        if getattr(self, "ptr", None):
            oracle().orc_table_free(self.ptr)
            self.ptr = None


def kcount(packed_bytes, offsets, k, n_longs=None, qual_cutoff=20, dmin_thres=2, dyn_min_depth=0.9) -> OracleTable:
    nl = n_longs or (k // 32 + 1)
    b = np.ascontiguousarray(packed_bytes, dtype=np.uint8)
    o = np.ascontiguousarray(offsets, dtype=np.uint64)
    ptr = oracle().orc_kcount(b.ctypes.data, o.ctypes.data, o.size - 1, k, nl, qual_cutoff, dmin_thres,
                              dyn_min_depth)
    return OracleTable(ptr, nl, k)


def kcount_mt(packed_bytes, offsets, k, n_longs=None, qual_cutoff=20, dmin_thres=2, dyn_min_depth=0.9,
              threads=8) -> OracleTable:
    """The multi-threaded restatement (oracle/kcount_mt.c); rows in no particular order."""
    nl = n_longs or (k // 32 + 1)
    b = np.ascontiguousarray(packed_bytes, dtype=np.uint8)
    o = np.ascontiguousarray(offsets, dtype=np.uint64)
    ptr = oracle().orc_kcount_mt(b.ctypes.data, o.ctypes.data, o.size - 1, k, nl, qual_cutoff, dmin_thres,
                                 dyn_min_depth, threads)
    return OracleTable(ptr, nl, k)


def kcount_mt_range(packed_bytes, offsets, k, part, n_parts, threads=8, qual_cutoff=20, dmin_thres=2,
                    dyn_min_depth=0.9) -> OracleTable:
    """Part `part` of n_parts of the multi-threaded restatement's table (the k-mers whose mt_range is `part`,
    oracle/kcount_mt.c): a table too large for host memory is built and checked one part at a time."""
    nl = k // 32 + 1
    b = np.ascontiguousarray(packed_bytes, dtype=np.uint8)
    o = np.ascontiguousarray(offsets, dtype=np.uint64)
    ptr = oracle().orc_kcount_mt_range(b.ctypes.data, o.ctypes.data, o.size - 1, k, nl, qual_cutoff, dmin_thres,
                                       dyn_min_depth, threads, part, n_parts)
    return OracleTable(ptr, nl, k)


MT_DIG = 6  # digest words per key range (oracle/kcount_mt.c): rows, xor, sum, sum of fmix, distinct, occurrences


def kcount_mt_digests(packed_bytes, offsets, k, part0, n_sel, n_parts, threads=8, qual_cutoff=20, dmin_thres=2,
                      dyn_min_depth=0.9) -> np.ndarray:
    """Row-fingerprint digests of the restatement's key-range parts [part0, part0 + n_sel) of n_parts, from one pass
    over the reads (oracle/kcount_mt.c orc_kcount_mt_digests): (n_sel, MT_DIG) uint64."""
    b = np.ascontiguousarray(packed_bytes, dtype=np.uint8)
    o = np.ascontiguousarray(offsets, dtype=np.uint64)
    out = np.zeros((n_sel, MT_DIG), dtype=np.uint64)
    rc = oracle().orc_kcount_mt_digests(b.ctypes.data, o.ctypes.data, o.size - 1, k, qual_cutoff, dmin_thres,
                                        dyn_min_depth, threads, part0, n_sel, n_parts, out.ctypes.data)
    if rc != 0:
        raise RuntimeError("orc_kcount_mt_digests failed (bad input or out of memory)")
    return out


def fp_digests(fps, parts, n_parts) -> np.ndarray:
    """The same digests of row fingerprints fps by their key-range parts (mt_ranges): (n_parts, MT_DIG) uint64, the
    distinct and occurrence words 0."""
    f = np.ascontiguousarray(fps, dtype=np.uint64)
    p = np.ascontiguousarray(parts, dtype=np.uint8)
    out = np.zeros((n_parts, MT_DIG), dtype=np.uint64)
    oracle().orc_fp_digests(f.ctypes.data, p.ctypes.data, f.size, n_parts, out.ctypes.data)
    return out


FP_CHAIN0 = 0x243F6A8885A308D3


def _fmix(x):
    m = (1 << 64) - 1
    x ^= x >> 33
    x = (x * 0xff51afd7ed558ccd) & m
    x ^= x >> 33
    x = (x * 0xc4ceb9fe1a85ec53) & m
    return x ^ (x >> 33)


def _fmix_inv(x):
    m = (1 << 64) - 1
    x ^= x >> 33  # (x >> 33 >> 33 == 0: an xor-shift by 33 is its own inverse on 64 bits)
    x = (x * pow(0xc4ceb9fe1a85ec53, -1, 1 << 64)) & m
    x ^= x >> 33
    x = (x * pow(0xff51afd7ed558ccd, -1, 1 << 64)) & m
    return x ^ (x >> 33)


def fp_row_values(fp, key_words):
    """(count, left, right) of the row whose fingerprint is fp if its key is key_words (orc_row_fingerprints inverted:
    the final fmix undone and the key's chain removed), else None."""
    h = FP_CHAIN0
    for w in key_words:
        h = (_fmix(h ^ int(w)) + 0x9E3779B97F4A7C15) & ((1 << 64) - 1)
    v = _fmix_inv(int(fp)) ^ h
    if v >> 32:
        return None
    return v & 0xFFFF, chr((v >> 16) & 0xFF), chr((v >> 24) & 0xFF)


def mt_ranges(keys, k, n_parts):
    """The kcount_mt_range part of every row of an (n, n_longs) key array."""
    kk = np.ascontiguousarray(keys, dtype=np.uint64)
    out = np.empty(kk.shape[0], dtype=np.uint8)
    oracle().orc_mt_ranges(kk.ctypes.data, kk.shape[0], kk.shape[1] if kk.ndim == 2 else 1, k // 32 + 1, n_parts,
                           out.ctypes.data)
    return out


def row_fingerprints(keys, counts, left, right, k):
    """A 64-bit fingerprint of every (key, count, left, right) row (oracle/kcount_mt.c orc_row_fingerprints)."""
    kk = np.ascontiguousarray(keys, dtype=np.uint64)
    c = np.ascontiguousarray(counts, dtype=np.uint16)
    lft = np.ascontiguousarray(left).view(np.uint8)
    rgt = np.ascontiguousarray(right).view(np.uint8)
    out = np.empty(kk.shape[0], dtype=np.uint64)
    oracle().orc_row_fingerprints(kk.ctypes.data, c.ctypes.data, lft.ctypes.data, rgt.ctypes.data, kk.shape[0],
                                  kk.shape[1] if kk.ndim == 2 else 1, k // 32 + 1, out.ctypes.data)
    return out


def target_ranks(keys, k, rank_n):
    """KmerDHT::get_kmer_target_rank of every row (oracle restatement, src/kcount/kmer_dht.cpp:193-196)."""
    kk = np.ascontiguousarray(keys, dtype=np.uint64)
    out = np.empty(kk.shape[0], dtype=np.uint8)
    oracle().orc_kmer_target_ranks(kk.ctypes.data, kk.shape[0], kk.shape[1] if kk.ndim == 2 else 1, k, k // 32 + 1,
                                   rank_n, out.ctypes.data)
    return out


def kcount_ctgs(packed_bytes, offsets, ctg_seqs, ctg_depths, k, n_longs=None, qual_cutoff=20, dmin_thres=2,
                dyn_min_depth=0.9) -> OracleTable:
    """Read pass + contig pass (add_ctg_kmers) + finalize. ctg_seqs: list of str; ctg_depths: uint16 values."""
    nl = n_longs or (k // 32 + 1)
    b = np.ascontiguousarray(packed_bytes, dtype=np.uint8)
    o = np.ascontiguousarray(offsets, dtype=np.uint64)
    blob = "".join(ctg_seqs).encode("ascii")
    co = np.zeros(len(ctg_seqs) + 1, dtype=np.uint64)
    np.cumsum([len(x) for x in ctg_seqs], out=co[1:])
    d = np.ascontiguousarray(ctg_depths, dtype=np.uint16)
    ptr = oracle().orc_kcount_ctgs(b.ctypes.data, o.ctypes.data, o.size - 1, blob, co.ctypes.data, d.ctypes.data,
                                   len(ctg_seqs), k, nl, qual_cutoff, dmin_thres, dyn_min_depth)
    return OracleTable(ptr, nl, k)


def kcount_mt_ctgs(packed_bytes, offsets, ctg_blob: bytes, ctg_offs, ctg_depths, k, threads=8, part=0, n_parts=1,
                   qual_cutoff=20, dmin_thres=2, dyn_min_depth=0.9) -> OracleTable:
    """The multi-threaded restatement with the contig pass (oracle/kcount_mt.c orc_kcount_mt_ctgs_range): contigs
    back to back in ctg_blob (ASCII, case = quality), ctg_offs their n + 1 offsets, in the order they are applied."""
    nl = k // 32 + 1
    b = np.ascontiguousarray(packed_bytes, dtype=np.uint8)
    o = np.ascontiguousarray(offsets, dtype=np.uint64)
    co = np.ascontiguousarray(ctg_offs, dtype=np.uint64)
    d = np.ascontiguousarray(ctg_depths, dtype=np.uint16)
    ptr = oracle().orc_kcount_mt_ctgs_range(b.ctypes.data, o.ctypes.data, o.size - 1, ctg_blob, co.ctypes.data,
                                            d.ctypes.data, d.size, k, nl, qual_cutoff, dmin_thres, dyn_min_depth,
                                            threads, part, n_parts)
    return OracleTable(ptr, nl, k)


def extract(packed_bytes, offsets, k, n_longs=None, qual_cutoff=20):
    nl = n_longs or (k // 32 + 1)
    b = np.ascontiguousarray(packed_bytes, dtype=np.uint8)
    o = np.ascontiguousarray(offsets, dtype=np.uint64)
    lens = np.diff(o.astype(np.int64))
    cap = int(np.clip(lens - k - 1, 0, None).sum()) + 1
    keys = np.empty((cap, nl), dtype=np.uint64)
    exts = np.empty(cap, dtype=np.uint8)
    n = oracle().orc_extract(b.ctypes.data, o.ctypes.data, o.size - 1, k, nl, qual_cutoff, keys.ctypes.data,
                             exts.ctypes.data, cap)
    if n < 0:
        raise ValueError("oracle extract failed")
    return keys[:n], exts[:n]


def count_records(keys, exts, k, n_longs=None, dmin_thres=2, dyn_min_depth=0.9) -> OracleTable:
    nl = n_longs or (k // 32 + 1)
    kk = np.ascontiguousarray(keys, dtype=np.uint64)
    ee = np.ascontiguousarray(exts, dtype=np.uint8)
    ptr = oracle().orc_count_records(kk.ctypes.data, ee.ctypes.data, ee.size, nl, dmin_thres, dyn_min_depth)
    return OracleTable(ptr, nl, k)


def kmer_hash(longs) -> int:
    a = np.ascontiguousarray(longs, dtype=np.uint64)
    return int(oracle().orc_kmer_hash(a.ctypes.data, a.size))


def kmer_from_string(s: str, n_longs: int) -> np.ndarray:
    a = np.zeros(n_longs, dtype=np.uint64)
    oracle().orc_kmer_from_string(s.encode(), len(s), n_longs, a.ctypes.data)
    return a


def kmer_to_string(longs, k: int) -> str:
    a = np.ascontiguousarray(longs, dtype=np.uint64)
    buf = C.create_string_buffer(k + 1)
    oracle().orc_kmer_to_string(a.ctypes.data, k, buf)
    return buf.value.decode()


def kmer_revcomp(longs, k: int) -> np.ndarray:
    a = np.ascontiguousarray(longs, dtype=np.uint64)
    out = np.zeros_like(a)
    oracle().orc_kmer_revcomp(a.ctypes.data, k, a.size, out.ctypes.data)
    return out


def minimizer_fast(longs, k: int, m: int, least_complement: bool = True) -> int:
    a = np.ascontiguousarray(longs, dtype=np.uint64)
    return int(oracle().orc_get_minimizer_fast(a.ctypes.data, k, a.size, m, 1 if least_complement else 0))


def minimizer_hash_fast(longs, k: int, m: int) -> int:
    a = np.ascontiguousarray(longs, dtype=np.uint64)
    return int(oracle().orc_minimizer_hash_fast(a.ctypes.data, k, a.size, m))


def target_rank(longs, k: int, rank_n: int) -> int:
    a = np.ascontiguousarray(longs, dtype=np.uint64)
    return int(oracle().orc_kmer_target_rank(a.ctypes.data, k, a.size, rank_n))


FQ_KINDS = {1: "id", 2: "plus", 3: "name", 4: "len", 5: "long", 6: "char", 7: "trunc", 8: "pair_name",
            9: "pair_number", 10: "qual"}


def fastq_pack(text: bytes, qual_offset: int = 33):
    """FASTQ text -> (PackedRead bytes, offsets), or raises FastqError(kind, record) where the reference
    DIEs (orc_fastq_pack: FastqReader::get_next_fq_record + PackedRead ctor)."""
    n = len(text)
    out = np.empty(max(n, 1), dtype=np.uint8)
    offs = np.empty(n // 6 + 2, dtype=np.uint64)
    err = np.zeros(1, dtype=np.uint64)
    r = oracle().orc_fastq_pack(text, n, qual_offset, out.ctypes.data, offs.ctypes.data, err.ctypes.data)
    if r < 0:
        raise FastqError(FQ_KINDS[-r], int(err[0]))
    return out[: int(offs[r])].copy(), offs[: r + 1].copy()


def merge_fastq(text: bytes, qual_offset: int = 33):
    """Interleaved paired FASTQ text -> merge_reads' PackedReads (merged read + "N" mate, or both mates) as
    (bytes, offsets, stats {pairs, merged, ambiguous, overlap_bases}), or raises FastqError where the reference
    DIEs (orc_merge_fastq: merge_reads.cpp:237-588 + PackedRead ctor)."""
    n = len(text)
    out = np.empty(max(n, 1), dtype=np.uint8)
    offs = np.empty(n // 6 + 4, dtype=np.uint64)
    stats = np.zeros(4, dtype=np.uint64)
    err = np.zeros(1, dtype=np.uint64)
    r = oracle().orc_merge_fastq(text, n, qual_offset, out.ctypes.data, offs.ctypes.data, stats.ctypes.data,
                                 err.ctypes.data)
    if r < 0:
        raise FastqError(FQ_KINDS[-r], int(err[0]))
    st = dict(zip(("pairs", "merged", "ambiguous", "overlap_bases"), (int(x) for x in stats)))
    return out[: int(offs[r])].copy(), offs[: r + 1].copy(), st


class FastqError(ValueError):
    def __init__(self, kind: str, record: int):
        super().__init__(f"{kind} at record {record}")
        self.kind = kind
        self.record = record
