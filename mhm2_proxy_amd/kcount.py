"""Host-side mirror of the reference kcount interface over the C ABI of libmhmkc.so.

Reference shapes kept (ajpowelsnl/mhm2_proxy):
  * PackedRead / PackedReads        src/packed_reads.hpp:60-167, src/packed_reads.cpp:73-159
  * Kmer<MAX_K> longs layout        src/kmer.hpp:61-160 (here: a tuple/array of n_longs uint64)
  * KmerCounts{count, left, right}  src/kcount/kmer_dht.hpp:62-68
  * KmerDHT (local_kmers, get_local_kmer_counts, get_kmer_target_rank, dump_kmers)
                                    src/kcount/kmer_dht.hpp:118-172, src/kcount/kmer_dht.cpp
  * analyze_kmers(...)              src/kcount/kcount.hpp:71-73, src/kcount/kcount.cpp:140-157

The counting itself always runs on the GPU through libmhmkc.so; nothing here falls back to the CPU.
"""
from __future__ import annotations

import ctypes as C
import gzip
import os
from dataclasses import dataclass
from pathlib import Path
from typing import Iterable, NamedTuple, Sequence

import numpy as np

from . import _native as N

NUCLEOTIDE_MAP = "ACGTN"
_BASE_CODE = {"A": 0, "C": 1, "G": 2, "T": 3, "N": 4}
_IUPAC = set("URYKMSWBDHV")  # mapped to N by the PackedRead constructor (packed_reads.cpp:90-101)


def n_longs_for(k: int) -> int:
    """N_LONGS of Kmer<MAX_K> with MAX_K = (k/32+1)*32 (src/main.cpp:170, src/kmer.hpp:64)."""
    return k // 32 + 1


# ------------------------------------------------------------------------------------------------
# Kmer helpers (2-bit MSB-first longs, src/kmer.cpp:178-188)


def kmer_from_string(s: str, n_longs: int | None = None) -> tuple:
    """set_kmer (src/kmer.cpp:274-296): A0 C1 G2 T3, the bit trick maps N to G."""
    k = len(s)
    nl = n_longs or n_longs_for(k)
    longs = [0] * nl
    for i, ch in enumerate(s):
        c = ord(ch)
        x = (c & 4) >> 1
        code = x + ((x ^ (c & 2)) >> 1)
        longs[i // 32] |= code << (2 * (31 - i % 32))
    return tuple(longs)


def kmer_to_string(longs: Sequence[int], k: int) -> str:
    """to_string (src/kmer.cpp:595-634)."""
    return "".join("ACGT"[(int(longs[i // 32]) >> (2 * (31 - i % 32))) & 3] for i in range(k))


def keys_to_strings(keys: np.ndarray, k: int) -> list:
    """Vectorised to_string for an (n, n_longs) uint64 key array."""
    keys = np.asarray(keys, dtype=np.uint64)
    n = keys.shape[0]
    out = np.empty((n, k), dtype=np.uint8)
    lut = np.frombuffer(b"ACGT", dtype=np.uint8)
    for i in range(k):
        w = keys[:, i // 32]
        out[:, i] = lut[((w >> np.uint64(2 * (31 - i % 32))) & np.uint64(3)).astype(np.intp)]
    return [bytes(r).decode() for r in out]


# ------------------------------------------------------------------------------------------------
# PackedReads


class PackedReads:
    """Reads in the PackedRead byte layout: one byte per base, code (A0 C1 G2 T3 N4) | min(q-off,31) << 3.

    Mirrors src/packed_reads.hpp:120-167. Reads are stored contiguously (bytes + CSR offsets) so the
    whole set can be handed to the device in one copy.
    """

    def __init__(self, qual_offset: int = 33, fname: str = ""):
        if qual_offset not in (33, 64):
            raise ValueError("qual_offset must be 33 or 64")
        self.qual_offset = qual_offset
        self.fname = fname
        self._chunks: list[np.ndarray] = []
        self._lens: list[int] = []
        self._ids: list[int] = []
        self._bytes: np.ndarray | None = None
        self._offsets: np.ndarray | None = None
        self.index = 0
        self.max_read_len = 0

    @classmethod
    def from_arrays(cls, packed_bytes: np.ndarray, offsets: np.ndarray, qual_offset: int = 33) -> "PackedReads":
        pr = cls(qual_offset)
        pr._bytes = np.ascontiguousarray(packed_bytes, dtype=np.uint8)
        pr._offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        if pr._offsets.size == 0 or pr._offsets[0] != 0 or int(pr._offsets[-1]) != pr._bytes.size:
            raise ValueError("offsets must start at 0 and end at len(bytes)")
        lens = np.diff(pr._offsets)
        pr.max_read_len = int(lens.max()) if lens.size else 0
        return pr

    @staticmethod
    def pack(seq: str, quals: str, qual_offset: int = 33) -> np.ndarray:
        """PackedRead constructor encoding (src/packed_reads.cpp:73-109); raises on illegal characters
        (the reference DIEs)."""
        if len(seq) != len(quals):
            raise ValueError("seq and quals differ in length")
        if len(seq) > 65535:
            raise ValueError("read longer than 65535 (read_len is uint16)")
        out = np.empty(len(seq), dtype=np.uint8)
        for i, (ch, q) in enumerate(zip(seq, quals)):
            if ch in _BASE_CODE:
                code = _BASE_CODE[ch]
            elif ch in _IUPAC:
                code = 4
            else:
                raise ValueError(f"Illegal char in comp nucleotide of '{ch}'")
            qq = min(ord(q) - qual_offset, 31)
            out[i] = (code | ((qq & 0xFF) << 3)) & 0xFF
        return out

    def add_read(self, read_id: str, seq: str, quals: str) -> None:
        """PackedReads::add_read (src/packed_reads.cpp:236-244)."""
        if self._bytes is not None:
            self._materialized_to_chunks()
        self._chunks.append(self.pack(seq, quals, self.qual_offset))
        self._lens.append(len(seq))
        self.max_read_len = max(self.max_read_len, len(seq))

    def _materialized_to_chunks(self):
        b, o = self._bytes, self._offsets
        self._chunks = [b[o[i]:o[i + 1]] for i in range(len(o) - 1)]
        self._lens = [int(o[i + 1] - o[i]) for i in range(len(o) - 1)]
        self._bytes = self._offsets = None

    def _materialize(self):
        if self._bytes is None:
            lens = np.asarray(self._lens, dtype=np.uint64)
            self._offsets = np.zeros(len(lens) + 1, dtype=np.uint64)
            np.cumsum(lens, out=self._offsets[1:])
            self._bytes = (np.concatenate(self._chunks) if self._chunks else np.zeros(0, np.uint8)).astype(np.uint8)
            self._chunks, self._lens = [], []

    @property
    def packed_bytes(self) -> np.ndarray:
        self._materialize()
        return self._bytes

    @property
    def offsets(self) -> np.ndarray:
        self._materialize()
        return self._offsets

    def get_local_num_reads(self) -> int:
        return len(self.offsets) - 1

    def get_bases(self) -> int:
        return int(self.offsets[-1])

    def get_max_read_len(self) -> int:
        return self.max_read_len

    def reset(self) -> None:
        self.index = 0

    def get_read(self, i: int) -> tuple[str, str, str]:
        """PackedRead::unpack (src/packed_reads.cpp:147-159); ids are synthetic '@r<i>/1'."""
        b = self.packed_bytes[int(self.offsets[i]):int(self.offsets[i + 1])]
        seq = "".join(NUCLEOTIDE_MAP[int(x) & 7] for x in b)
        quals = "".join(chr(self.qual_offset + (int(x) >> 3)) for x in b)
        return f"@r{i}/1", seq, quals

    def get_next_read(self):
        if self.index >= self.get_local_num_reads():
            return None
        r = self.get_read(self.index)
        self.index += 1
        return r


# ------------------------------------------------------------------------------------------------
# The counter (C ABI wrapper)


class KmerCounts(NamedTuple):
    """KmerCounts (src/kcount/kmer_dht.hpp:62-68) without the dbjg-only uutig_frag pointer."""
    count: int
    left: str
    right: str


@dataclass
class KmerTable:
    """Finished count table on the host: keys (n, n_longs) uint64, counts uint16, left/right bytes."""
    k: int
    keys: np.ndarray
    counts: np.ndarray
    left: np.ndarray
    right: np.ndarray

    def __len__(self) -> int:
        return int(self.counts.shape[0])

    def sorted(self) -> "KmerTable":
        """Rows in Kmer::operator< order (word-wise unsigned, src/kmer.cpp:265-272)."""
        if len(self) == 0:
            return self
        order = np.lexsort(tuple(self.keys[:, w] for w in range(self.keys.shape[1] - 1, -1, -1)))
        return KmerTable(self.k, self.keys[order], self.counts[order], self.left[order], self.right[order])

    def lines(self) -> Iterable[str]:
        """dump_kmers line format "KMER count L R" (src/kcount/kmer_dht.cpp:243-266)."""
        strs = keys_to_strings(self.keys, self.k)
        for s, c, l, r in zip(strs, self.counts, self.left, self.right):
            yield f"{s} {int(c)} {chr(int(l))} {chr(int(r))}"


class KmerCounter:
    """One GPU's k-mer counter; wraps mhmkc_* (include/mhmkc.h).

    The lifecycle mirrors HashTableInserter (src/kcount/kmer_dht.hpp:95-116): construct (init), add reads
    (insert_supermer via process_seq), finish (flush_inserts + insert_into_local_hashtable), fetch.
    """

    def __init__(self, k: int, *, n_longs: int = 0, qual_offset: int = 33, qual_cutoff: int = 20,
                 dmin_thres: int = 2, dyn_min_depth: float = 0.9, device: int = -1, rank: int = 0,
                 n_ranks: int = 1, comm_id: bytes | None = None, stream: int | None = None,
                 transport: "TorchDistTransport | None" = None, output_owner: int = N.MHMKC_OWNER_HASH,
                 minimizer_len: int = 0):
        L = N.lib()
        cfg = N.MhmkcConfig()
        N.check(L.mhmkc_config_init(C.byref(cfg)))
        cfg.k, cfg.n_longs, cfg.qual_offset, cfg.qual_cutoff = k, n_longs, qual_offset, qual_cutoff
        cfg.dmin_thres, cfg.dyn_min_depth, cfg.device = dmin_thres, dyn_min_depth, device
        cfg.rank, cfg.n_ranks = rank, n_ranks
        cfg.output_owner, cfg.minimizer_len = output_owner, minimizer_len
        self._comm_buf = None
        if comm_id is not None:
            if len(comm_id) != N.MHMKC_COMM_ID_BYTES:
                raise ValueError("comm_id must be 128 bytes")
            self._comm_buf = C.create_string_buffer(bytes(comm_id), N.MHMKC_COMM_ID_BYTES)
            cfg.comm_id = C.cast(self._comm_buf, C.c_void_p)
        cfg.stream = stream
        h = C.c_void_p()
        N.check(L.mhmkc_create(C.byref(h), C.byref(cfg)))
        self._h = h
        self.k = k
        self.n_longs = n_longs or n_longs_for(k)
        self.rank, self.n_ranks = rank, n_ranks
        self.n_out = None
        self._transport = None
        if transport is not None:
            self.set_transport(transport)

    # -- lifecycle
    def close(self) -> None:
        if getattr(self, "_h", None):
            N.lib().mhmkc_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int) -> None:
        N.check(rc, self._h)

    # -- input
    def add_packed_reads(self, packed_bytes: np.ndarray, offsets: np.ndarray) -> None:
        b = np.ascontiguousarray(packed_bytes, dtype=np.uint8)
        o = np.ascontiguousarray(offsets, dtype=np.uint64)
        if o.size < 1:
            raise ValueError("offsets needs n_reads + 1 entries")
        self._check(N.lib().mhmkc_add_reads(self._h, b.ctypes.data, o.ctypes.data, o.size - 1))

    def add_packed_reads_device(self, bytes_ptr: int, offsets_ptr: int, n_reads: int, n_bases: int) -> None:
        self._check(N.lib().mhmkc_add_reads_device(self._h, bytes_ptr, offsets_ptr, n_reads, n_bases))

    def wait_stream(self, stream_ptr: int | None) -> None:
        """Order the counter's device work after what is enqueued on another stream (mhmkc_wait_stream)."""
        self._check(N.lib().mhmkc_wait_stream(self._h, stream_ptr))

    def _after_torch(self, t) -> None:
        """Device tensors are read on the counter's own stream: order it after torch's current stream."""
        import torch

        self.wait_stream(torch.cuda.current_stream(t.device).cuda_stream)

    def add_tensors(self, bytes_t, offsets_t, n_bases: int | None = None) -> None:
        """Device-resident torch tensors (uint8 bytes, int64/uint64 offsets with n_reads+1 entries). n_bases
        defaults to offsets_t[-1] (one device read); the library checks the offsets on the device."""
        n_reads = int(offsets_t.numel()) - 1
        if n_bases is None:
            n_bases = int(offsets_t[-1]) if n_reads >= 0 else 0
        if n_bases > int(bytes_t.numel()):
            raise ValueError("offsets_t[-1] exceeds the bytes tensor")
        self._after_torch(bytes_t)
        self.add_packed_reads_device(bytes_t.data_ptr(), offsets_t.data_ptr(), n_reads, n_bases)

    def add_fastq(self, text) -> None:
        """FASTQ text (bytes or str), parsed and packed on the device, then counted: FastqReader +
        PackedRead construction (src/fastq.cpp:504-551, src/packed_reads.cpp:73-109) for reads that reach
        kcount unmerged. Malformed input raises MhmkcError where the reference DIEs."""
        blob = text.encode("ascii") if isinstance(text, str) else bytes(text)
        self._check(N.lib().mhmkc_add_fastq(self._h, blob, len(blob)))

    def add_fastq_pairs(self, text) -> None:
        """Interleaved paired FASTQ text (mates /1, /2 back to back), parsed on the device, the pairs merged as
        merge_reads does (src/merge_reads.cpp:237-588: merged read + dummy "N" mate, or both mates), then
        counted. stats() reports fq_pairs / fq_merged / fq_ambiguous / fq_overlap_bases; fastq_packed() returns
        merge_reads' PackedReads."""
        blob = text.encode("ascii") if isinstance(text, str) else bytes(text)
        self._check(N.lib().mhmkc_add_fastq_pairs(self._h, blob, len(blob)))

    def add_fastq_file(self, path, pairs: bool = False) -> None:
        """A FASTQ file (interleaved pairs with pairs=True) read in blocks into pinned memory, each block parsed
        and counted on the device while the next is read (mhmkc_add_fastq_file: the file I/O overlapped with the
        kernels). Block size: MHMKC_FQ_BLOCK bytes (default 256 MB). fastq_packed() then holds the PackedReads of
        the whole file (for the later k rounds, as the reference keeps packed_reads_list)."""
        fn = N.lib().mhmkc_add_fastq_pairs_file if pairs else N.lib().mhmkc_add_fastq_file
        self._check(fn(self._h, os.fsencode(str(path))))

    def add_fastq_tensor(self, text_t, n_bytes: int | None = None, pairs: bool = False) -> None:
        """FASTQ text already in HBM (a uint8 torch tensor on the counter's device). The parser reads whole
        aligned dwords, so the buffer must extend 4 bytes past the text: pass n_bytes <= numel - 4 to use the
        tensor as is; otherwise the text is copied into a padded buffer first."""
        import torch

        n = int(text_t.numel()) if n_bytes is None else int(n_bytes)
        if int(text_t.numel()) < n + 4:
            padded = torch.zeros(n + 16, dtype=torch.uint8, device=text_t.device)
            padded[:n].copy_(text_t.reshape(-1)[:n])
            text_t = padded
        self._fq_text = text_t  # keep it alive while the call runs
        self._after_torch(text_t)
        fn = N.lib().mhmkc_add_fastq_pairs_device if pairs else N.lib().mhmkc_add_fastq_device
        self._check(fn(self._h, text_t.data_ptr(), n))

    def fastq_packed(self) -> tuple[np.ndarray, np.ndarray]:
        """The PackedReads (bytes, offsets) of the last add_fastq call, copied to the host."""
        n_reads, n_bases = C.c_uint64(), C.c_uint64()
        self._check(N.lib().mhmkc_fastq_packed(self._h, None, None, C.byref(n_reads), C.byref(n_bases)))
        b = np.empty(int(n_bases.value), dtype=np.uint8)
        o = np.empty(int(n_reads.value) + 1, dtype=np.uint64)
        self._check(N.lib().mhmkc_fastq_fetch(self._h, b.ctypes.data, o.ctypes.data))
        return b, o

    def add_reads(self, reads: PackedReads) -> None:
        self.add_packed_reads(reads.packed_bytes, reads.offsets)

    def add_seqs(self, seqs: Sequence[str], depth: int = 1) -> None:
        """Sequences whose lowercase letters mark bases below the quality cutoff (the string given to
        SeqBlockInserter::process_seq, src/kcount/kcount.cpp:80-86)."""
        lens = np.fromiter((len(s) for s in seqs), dtype=np.uint64, count=len(seqs))
        offs = np.zeros(len(seqs) + 1, dtype=np.uint64)
        np.cumsum(lens, out=offs[1:])
        blob = "".join(seqs).encode("ascii")
        self._check(N.lib().mhmkc_add_seqs(self._h, blob, offs.ctypes.data, len(seqs), depth))

    def add_ctgs(self, seqs: Sequence[str], depths) -> None:
        """Contigs for the contig pass (add_ctg_kmers, src/kcount/kcount.cpp:100-138): uint16 depths as
        Contig::get_uint16_t_depth() gives them (src/contigs.hpp:65). Applied at finish, after the reads,
        in the order added."""
        d = np.ascontiguousarray(depths, dtype=np.uint16)
        if d.size != len(seqs):
            raise ValueError("one depth per contig")
        lens = np.fromiter((len(s) for s in seqs), dtype=np.uint64, count=len(seqs))
        offs = np.zeros(len(seqs) + 1, dtype=np.uint64)
        np.cumsum(lens, out=offs[1:])
        blob = "".join(seqs).encode("ascii")
        self._check(N.lib().mhmkc_add_ctgs(self._h, blob, offs.ctypes.data, d.ctypes.data, len(seqs)))

    # -- ranks, thresholds
    def set_transport(self, transport: "TorchDistTransport") -> None:
        """Host-staged exchange between ranks (mhmkc_set_transport), e.g. over a gloo process group."""
        self._transport = transport  # the callbacks must outlive the handle
        self._check(N.lib().mhmkc_set_transport(self._h, C.byref(transport.struct)))

    def set_dmin_thres(self, dmin_thres: int) -> None:
        """The finish's depth threshold, the reference's _dmin_thres (src/kcount/kmer_dht.hpp:57), set by
        analyze_kmers (src/kcount/kcount.cpp:145)."""
        self._check(N.lib().mhmkc_set_dmin_thres(self._h, int(dmin_thres)))

    def minimizer_hashes(self, keys: np.ndarray, m: int = 0) -> np.ndarray:
        """Kmer::minimizer_hash_fast of (n, n_longs) keys, on the GPU (src/kmer.cpp:344-393,454-463)."""
        kk = np.ascontiguousarray(keys, dtype=np.uint64)
        if kk.ndim == 1:
            kk = kk.reshape(-1, 1)
        out = np.empty(kk.shape[0], dtype=np.uint64)
        self._check(N.lib().mhmkc_minimizer_hashes(self._h, kk.ctypes.data, kk.shape[0], kk.shape[1], m,
                                                   out.ctypes.data))
        return out

    def target_ranks(self, keys: np.ndarray, rank_n: int) -> np.ndarray:
        """KmerDHT::get_kmer_target_rank of every key (src/kcount/kmer_dht.cpp:193-196), on the GPU."""
        return (self.minimizer_hashes(keys) % np.uint64(rank_n)).astype(np.int64)

    # -- finish / output
    def finish(self) -> int:
        n = C.c_uint64()
        self._check(N.lib().mhmkc_finish(self._h, C.byref(n)))
        self.n_out = int(n.value)
        return self.n_out

    def fetch(self, ordered: bool = False, out: KmerTable | None = None) -> KmerTable:
        """The finished table on the host (mhmkc_fetch). ordered=True: rows in the order of the top 32 bits of
        map_hash(key) (mhmkc_fetch_ordered, a device sort), the slot order of the C++ adapter's KmerMap.
        out: a table whose arrays are filled (at least n_out rows; e.g. pinned host memory, which the copies reach
        directly) instead of new ones."""
        if self.n_out is None:
            raise RuntimeError("fetch before finish")
        n = self.n_out
        if out is not None:
            # (the native copy writes n * 8 * n_longs, n * 2, n and n bytes: the dtypes must be those widths)
            if (len(out) < n or out.keys.ndim != 2 or out.keys.shape[1] != self.n_longs or out.keys.dtype != np.uint64
                    or out.counts.dtype != np.uint16 or out.left.dtype.itemsize != 1 or out.right.dtype.itemsize != 1
                    or min(len(out.counts), len(out.left), len(out.right)) < n
                    or not all(a.flags.c_contiguous for a in (out.keys, out.counts, out.left, out.right))):
                raise ValueError("out: contiguous arrays of at least n_out rows: keys uint64 [n, n_longs], counts "
                                 "uint16, left / right one byte per row")
            keys, counts, left, right = out.keys[:n], out.counts[:n], out.left[:n], out.right[:n]
        else:
            keys = np.empty((n, self.n_longs), dtype=np.uint64)
            counts = np.empty(n, dtype=np.uint16)
            left = np.empty(n, dtype=np.uint8)
            right = np.empty(n, dtype=np.uint8)
        fn = N.lib().mhmkc_fetch_ordered if ordered else N.lib().mhmkc_fetch
        self._check(fn(self._h, keys.ctypes.data, counts.ctypes.data, left.ctypes.data, right.ctypes.data))
        return KmerTable(self.k, keys, counts, left, right)

    def device_output(self) -> dict:
        ptrs = [C.c_void_p() for _ in range(4)]
        n = C.c_uint64()
        self._check(N.lib().mhmkc_device_output(self._h, *(C.byref(p) for p in ptrs), C.byref(n)))
        return {"keys": ptrs[0].value, "counts": ptrs[1].value, "left": ptrs[2].value, "right": ptrs[3].value,
                "n_out": int(n.value), "n_longs": self.n_longs}

    def stats(self) -> dict:
        s = N.MhmkcStats()
        self._check(N.lib().mhmkc_get_stats(self._h, C.byref(s)))
        return s.as_dict()

    def reset(self) -> None:
        self._check(N.lib().mhmkc_reset(self._h))
        self.n_out = None

    def set_profiling(self, on: "bool | int" = True) -> None:
        """Per-stage event timing (stats()["ms_kernel"]): True / 1 every stage, 2 the heavy stages only, False off."""
        self._check(N.lib().mhmkc_set_profiling(self._h, int(on) if on is not True else 1))


class TorchDistTransport:
    """mhmkc_transport (host-staged exchange, include/mhmkc.h) over a torch.distributed process group whose
    backend moves CPU tensors (gloo). It stands where the reference's UPC++ RPC stands
    (src/kcount/kmer_dht.cpp:133-149,222-231) for hosts without RCCL between the ranks: several nodes, or
    several ranks sharing one GPU."""

    def __init__(self, group=None):
        import torch.distributed as dist

        self.dist, self.group = dist, group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.error: BaseException | None = None
        self._ag = N.ALLGATHER_FN(self._allgather)
        self._a2a = N.ALLTOALLV_FN(self._alltoallv)
        self.struct = N.MhmkcTransport(None, self._ag, self._a2a)

    @staticmethod
    def _view(ptr: int, n: int):
        import torch

        if n == 0:
            return torch.empty(0, dtype=torch.uint8)
        return torch.frombuffer((C.c_uint8 * n).from_address(ptr), dtype=torch.uint8)

    def _allgather(self, _ctx, send, recv, nbytes):
        try:
            if nbytes:
                import torch

                outs = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(self.world)]
                self.dist.all_gather(outs, self._view(send, nbytes).clone(), group=self.group)
                dst = self._view(recv, self.world * nbytes)
                for r in range(self.world):
                    dst[r * nbytes:(r + 1) * nbytes].copy_(outs[r])
            return 0
        except BaseException as e:  # the C side turns a non-zero return into MHMKC_ETRANSPORT
            self.error = e
            return 1

    def _alltoallv(self, _ctx, send, send_bytes, recv, recv_bytes):
        try:
            sb = [int(send_bytes[p]) for p in range(self.world)]
            rb = [int(recv_bytes[p]) for p in range(self.world)]
            inp, out = self._view(send, sum(sb)), self._view(recv, sum(rb))
            self.dist.all_to_all_single(out, inp, output_split_sizes=rb, input_split_sizes=sb, group=self.group)
            return 0
        except BaseException as e:
            self.error = e
            return 1


class SharedGpuCounter:
    """Several host ranks over fewer GPU counters: the reference's launch runs one rank per core and maps rank r to
    GPU r % n_devices (gpu_utils::set_gpu_device, src/gpu-utils/gpu_utils.cpp:68-75; src/devices_gpu.cpp:61), while
    one GPU holds one counter. Rank r belongs to counter group g = r % n_counters; the group's leader (rank g) owns
    the counter (KmerCounter rank g of n_counters, MHMKC_OWNER_MINIMIZER, the leaders exchanging through the host
    transport over their own process group), the other members hand their PackedReads to it, and after the finish
    the leader sends every member the rows it owns. With n_counters dividing the number of ranks, the rows of
    counter g (get_kmer_target_rank % n_counters == g) are exactly those whose get_kmer_target_rank over all ranks
    is a member of group g (t % n_ranks = r implies t % n_counters = r % n_counters), so every rank ends with the
    table the reference's KmerDHT would hold (kmer_dht.cpp:193-196). Non-leaders never touch a GPU.

    Collective over the default torch.distributed process group (gloo: CPU tensors); every rank creates it."""

    def __init__(self, k: int, n_counters: int, *, device: int = 0, **counter_kwargs):
        import torch.distributed as dist

        self.dist = dist
        self.k, self.world, self.rank = k, dist.get_world_size(), dist.get_rank()
        if n_counters < 1 or self.world % n_counters:
            raise ValueError("n_counters must divide the number of ranks")
        self.n_counters = n_counters
        self.group_id = self.rank % n_counters
        self.leader = self.group_id
        self.members = list(range(self.group_id, self.world, n_counters))
        # every rank takes part in creating every group (torch.distributed.new_group is collective)
        leaders = dist.new_group(list(range(n_counters)))
        self.counter = None
        if self.rank == self.leader:
            self.counter = KmerCounter(k, device=device, rank=self.group_id, n_ranks=n_counters,
                                       transport=TorchDistTransport(leaders) if n_counters > 1 else None,
                                       output_owner=N.MHMKC_OWNER_MINIMIZER, **counter_kwargs)
        self._reads = []

    def add_packed_reads(self, packed_bytes: np.ndarray, offsets: np.ndarray) -> None:
        self._reads.append((np.ascontiguousarray(packed_bytes, dtype=np.uint8),
                            np.ascontiguousarray(offsets, dtype=np.uint64)))

    def _send_arrays(self, arrays, dst: int) -> None:
        import torch

        sizes = torch.tensor([a.nbytes for a in arrays], dtype=torch.int64)
        self.dist.send(torch.tensor([len(arrays)], dtype=torch.int64), dst)
        self.dist.send(sizes, dst)
        for a in arrays:
            if a.nbytes:
                self.dist.send(torch.from_numpy(a.view(np.uint8).reshape(-1).copy()), dst)

    def _recv_arrays(self, src: int) -> list:
        import torch

        n = torch.zeros(1, dtype=torch.int64)
        self.dist.recv(n, src)
        sizes = torch.zeros(int(n.item()), dtype=torch.int64)
        self.dist.recv(sizes, src)
        out = []
        for sz in sizes.tolist():
            t = torch.empty(sz, dtype=torch.uint8)
            if sz:
                self.dist.recv(t, src)
            out.append(t.numpy())
        return out

    def finish(self) -> KmerTable:
        """Count every member's reads on the group's GPU, exchange between the counters, and return this rank's
        rows (the k-mers whose get_kmer_target_rank over all ranks is this rank)."""
        if self.rank != self.leader:  # members: reads to the leader, then this rank's rows back
            flat = [a for pair in self._reads for a in pair]
            self._send_arrays(flat, self.leader)
            width, keys, counts, left, right = self._recv_arrays(self.leader)
            nl = int(width.view(np.int64)[0])  # the leader's key width (its counter's n_longs)
            return KmerTable(self.k, keys.view(np.uint64).reshape(-1, nl), counts.view(np.uint16), left, right)
        c = self.counter
        for b, o in self._reads:
            c.add_packed_reads(b, o)
        for m in self.members[1:]:
            got = self._recv_arrays(m)
            for i in range(0, len(got), 2):
                c.add_packed_reads(got[i], got[i + 1].view(np.uint64))
        c.finish()
        t = c.fetch()
        owner = c.target_ranks(t.keys, self.world) if len(t) else np.zeros(0, np.int64)
        mine = None
        for m in self.members:
            sel = np.flatnonzero(owner == m)
            part = [np.ascontiguousarray(t.keys[sel]), np.ascontiguousarray(t.counts[sel]),
                    np.ascontiguousarray(t.left[sel]), np.ascontiguousarray(t.right[sel])]
            if m == self.rank:
                mine = KmerTable(self.k, *part)
            else:
                self._send_arrays([np.array([c.n_longs], dtype=np.int64)] + part, m)
        return mine

    def close(self) -> None:
        if self.counter is not None:
            self.counter.close()
            self.counter = None


def comm_id() -> bytes:
    """RCCL unique id for multi-rank counters (rank 0 creates it and broadcasts it)."""
    buf = C.create_string_buffer(N.MHMKC_COMM_ID_BYTES)
    N.check(N.lib().mhmkc_comm_id(buf))
    return buf.raw


# ------------------------------------------------------------------------------------------------
# KmerDHT / analyze_kmers mirror


def map_hash(longs) -> int:
    """mhmkc_map_hash (include/mhmkc.h): the C++ adapter's KmerMap hash of a key's words."""
    M = (1 << 64) - 1
    h = 0x9E3779B97F4A7C15
    for w in longs:
        h = ((h ^ int(w)) * 0xBF58476D1CE4E5B9) & M
        h ^= h >> 31
    h = (h * 0x94D049BB133111EB) & M
    return h ^ (h >> 29)


def _quick_hash(v: int) -> int:
    """quick_hash (src/hash_funcs.c:332-342)."""
    M = (1 << 64) - 1
    v = (v * 3935559000370003845 + 2691343689449507681) & M
    v ^= v >> 21
    v = (v ^ (v << 37)) & M
    v ^= v >> 4
    v = (v * 4768777513237032717) & M
    v = (v ^ (v << 20)) & M
    v ^= v >> 41
    v = (v ^ (v << 5)) & M
    return v


def _revcomp_longs(longs: Sequence[int], k: int) -> tuple:
    s = kmer_to_string(longs, k)
    comp = {"A": "T", "C": "G", "G": "C", "T": "A"}
    return kmer_from_string("".join(comp[c] for c in reversed(s)), len(longs))


def minimizer_len(k: int) -> int:
    """KmerDHT minimizer length (src/kcount/kmer_dht.cpp:114-116)."""
    return min(27, max(15, k * 2 // 3 + 1))


def get_minimizer_fast(longs: Sequence[int], k: int, m: int) -> int:
    """Greatest least-complement m-mer (Kmer::get_minimizer_fast, src/kmer.cpp:344-403)."""
    M = (1 << 64) - 1
    mask = (M << (64 - 2 * m)) & M
    s = kmer_to_string(longs, k)
    rc = kmer_to_string(_revcomp_longs(longs, k), k)
    best = 0
    for i in range(k - m + 1):
        f = kmer_from_string(s[i:i + m], 1)[0] & mask
        r = kmer_from_string(rc[k - m - i:k - i], 1)[0] & mask
        best = max(best, min(f, r))
    return best


def get_kmer_target_rank(longs: Sequence[int], k: int, rank_n: int) -> int:
    """KmerDHT::get_kmer_target_rank (src/kcount/kmer_dht.cpp:193-196): the owner rank dbjg expects."""
    return _quick_hash(get_minimizer_fast(longs, k, minimizer_len(k))) % rank_n


class KmerDHT:
    """Per-rank result holder shaped like KmerDHT<MAX_K> (src/kcount/kmer_dht.hpp:118-172)."""

    def __init__(self, k: int, my_num_kmers: int = 0, *, counter: KmerCounter | None = None, rank: int = 0,
                 n_ranks: int = 1, **counter_kwargs):
        self.k = k
        self.my_num_kmers = my_num_kmers
        self.rank, self.n_ranks = rank, n_ranks
        self.counter = counter or KmerCounter(k, rank=rank, n_ranks=n_ranks, **counter_kwargs)
        self.minimizer_len = minimizer_len(k)
        self.table: KmerTable | None = None
        self._map: dict | None = None

    def get_minimizer_len(self) -> int:
        return self.minimizer_len

    def finish_updates(self) -> None:
        """flush_updates + finish_updates (src/kcount/kmer_dht.cpp:227-236)."""
        self.counter.finish()
        self.table = self.counter.fetch()
        self._map = None

    @property
    def local_kmers(self) -> dict:
        """KmerMap: {longs tuple: KmerCounts} (materialised lazily; use .table for large sets)."""
        if self._map is None:
            t = self.table
            self._map = {tuple(int(x) for x in t.keys[i]): KmerCounts(int(t.counts[i]), chr(int(t.left[i])),
                                                                       chr(int(t.right[i])))
                         for i in range(len(t))}
        return self._map

    def get_local_num_kmers(self) -> int:
        return 0 if self.table is None else len(self.table)

    def get_num_kmers(self) -> int:
        return self.get_local_num_kmers()

    def get_local_kmer_counts(self, kmer) -> KmerCounts | None:
        key = kmer_from_string(kmer) if isinstance(kmer, str) else tuple(int(x) for x in kmer)
        return self.local_kmers.get(key)

    def get_kmer_target_rank(self, kmer) -> int:
        longs = kmer_from_string(kmer) if isinstance(kmer, str) else kmer
        return get_kmer_target_rank(longs, self.k, self.n_ranks)

    def dump_kmers(self, out_dir: str | os.PathLike = ".") -> Path:
        """dump_kmers (src/kcount/kmer_dht.cpp:243-266): kmers-<k>.txt.gz in this rank's directory
        (get_rank_path: per_rank/<rank / 1000>/<rank>/, upcxx-utils/src/log.cpp:283-312), lines
        "KMER count L R"."""
        path = Path(out_dir) / "per_rank" / f"{self.rank // 1000:08d}" / f"{self.rank:08d}" / f"kmers-{self.k}.txt.gz"
        path.parent.mkdir(parents=True, exist_ok=True)
        with gzip.open(path, "wt") as f:
            for line in self.table.lines():
                f.write(line + "\n")
        return path

    def clear_stores(self) -> None:
        self.counter.reset()


def analyze_kmers(kmer_len: int, prev_kmer_len: int, qual_offset: int, packed_reads_list: Sequence[PackedReads],
                  dmin_thres: int, ctgs: Sequence, kmer_dht: KmerDHT, dump_kmers: bool = False,
                  dump_dir: str | os.PathLike = ".") -> None:
    """analyze_kmers<MAX_K> (src/kcount/kcount.hpp:71-73, src/kcount/kcount.cpp:140-157).

    Counts every read of every PackedReads on this rank's GPU, exchanges by hash range with the other
    ranks, applies the contig pass when ctgs is not empty (add_ctg_kmers, kcount.cpp:100-138; single rank),
    purges and chooses extensions; the result is kmer_dht.table / kmer_dht.local_kmers. ctgs: objects with
    .seq and .depth (a float, as Contig), or (seq, depth) pairs.
    """
    if kmer_len != kmer_dht.k:
        raise ValueError("kmer_len differs from the KmerDHT's k")
    kmer_dht.counter.set_dmin_thres(dmin_thres)  # _dmin_thres = dmin_thres (kcount.cpp:145)
    for pr in packed_reads_list:
        if pr.qual_offset != qual_offset:
            raise ValueError("PackedReads qual_offset differs")
        kmer_dht.counter.add_reads(pr)
    if len(ctgs):
        seqs, depths = [], []
        for c in ctgs:
            seq, depth = (c.seq, c.depth) if hasattr(c, "seq") else (c[0], c[1])
            seqs.append(seq)
            depths.append(min(int(depth), 65535))  # Contig::get_uint16_t_depth (src/contigs.hpp:65)
        kmer_dht.counter.add_ctgs(seqs, depths)
    kmer_dht.finish_updates()
    if dump_kmers:
        kmer_dht.dump_kmers(dump_dir)


# ------------------------------------------------------------------------------------------------
# synthetic reads


def synth_genome(genome_len: int, seed: int) -> np.ndarray:
    S = N.synth()
    cfg = N.SynthConfig()
    S.mhmkc_synth_config_init(C.byref(cfg), genome_len, 150, seed)
    g = np.empty(genome_len, dtype=np.uint8)
    if S.mhmkc_synth_genome(C.byref(cfg), g.ctypes.data) != 0:
        raise RuntimeError("mhmkc_synth_genome failed")
    return g


def synth_reads(genome: np.ndarray, n_reads: int, read_len: int, seed: int, first_read: int = 0,
                threads: int = 0, **rates) -> tuple[np.ndarray, np.ndarray]:
    """(packed_bytes, offsets) of reads first_read .. first_read + n_reads - 1 of the global set."""
    S = N.synth()
    cfg = N.SynthConfig()
    S.mhmkc_synth_config_init(C.byref(cfg), genome.size, read_len, seed)
    for key, val in rates.items():
        setattr(cfg, key, val)
    b = np.empty(n_reads * read_len, dtype=np.uint8)
    o = np.empty(n_reads + 1, dtype=np.uint64)
    g = np.ascontiguousarray(genome, dtype=np.uint8)
    nt = threads or min(16, os.cpu_count() or 1)
    if S.mhmkc_synth_reads(C.byref(cfg), g.ctypes.data, first_read, n_reads, b.ctypes.data, o.ctypes.data, nt) != 0:
        raise RuntimeError("mhmkc_synth_reads failed")
    return b, o
