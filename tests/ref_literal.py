"""Literal string-level restatement of the reference kcount read pass (TEST INFRASTRUCTURE ONLY).

Written independently of oracle/kcount_oracle.c and as close as Python allows to the reference's own
control flow, to cross-check the C oracle on small inputs. Every function cites the code it follows
(ajpowelsnl/mhm2_proxy). Pure Python loops: small cases only.
"""
from __future__ import annotations

NUCLEOTIDE_MAP = "ACGTN"  # PackedRead::nucleotide_map (src/packed_reads.hpp:61)
KCOUNT_QUAL_CUTOFF = 20  # CMakeDefinitions.txt:46
DYN_MIN_DEPTH = 0.9  # CMakeDefinitions.txt:60
U16_MAX = 65535
M64 = (1 << 64) - 1


def unpack(packed: bytes, qual_offset: int):
    """PackedRead::unpack (src/packed_reads.cpp:147-159)."""
    seq = "".join(NUCLEOTIDE_MAP[b & 7] for b in packed)
    quals = "".join(chr(qual_offset + (b >> 3)) for b in packed)
    return seq, quals


def set_kmer(s: str, k: int, n_longs: int):
    """Kmer::set_kmer (src/kmer.cpp:274-296)."""
    longs = [0] * n_longs
    for i in range(k):
        c = ord(s[i])
        x = (c & 4) >> 1
        longs[i // 32] |= (x + ((x ^ (c & 2)) >> 1)) << (2 * (31 - i % 32))
    return longs


def get_kmers(kmer_len: int, seq: str, n_longs: int):
    """Kmer::get_kmers (src/kmer.cpp:155-257): uppercase copy, every window (N encodes as G)."""
    seq = seq.upper()
    return [tuple(set_kmer(seq[i:i + kmer_len], kmer_len, n_longs)) for i in range(len(seq) - kmer_len + 1)]


def _twin(b: int) -> int:
    out = 0
    for j in range(4):
        out |= (3 - ((b >> (6 - 2 * j)) & 3)) << (2 * j)
    return out


TWIN_TABLE = [_twin(b) for b in range(256)]  # src/kmer.cpp:66-79


def revcomp(longs, k: int):
    """Kmer::revcomp (src/kmer.cpp:485-505)."""
    n_longs = len(longs)
    km = [0] * n_longs
    last_long = (k + 31) // 32
    for i in range(last_long):
        v = longs[i]
        r = 0
        for byte in range(8):
            r |= TWIN_TABLE[(v >> (8 * byte)) & 0xFF] << (56 - 8 * byte)
        km[last_long - 1 - i] = r
    shift = 2 * (32 - (k % 32)) if k % 32 else 0
    shiftmask = ((((1 << shift) - 1) << (64 - shift)) & M64) if k % 32 else 0
    km[0] = (km[0] << shift) & M64
    for i in range(1, last_long):
        km[i - 1] |= (km[i] & shiftmask) >> (64 - shift)
        km[i] = (km[i] << shift) & M64
    return tuple(km)


def comp_nucleotide(ch: str) -> str:
    """comp_nucleotide (src/utils.cpp:121-143)."""
    return {"A": "T", "C": "G", "G": "C", "T": "A", "N": "N", "0": "0"}[ch]


class ExtCounts:
    """ExtCounts (src/kcount/kcount_cpu.cpp:115-183)."""

    def __init__(self):
        self.c = {"A": 0, "C": 0, "G": 0, "T": 0}

    def inc(self, ext: str, count: int):
        if ext in self.c:
            self.c[ext] = min(self.c[ext] + count, U16_MAX)

    def get_sorted(self):
        items = [("A", self.c["A"]), ("C", self.c["C"]), ("G", self.c["G"]), ("T", self.c["T"])]
        # descending count; equal counts: higher char first (std::sort comparator at :136-141)
        return sorted(items, key=lambda e: (-e[1], -ord(e[0])))

    def get_ext(self, count: int, dmin_thres: int) -> str:
        s = self.get_sorted()
        top, runner_up = s[0][1], s[1][1]
        dmin_dyn = max(int((1.0 - DYN_MIN_DEPTH) * count), dmin_thres)
        if top < dmin_dyn:
            return "X"
        if runner_up >= dmin_dyn:
            return "F"
        return s[0][0]


class KmerExtsCounts:
    def __init__(self):
        self.left_exts, self.right_exts, self.count, self.from_ctg = ExtCounts(), ExtCounts(), 0, False


def get_kmers_and_exts(supermer_seq: str, k: int, n_longs: int):
    """get_kmers_and_exts (src/kcount/kcount_cpu.cpp:307-335)."""
    quals = [c.isupper() for c in supermer_seq]
    seq = supermer_seq.upper()
    kmers = get_kmers(k, seq, n_longs)
    out = []
    for i in range(1, len(seq) - k):
        kmer = kmers[i]
        left = seq[i - 1] if quals[i - 1] else "0"
        right = seq[i + k] if quals[i + k] else "0"
        rc = revcomp(kmer, k)
        if rc < kmer:
            kmer = rc
            left, right = comp_nucleotide(right), comp_nucleotide(left)
        out.append((kmer, left, right))
    return out


def analyze_kmers(reads, k: int, qual_offset: int = 33, dmin_thres: int = 2, qual_cutoff: int = KCOUNT_QUAL_CUTOFF,
                  ctgs=()):
    """count_kmers + [add_ctg_kmers] + finish at rank_n()==1 (src/kcount/kcount.cpp:54-157;
    kcount_cpu.cpp:73-103, 337-406, 490-528). reads: iterable of PackedRead byte strings; ctgs: iterable of
    (contig sequence, uint16 depth) in contig order. Returns {kmer longs: (count, L, R)}."""
    n_longs = k // 32 + 1
    table: dict = {}
    for packed in reads:
        seq, quals = unpack(bytes(packed), qual_offset)
        if len(seq) < k:
            continue
        seq = "".join(c.lower() if ord(q) < qual_offset + qual_cutoff else c for c, q in zip(seq, quals))
        # process_seq: one supermer = the whole read at one rank, emitted when length >= k + 2
        if len(seq) < k + 2:
            continue
        for ch in seq:
            if ch.upper() not in "ACGTN":
                raise ValueError("bad char")  # DIE (kcount_cpu.cpp:453-458)
        for kmer, left, right in get_kmers_and_exts(seq, k, n_longs):
            e = table.get(kmer)
            if e is None:
                e = table[kmer] = KmerExtsCounts()
            e.count = min(e.count + 1, U16_MAX)
            e.left_exts.inc(left, 1)
            e.right_exts.inc(right, 1)
    for seq, depth in ctgs:  # add_ctg_kmers (kcount.cpp:125-130)
        if len(seq) < k + 2:
            continue
        depth = depth or 1  # SeqBlockInserter::process_seq (kcount_cpu.cpp:75)
        for kmer, left, right in get_kmers_and_exts(seq, k, n_longs):  # insert_supermer_from_ctg (:356-406)
            count = depth
            e = table.get(kmer)
            is_new = e is None
            if is_new:
                e = table[kmer] = KmerExtsCounts()
            insert_it = False
            if is_new:
                insert_it = True
            elif not e.from_ctg:
                if e.count == 1:
                    insert_it = True
                else:
                    le, re_ = e.left_exts.get_ext(e.count, dmin_thres), e.right_exts.get_ext(e.count, dmin_thres)
                    if le in "XF" or re_ in "XF":
                        insert_it = True
            elif e.count:
                insert_it = True
                le, re_ = e.left_exts.get_ext(e.count, dmin_thres), e.right_exts.get_ext(e.count, dmin_thres)
                if le != left or re_ != right:
                    count = 0
                else:
                    count = min(count, e.count)
            if insert_it:
                e.left_exts, e.right_exts, e.count, e.from_ctg = ExtCounts(), ExtCounts(), count, True
                e.left_exts.inc(left, count)
                e.right_exts.inc(right, count)
    out = {}
    for kmer, e in table.items():
        if e.count < 2:
            continue
        left = e.left_exts.get_ext(e.count, dmin_thres)
        right = e.right_exts.get_ext(e.count, dmin_thres)
        if left == "X" and right == "X":
            continue
        out[kmer] = (e.count, left, right)
    return out
