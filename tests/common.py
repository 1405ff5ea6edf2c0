"""Shared helpers for the parity tests (inputs, table comparison)."""
from __future__ import annotations

import gzip
from pathlib import Path

import numpy as np

import mhm2_proxy_amd as m
import oracle_lib as O

GOLDEN = Path(__file__).resolve().parent / "golden"


def synth_set(n_reads: int, genome_len: int, seed: int, read_len: int = 150, **rates):
    g = m.synth_genome(genome_len, seed)
    return m.synth_reads(g, n_reads, read_len, seed, **rates)


def edge_case_set(seed: int = 5, n: int = 1500):
    """Variable-length reads incl. L < k, L = k, k+1, k+2, all-N, poly-A (hot k-mer), low quality and
    every PackedRead code; built deterministically from synthetic reads."""
    rng = np.random.default_rng(seed)
    b, o = synth_set(n, 20000, seed)
    reads = [b[o[i]:o[i + 1]].copy() for i in range(n)]
    out = []
    for i, r in enumerate(reads):
        mode = i % 10
        if mode == 0:
            r = r[: int(rng.integers(0, 150))]
        elif mode == 1:
            r = r[: int(rng.integers(18, 26))]
        elif mode == 2:
            r = np.full(int(rng.integers(20, 150)), 4 | (31 << 3), dtype=np.uint8)  # all N, good quality
        elif mode == 3:
            r = np.full(150, 0 | (31 << 3), dtype=np.uint8)  # poly-A
        elif mode == 4:
            r = (r & 7) | (np.uint8(5) << 3)  # all low quality
        elif mode == 5:
            q = rng.integers(0, 32, size=r.size).astype(np.uint8)
            r = (r & 7) | (q << 3)
        out.append(r.astype(np.uint8))
    out.append(np.zeros(0, np.uint8))
    lens = np.array([x.size for x in out], dtype=np.uint64)
    offs = np.zeros(len(out) + 1, dtype=np.uint64)
    np.cumsum(lens, out=offs[1:])
    return np.concatenate(out).astype(np.uint8), offs


def hot_set(n_poly: int = 800, seed: int = 9, n_reads: int = 400, genome_len: int = 20000):
    """Enough poly-A reads that one canonical k-mer passes 65535 occurrences (u16 saturation) and its
    extension counters pass the 0xC000 clamp of the LDS counters (after n_reads random reads)."""
    b, o = synth_set(n_reads, genome_len, seed)
    poly = np.full(150, 0 | (31 << 3), dtype=np.uint8)
    reads = [b[o[i]:o[i + 1]] for i in range(n_reads)] + [poly] * n_poly
    lens = np.array([x.size for x in reads], dtype=np.uint64)
    offs = np.zeros(len(reads) + 1, dtype=np.uint64)
    np.cumsum(lens, out=offs[1:])
    return np.concatenate(reads).astype(np.uint8), offs


def ctg_set(seed: int = 21, n_reads: int = 300, genome_len: int = 6000, n_ctgs: int = 200):
    """Reads plus contigs for the contig pass (add_ctg_kmers): genome substrings (both strands), exact
    duplicates with other depths (min rule), mutated copies (read entries replaced, contig conflicts),
    overlapping pieces, novel sequence (keys absent from the reads), N bases, lowercase (low quality),
    contigs shorter than k + 2 (skipped) and depths 0, 1, 2, 3, ..., 65535."""
    rng = np.random.default_rng(seed)
    g = m.synth_genome(genome_len, seed)
    b, o = m.synth_reads(g, n_reads, 150, seed)
    gs = "".join("ACGT"[int(x)] for x in g)
    comp = {"A": "T", "C": "G", "G": "C", "T": "A", "N": "N"}
    seqs, depths = [], []
    depth_choices = [0, 1, 2, 3, 5, 12, 40, 300, 65535]
    for i in range(n_ctgs):
        mode = i % 8
        L = int(rng.integers(10, 420))
        st = int(rng.integers(0, genome_len - L))
        s = gs[st:st + L]
        if mode in (1, 7) and seqs:  # exact duplicate of an earlier contig, other depth
            s = seqs[int(rng.integers(0, len(seqs)))].upper()
        elif mode == 6 and seqs:  # mutated copy of an earlier contig: shared k-mers, other extensions
            s = list(seqs[int(rng.integers(0, len(seqs)))].upper())
            for _ in range(max(1, len(s) // 50)):
                j = int(rng.integers(0, len(s)))
                s[j] = "ACGT"[(("ACGTN".index(s[j]) + int(rng.integers(1, 4))) % 4)]
            s = "".join(s)
        elif mode == 2:  # point mutations
            s = list(s)
            for _ in range(max(1, L // 60)):
                j = int(rng.integers(0, L))
                s[j] = "ACGT"[(("ACGT".index(s[j]) + int(rng.integers(1, 4))) % 4)]
            s = "".join(s)
        elif mode == 3:  # novel sequence
            s = "".join("ACGT"[int(x)] for x in rng.integers(0, 4, L))
        elif mode == 4:  # N bases
            s = list(s)
            for _ in range(2):
                s[int(rng.integers(0, L))] = "N"
            s = "".join(s)
        elif mode == 5:  # lowercase stretch (bases below the quality cutoff)
            j = int(rng.integers(0, L))
            s = s[:j] + s[j:j + 5].lower() + s[j + 5:]
        if rng.integers(0, 2):
            s = "".join(comp.get(c.upper(), c.upper()) if c.isupper() else comp[c.upper()].lower() for c in reversed(s))
        seqs.append(s)
        depths.append(int(depth_choices[int(rng.integers(0, len(depth_choices)))]))
    return b, o, seqs, np.array(depths, dtype=np.uint16)


def oracle_ctg_table(b, o, seqs, depths, k, **kw) -> m.KmerTable:
    t = O.kcount_ctgs(b, o, seqs, depths, k, **kw)
    keys, c, l, r = t.fetch()
    return m.KmerTable(k, keys, c, l, r)


def oracle_table(b, o, k, **kw) -> m.KmerTable:
    t = O.kcount(b, o, k, **kw)
    keys, c, l, r = t.fetch()
    return m.KmerTable(k, keys, c, l, r)


def assert_tables_equal(a: m.KmerTable, b: m.KmerTable, what: str = ""):
    a, b = a.sorted(), b.sorted()
    assert len(a) == len(b), f"{what}: {len(a)} vs {len(b)} k-mers"
    if len(a) == 0:
        return
    bad = np.flatnonzero((a.keys != b.keys).any(axis=1) | (a.counts != b.counts) | (a.left != b.left) |
                         (a.right != b.right))
    if bad.size:
        i = int(bad[0])
        ka = m.keys_to_strings(a.keys[i:i + 1], a.k)[0]
        kb = m.keys_to_strings(b.keys[i:i + 1], b.k)[0]
        raise AssertionError(f"{what}: {bad.size} rows differ; first at {i}: {ka} {a.counts[i]} {chr(a.left[i])} "
                             f"{chr(a.right[i])} vs {kb} {b.counts[i]} {chr(b.left[i])} {chr(b.right[i])}")


def _mix64(x: np.ndarray) -> np.ndarray:
    """splitmix64's finalizer over a uint64 array (wrapping arithmetic)."""
    x = x ^ (x >> np.uint64(30))
    x *= np.uint64(0xBF58476D1CE4E5B9)
    x ^= x >> np.uint64(27)
    x *= np.uint64(0x94D049BB133111EB)
    x ^= x >> np.uint64(31)
    return x


def table_digest(t: m.KmerTable, sample_bits: int = 8) -> dict:
    """Order-independent digest of a (large) table for the tests whose tables hold hundreds of millions of rows:
    the row count, two wrapping sums of independent 64-bit row fingerprints (key words, count, left, right), and the
    rows whose key fingerprint has its top sample_bits bits zero (a fixed 1/2^sample_bits subsample of the key space,
    the same keys on both sides, for a row-by-row check). Two tables with equal digests hold the same multiset of
    rows except with probability ~2^-64; the sample is compared exactly (assert_digests_equal)."""
    keys = np.ascontiguousarray(t.keys, dtype=np.uint64)
    kf = _mix64(keys[:, 0] ^ np.uint64(0x9E3779B97F4A7C15))
    for w in range(1, keys.shape[1]):
        kf = _mix64(kf ^ keys[:, w])
    v = (t.counts.astype(np.uint64) | (t.left.astype(np.uint64) << np.uint64(32)) |
         (t.right.astype(np.uint64) << np.uint64(40)))
    rf = _mix64(kf ^ v)
    s1 = int(rf.sum(dtype=np.uint64))
    rf ^= np.uint64(0xD6E8FEB86659FD93)
    s2 = int(_mix64(rf).sum(dtype=np.uint64))
    del rf, v
    sel = (kf >> np.uint64(64 - sample_bits)) == 0
    return {"n": len(t), "s1": s1, "s2": s2, "keys": keys[sel], "counts": t.counts[sel], "left": t.left[sel],
            "right": t.right[sel]}


def merge_digests(ds: list) -> dict:
    """The digest of the union of disjoint tables (e.g. the owners' parts of one table)."""
    mask = (1 << 64) - 1
    out = {"n": sum(int(d["n"]) for d in ds), "s1": sum(int(d["s1"]) for d in ds) & mask,
           "s2": sum(int(d["s2"]) for d in ds) & mask}
    for f in ("keys", "counts", "left", "right"):
        out[f] = np.concatenate([np.asarray(d[f]) for d in ds])
    return out


def assert_digests_equal(a: dict, b: dict, k: int, what: str = ""):
    assert int(a["n"]) == int(b["n"]), f"{what}: {int(a['n'])} vs {int(b['n'])} k-mers"
    sa = m.KmerTable(k, a["keys"], a["counts"], a["left"], a["right"])
    sb = m.KmerTable(k, b["keys"], b["counts"], b["left"], b["right"])
    assert_tables_equal(sa, sb, f"{what} (sampled rows)")
    assert (int(a["s1"]), int(a["s2"])) == (int(b["s1"]), int(b["s2"])), f"{what}: row fingerprints differ"


def read_reads_file(path: Path):
    """'seq qual' lines (BASELINE.md input format) -> PackedRead bytes + offsets."""
    seqs = []
    with gzip.open(path, "rt") as f:
        for line in f:
            parts = line.split()
            seqs.append(m.PackedReads.pack(parts[0], parts[1]) if parts else np.zeros(0, np.uint8))
    lens = np.array([s.size for s in seqs], dtype=np.uint64)
    offs = np.zeros(len(seqs) + 1, dtype=np.uint64)
    np.cumsum(lens, out=offs[1:])
    return (np.concatenate(seqs) if seqs else np.zeros(0, np.uint8)).astype(np.uint8), offs


def read_table_file(path: Path, k: int) -> m.KmerTable:
    """dump_kmers lines 'KMER count L R' -> KmerTable."""
    nl = m.n_longs_for(k)
    keys, counts, left, right = [], [], [], []
    with gzip.open(path, "rt") as f:
        for line in f:
            s, c, l, r = line.split()
            keys.append(m.kmer_from_string(s, nl))
            counts.append(int(c))
            left.append(ord(l))
            right.append(ord(r))
    return m.KmerTable(k, np.array(keys, dtype=np.uint64).reshape(-1, nl), np.array(counts, dtype=np.uint16),
                       np.array(left, dtype=np.uint8), np.array(right, dtype=np.uint8))


NAME_STYLES = ("illumina18", "slash", "hudson", "tab", "plain", "slash_comment")


def fastq_text(packed_bytes, offsets, *, seed: int = 0, crlf_every: int = 0, trailing_ws: bool = False,
               iupac: bool = False, final_newline: bool = True, qual_offset: int = 33) -> bytes:
    """FASTQ text of packed reads, in every read-name style get_fq_name accepts (src/fastq.cpp:73-122),
    optionally with CRLF lines, trailing whitespace and IUPAC codes for N (all of which pack back to the
    same PackedRead bytes)."""
    rng = np.random.default_rng(seed)
    b = np.asarray(packed_bytes, dtype=np.uint8)
    codes = np.frombuffer(b"ACGTN", dtype=np.uint8)
    seq_all = codes[np.minimum(b & 7, 4)].copy()
    if iupac:
        amb = np.frombuffer(b"NURYKMSWBDHV", dtype=np.uint8)
        isn = seq_all == ord("N")
        seq_all[isn] = amb[rng.integers(0, len(amb), size=int(isn.sum()))]
    qual_all = ((b >> 3) + qual_offset).astype(np.uint8)
    out = []
    n = len(offsets) - 1
    for i in range(n):
        lo, hi = int(offsets[i]), int(offsets[i + 1])
        style = NAME_STYLES[(i + seed) % len(NAME_STYLES)]
        mate = 1 + (i & 1)
        name = {"illumina18": f"@M0:{i}:FC:1:{i % 97}:{i % 13}:{i} {mate}:N:0:ACGT",
                "slash": f"@read{i}/{mate}", "hudson": f"@pair{i}-R{mate}",
                "tab": f"@read{i}/{mate}\textra", "plain": f"@r{i}",
                "slash_comment": f"@read{i}/{mate} comment here"}[style]
        eol = "\r\n" if crlf_every and i % crlf_every == 0 else "\n"
        ws = "  \t" if trailing_ws and i % 3 == 0 else ""
        out.append(f"{name}{ws}{eol}".encode())
        out.append(seq_all[lo:hi].tobytes() + ws.encode() + eol.encode())
        out.append(f"+{eol}".encode())
        out.append(qual_all[lo:hi].tobytes() + eol.encode())
    t = b"".join(out)
    if not final_newline and t.endswith(b"\n"):
        t = t[:-2] if t.endswith(b"\r\n") else t[:-1]
    return t


PAIR_NAME_STYLES = ("illumina18", "slash", "hudson", "tab", "slash_comment")


def paired_fastq_text(n_pairs: int, seed: int = 0, *, genome_len: int = 200_000, read_len: int = 150,
                      frag_mean: int = 240, frag_sd: int = 40, subst: float = 0.01, n_rate: float = 0.002,
                      iupac: bool = True, low_q: float = 0.05, qual_offset: int = 33, uneven: bool = True) -> bytes:
    """Interleaved paired FASTQ (mate 1 = a fragment's start, mate 2 = the reverse complement of its end), so
    that most pairs overlap by 2L - F bases: substitutions at random qualities, N and IUPAC codes, low-quality
    runs, unequal mate lengths, every name style get_fq_name accepts with /1 and /2 mates."""
    rng = np.random.default_rng(seed)
    g = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, size=genome_len)]
    comp = np.zeros(256, dtype=np.uint8)
    for a, b in (b"AT", b"CG", b"GC", b"TA"):
        comp[a] = b
    amb = np.frombuffer(b"NRYKMSWBDHV", dtype=np.uint8)
    out = []
    for i in range(n_pairs):
        F = int(np.clip(rng.normal(frag_mean, frag_sd), 40, 2 * read_len + 60))
        a = int(rng.integers(0, genome_len - F))
        frag = g[a:a + F]
        L1 = read_len if not uneven or i % 7 else int(rng.integers(20, read_len + 1))
        L2 = read_len if not uneven or i % 11 else int(rng.integers(20, read_len + 1))
        m1 = frag[:min(L1, F)].copy()
        m2 = comp[frag[::-1][:min(L2, F)]].copy()
        quals = []
        for m in (m1, m2):
            q = rng.integers(30, 41, size=m.size).astype(np.uint8)
            tail = int(rng.integers(0, m.size // 3 + 1)) if rng.random() < 0.3 else 0
            if tail:
                q[m.size - tail:] = rng.integers(2, 20, size=tail)
            sub = rng.random(m.size) < subst
            m[sub] = g[rng.integers(0, 4, size=int(sub.sum()))]
            q[sub] = rng.integers(2, 41, size=int(sub.sum()))
            nn = rng.random(m.size) < n_rate
            m[nn] = amb[rng.integers(0, len(amb) if iupac else 1, size=int(nn.sum()))]
            lq = rng.random(m.size) < low_q
            q[lq] = rng.integers(0, 12, size=int(lq.sum()))
            quals.append((q + qual_offset).astype(np.uint8))
        style = PAIR_NAME_STYLES[i % len(PAIR_NAME_STYLES)]
        for mate, (m, q) in enumerate(((m1, quals[0]), (m2, quals[1])), start=1):
            name = {"illumina18": f"@M0:{i}:FC:1:{i % 97}:{i % 13}:{i} {mate}:N:0:ACGT",
                    "slash": f"@frag {i}/{mate}", "hudson": f"@pair{i}-R{mate}",
                    "tab": f"@read{i}/{mate}\textra", "slash_comment": f"@read{i}/{mate} comment here"}[style]
            out.append(name.encode() + b"\n" + m.tobytes() + b"\n+\n" + q.tobytes() + b"\n")
    return b"".join(out)


def paired_fastq_bulk(n_pairs: int, seed: int, genome_len: int, *, read_len: int = 150, frag_mean: int = 240,
                      frag_sd: int = 40, subst: float = 0.005, n_rate: float = 0.001, low_q: float = 0.03,
                      qual_offset: int = 33) -> bytes:
    """paired_fastq_text's model at scale (vectorised, millions of pairs): fragments of a synthetic genome
    (m.synth_genome) of read_len <= F <= 2 read_len + 60 bases, mate 1 its start, mate 2 the reverse complement of
    its end, substitutions at random qualities, N bases, low-quality bases; names "@p<9 digits>/1" and "/2"."""
    rng = np.random.default_rng(seed)
    g = np.frombuffer(b"ACGT", dtype=np.uint8)[m.synth_genome(genome_len, seed).astype(np.int64) & 3]
    comp = np.zeros(256, dtype=np.uint8)
    for a, b in (b"AT", b"CG", b"GC", b"TA"):
        comp[a] = b
    L = read_len
    F = np.clip(rng.normal(frag_mean, frag_sd, n_pairs), L, 2 * L + 60).astype(np.int64)
    start = (rng.random(n_pairs) * (genome_len - F)).astype(np.int64)
    col = np.arange(L, dtype=np.int64)
    m1 = g[start[:, None] + col]
    m2 = comp[g[(start + F - 1)[:, None] - col]]
    recs = []
    for mate, s in ((1, m1), (2, m2)):
        q = rng.integers(30, 41, size=s.shape, dtype=np.uint8)
        sub = rng.random(s.shape) < subst
        s[sub] = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, size=int(sub.sum()))]
        q[sub] = rng.integers(2, 41, size=int(sub.sum()), dtype=np.uint8)
        s[rng.random(s.shape) < n_rate] = ord("N")
        lq = rng.random(s.shape) < low_q
        q[lq] = rng.integers(0, 12, size=int(lq.sum()), dtype=np.uint8)
        name = np.empty((n_pairs, 14), dtype=np.uint8)  # "@p" + 9 digits + "/m" + "\n"
        name[:, 0], name[:, 1] = ord("@"), ord("p")
        idx = np.arange(n_pairs, dtype=np.int64)
        for d in range(9):
            name[:, 10 - d] = 48 + (idx // 10 ** d) % 10
        name[:, 11], name[:, 12], name[:, 13] = ord("/"), 48 + mate, ord("\n")
        nl = np.full((n_pairs, 1), ord("\n"), dtype=np.uint8)
        plus = np.frombuffer(b"+\n", dtype=np.uint8)[None, :].repeat(n_pairs, 0)
        recs.append(np.concatenate([name, s, nl, plus, (q + qual_offset).astype(np.uint8), nl], axis=1))
    return np.stack(recs, axis=1).reshape(-1).tobytes()
