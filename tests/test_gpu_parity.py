"""Parity of the HIP path (through the C ABI of libmhmkc.so) with the CPU oracle and the golden fixtures.

Bit-exact: every (canonical k-mer, count, left, right) row must be identical; order is free, as the
reference's KmerMap iteration order is.
"""
from __future__ import annotations

import os

import numpy as np
import pytest

import mhm2_proxy_amd as m
import oracle_lib as O
from common import (GOLDEN, assert_tables_equal, ctg_set, edge_case_set, hot_set, oracle_ctg_table, oracle_table,
                    read_reads_file, read_table_file, synth_set)

pytestmark = pytest.mark.gpu


def hip_table(b, o, k, batches=1, **kw):
    with m.KmerCounter(k, **kw) as c:
        n = o.size - 1
        cuts = [n * i // batches for i in range(batches + 1)]
        for a, z in zip(cuts[:-1], cuts[1:]):
            base = int(o[a])
            c.add_packed_reads(b[base:int(o[z])], (o[a:z + 1] - o[a]).astype(np.uint64))
        c.finish()
        return c.fetch(), c.stats()


def check_stats(st, oracle_stats=None):
    assert st["count_sum"] == st["owned_records"] == st["occurrences"]
    assert st["distinct"] == st["n_out"] + st["purged"]
    assert st["dropped"] == 0
    if oracle_stats:
        assert st["occurrences"] == oracle_stats["occurrences"]
        assert st["distinct"] == oracle_stats["distinct"]
        assert st["purged"] == oracle_stats["purged"]


@pytest.mark.parametrize("k", [21, 33, 55, 63, 77, 99, 15, 31, 45, 127, 9, 10, 11, 19, 22])
def test_synthetic_vs_oracle(k):
    b, o = synth_set(2000, 10000, 100 + k)
    ref = O.kcount(b, o, k)
    keys, c, l, r = ref.fetch()
    got, st = hip_table(b, o, k)
    assert_tables_equal(got, m.KmerTable(k, keys, c, l, r), f"k={k}")
    check_stats(st, ref.stats())


@pytest.mark.parametrize("k", [21, 33, 63, 99])
def test_edge_cases_vs_oracle(k):
    b, o = edge_case_set()
    got, st = hip_table(b, o, k)
    assert_tables_equal(got, oracle_table(b, o, k), f"edge k={k}")
    check_stats(st)


@pytest.mark.parametrize("k", [21, 63])
def test_hot_kmer_saturation(k):
    """One k-mer with > 65535 occurrences: u16 saturation, the LDS extension-counter clamp, and the
    capped coarse/fine buckets overflowing into the exact (histogram) fallback."""
    b, o = hot_set()
    got, st = hip_table(b, o, k)
    exp = oracle_table(b, o, k)
    assert (exp.counts == 65535).any(), "fixture must saturate a count"
    assert st["exact_reruns"] >= 1
    assert_tables_equal(got, exp, f"hot k={k}")


@pytest.mark.parametrize("k", [21, 63, 99])
def test_exact_partition_path(k, knob):
    """The histogram-sized (exact) partition path, forced for ordinary input."""
    b, o = synth_set(2500, 12000, 17 + k)
    exp = oracle_table(b, o, k)
    knob("exact", 1)
    got, st = hip_table(b, o, k)
    assert_tables_equal(got, exp, "exact path")
    check_stats(st)


@pytest.mark.parametrize("cutoff,dmin,dyn", [(0, 2, 0.9), (32, 2, 0.9), (20, 1, 0.9), (20, 5, 0.9), (20, 2, 0.5),
                                             (20, 2, 1.0), (20, 0, 0.0), (25, 3, 0.75)])
def test_parameters_vs_oracle(cutoff, dmin, dyn):
    b, o = synth_set(1500, 8000, 7)
    got, _ = hip_table(b, o, 21, qual_cutoff=cutoff, dmin_thres=dmin, dyn_min_depth=dyn)
    exp = oracle_table(b, o, 21, qual_cutoff=cutoff, dmin_thres=dmin, dyn_min_depth=dyn)
    assert_tables_equal(got, exp, f"cutoff={cutoff} dmin={dmin} dyn={dyn}")


@pytest.mark.parametrize("k", [21, 55])
def test_batches_equal_single(k):
    b, o = synth_set(3000, 15000, 11)
    one, _ = hip_table(b, o, k)
    many, _ = hip_table(b, o, k, batches=5)
    assert_tables_equal(many, one, "5 batches vs 1")


@pytest.mark.parametrize("k,wide", [(21, True), (15, False), (17, False), (63, False), (77, False), (99, False)])
def test_forced_overflow_sweeps(k, wide, knob):
    """Tiny LDS tables force the multi-sweep path (a closed table overflows whole keys to the next sweep).
    Compact records (k <= 21) need >= 2k - 34 fine bits, so k = 15, 17 cover them with one fine bucket."""
    b, o = synth_set(3000, 50000, 13)
    exp = oracle_table(b, o, k)
    knob("cap", 64)
    knob("fine_bits", 0)
    if wide:
        knob("wide_records", 1)
    got, st = hip_table(b, o, k)
    assert st["overflow_sweeps"] > 0
    assert_tables_equal(got, exp, "forced overflow")
    check_stats(st)


@pytest.mark.parametrize("k,wide", [(15, False), (21, True), (63, False), (77, False)])
def test_forced_overflow_hot_sweep(k, wide, knob):
    """A hot first sweep (>= 0xC000 records: the checked round loop with its round barrier and clamp) that
    overflows a 64-slot table: the poly-A k-mer's bucket also holds ~100-200 distinct keys of the random reads,
    so keys are deferred with the per-wave defer positions, then counted by a re-sweep with its own round bound
    (no earlier test overflowed a non-cold sweep)."""
    b, o = hot_set()
    exp = oracle_table(b, o, k)
    knob("cap", 64)
    knob("fine_bits", 0)
    if wide:
        knob("wide_records", 1)
    got, st = hip_table(b, o, k)
    assert st["max_bucket"] >= 0xC000, st["max_bucket"]
    assert st["overflow_sweeps"] > 0
    assert_tables_equal(got, exp, f"hot sweep overflow k={k}")


def test_add_seqs_matches_packed():
    b, o = synth_set(500, 5000, 21)
    pr = m.PackedReads.from_arrays(b, o)
    seqs = []
    for i in range(pr.get_local_num_reads()):
        _, s, q = pr.get_read(i)
        seqs.append("".join(ch.lower() if ord(qq) < 33 + 20 else ch for ch, qq in zip(s, q)))
    with m.KmerCounter(21) as c:
        c.add_seqs(seqs)
        c.finish()
        got = c.fetch()
    assert_tables_equal(got, oracle_table(b, o, 21), "add_seqs")


def test_reset_and_reuse():
    b1, o1 = synth_set(800, 6000, 31)
    b2, o2 = synth_set(900, 7000, 32)
    with m.KmerCounter(33) as c:
        for b, o in ((b1, o1), (b2, o2), (b1, o1)):
            c.add_packed_reads(b, o)
            c.finish()
            assert_tables_equal(c.fetch(), oracle_table(b, o, 33), "reuse")
            c.reset()


def test_n_longs_padding():
    b, o = synth_set(600, 5000, 41)
    got, _ = hip_table(b, o, 21, n_longs=2)
    exp = oracle_table(b, o, 21)
    assert got.keys.shape[1] == 2 and (got.keys[:, 1] == 0).all()
    assert_tables_equal(m.KmerTable(21, got.keys[:, :1].copy(), got.counts, got.left, got.right), exp, "n_longs=2")


def test_device_tensor_input():
    torch = pytest.importorskip("torch")
    b, o = synth_set(1000, 8000, 51)
    bt = torch.from_numpy(b).cuda()
    ot = torch.from_numpy(o.astype(np.int64)).cuda()
    with m.KmerCounter(21) as c:
        c.add_tensors(bt, ot)
        c.finish()
        got = c.fetch()
    assert_tables_equal(got, oracle_table(b, o, 21), "device tensors")


def test_bad_input_rejected():
    b, o = synth_set(50, 2000, 3)
    b = b.copy()
    b[17] = 6  # code 6 is not A,C,G,T,N: the reference DIEs
    with m.KmerCounter(21) as c:
        c.add_packed_reads(b, o)
        with pytest.raises(m.kcount.N.MhmkcError) as e:
            c.finish()
        assert e.value.code == -6


def test_empty_input():
    with m.KmerCounter(21) as c:
        c.add_packed_reads(np.zeros(0, np.uint8), np.zeros(1, np.uint64))
        assert c.finish() == 0


@pytest.mark.parametrize("name", sorted(p.name for p in GOLDEN.glob("table_*.tsv.gz")))
def test_golden_fixtures(name):
    _, setname, kk = name[:-len(".tsv.gz")].split("_")
    k = int(kk[1:])
    b, o = read_reads_file(GOLDEN / f"reads_{setname}.txt.gz")
    got, _ = hip_table(b, o, k)
    assert_tables_equal(got, read_table_file(GOLDEN / name, k), name)


@pytest.mark.slow
def test_medium_vs_oracle():
    """400k reads x 150 bp (51M windows) against the oracle."""
    b, o = synth_set(400_000, 2_000_000, 77)
    ref = O.kcount(b, o, 21)
    keys, c, l, r = ref.fetch()
    got, st = hip_table(b, o, 21)
    assert_tables_equal(got, m.KmerTable(21, keys, c, l, r), "medium")
    check_stats(st, ref.stats())


@pytest.mark.slow
def test_c2_scale_properties():
    """Config C2 (10M x 150 bp, G = 50 Mbp, k = 21): size-independent properties at full size —
    one batch equals four batches (order independence), conservation (count_sum == occurrences ==
    10M * 128), distinct == n_out + purged, every output key is canonical and unique."""
    g = m.synth_genome(50_000_000, 2)
    b, o = m.synth_reads(g, 10_000_000, 150, 2)
    one, st = hip_table(b, o, 21)
    assert st["occurrences"] == 10_000_000 * 128
    check_stats(st)
    four, st4 = hip_table(b, o, 21, batches=4)
    assert st4["distinct"] == st["distinct"]
    assert_tables_equal(four, one, "C2: 4 batches vs 1")
    keys = one.sorted().keys[:, 0]
    assert (np.diff(keys.astype(np.uint64)) > 0).all()
    # canonical: key <= revcomp(key) on a sample
    idx = np.random.default_rng(0).choice(len(keys), 2000, replace=False)
    for i in idx:
        kk = np.array([keys[i]], dtype=np.uint64)
        rc = O.kmer_revcomp(kk, 21)
        assert int(kk[0]) <= int(rc[0])


# ---- contig pass (add_ctg_kmers -> insert_supermer_from_ctg) ----------------------------------------

def ctg_table(b, o, seqs, depths, k, splits=1, **kw):
    with m.KmerCounter(k, **kw) as c:
        c.add_packed_reads(b, o)
        cuts = [len(seqs) * i // splits for i in range(splits + 1)]
        for a, z in zip(cuts[:-1], cuts[1:]):
            c.add_ctgs(seqs[a:z], depths[a:z])
        c.finish()
        return c.fetch(), c.stats()


@pytest.mark.parametrize("k,dmin", [(21, 2), (21, 1), (21, 3), (33, 2), (55, 2), (63, 4), (77, 2), (99, 3), (31, 2)])
def test_contig_pass_vs_oracle(k, dmin):
    """Reads, then contigs in order (replacement of non-UU / singleton read entries, min of agreeing contig
    depths, conflicts purged, contig-only k-mers), bit-exact with the reference's sequential rules."""
    b, o, seqs, depths = ctg_set(seed=40 + k + dmin)
    got, st = ctg_table(b, o, seqs, depths, k, dmin_thres=dmin)
    assert st["ctg_kmers"] > 0
    assert_tables_equal(got, oracle_ctg_table(b, o, seqs, depths, k, dmin_thres=dmin), f"contigs k={k} dmin={dmin}")
    assert st["distinct"] == st["n_out"] + st["purged"]


def test_contig_pass_order_kept_across_calls():
    b, o, seqs, depths = ctg_set(seed=77)
    got, _ = ctg_table(b, o, seqs, depths, 21, splits=4)
    assert_tables_equal(got, oracle_ctg_table(b, o, seqs, depths, 21), "contigs in 4 calls")


@pytest.mark.parametrize("k,wide", [(21, True), (17, False), (63, False)])
def test_contig_pass_with_overflow_sweeps(k, wide, knob):
    """Tiny LDS tables: read entries are spread over several sweeps of a bucket; a contig k-mer must meet
    its read entry in whichever sweep holds it, and only count as contig-only after the last sweep."""
    b, o, seqs, depths = ctg_set(seed=91, n_reads=600)
    knob("cap", 64)
    knob("fine_bits", 0)
    if wide:
        knob("wide_records", 1)
    got, st = ctg_table(b, o, seqs, depths, k)
    assert st["overflow_sweeps"] > 0
    assert_tables_equal(got, oracle_ctg_table(b, o, seqs, depths, k), "contigs + overflow sweeps")


def test_contig_pass_exact_partition(knob):
    b, o, seqs, depths = ctg_set(seed=92)
    knob("exact", 1)
    got, _ = ctg_table(b, o, seqs, depths, 33)
    assert_tables_equal(got, oracle_ctg_table(b, o, seqs, depths, 33), "contigs, exact partition")


def test_contigs_without_reads():
    _, _, seqs, depths = ctg_set(seed=93)
    b, o = np.zeros(0, np.uint8), np.zeros(1, np.uint64)
    got, st = ctg_table(b, o, seqs, depths, 21)
    assert st["occurrences"] == 0
    assert_tables_equal(got, oracle_ctg_table(b, o, seqs, depths, 21), "contigs only")


def test_analyze_kmers_with_contigs():
    """The analyze_kmers mirror (src/kcount/kcount.cpp:140-157) with a Contigs list."""
    b, o, seqs, depths = ctg_set(seed=94)
    pr = m.PackedReads.from_arrays(b, o)
    dht = m.KmerDHT(21)
    ctgs = [(s_, float(d) + 0.7) for s_, d in zip(seqs, depths)]  # get_uint16_t_depth truncates
    m.analyze_kmers(21, 0, 33, [pr], 2, ctgs, dht)
    assert_tables_equal(dht.table, oracle_ctg_table(b, o, seqs, depths, 21), "analyze_kmers + contigs")
    dht.counter.close()


@pytest.mark.parametrize("k", [21, 19])
def test_compact_overflow_at_min_fine_bits(k, knob):
    """Compact records at their smallest fine partition (2k - 34 fine bits at k = 21): ~120 distinct
    k-mers per fine bucket against 64-slot tables, so most buckets need several sweeps."""
    b, o = synth_set(60000, 4_000_000, 23)
    exp = oracle_table(b, o, k)
    knob("cap", 64)
    knob("fine_bits", 0)
    got, st = hip_table(b, o, k)
    assert st["overflow_sweeps"] > 0
    assert_tables_equal(got, exp, "compact overflow")
    check_stats(st)


@pytest.mark.parametrize("k", [21, 12, 33, 47, 63, 65, 77, 95, 99, 127])
def test_compact_equals_wide_records(k, knob):
    """The mixed record layouts (compact 4/5-byte at k <= 21, two-word m2_mix at 33 <= k <= 63, three- and four-word
    mx_mix at 64 < k < 128; the key rebuilt from the bucket digits) and the plain key-word records give the same
    table, through the capped and the exact partition paths."""
    b, o = synth_set(20000, 300000, 31)
    cmp_t, st_c = hip_table(b, o, k)
    knob("wide_records", 1)
    wide_t, st_w = hip_table(b, o, k)
    assert_tables_equal(cmp_t, wide_t, "compact vs wide")
    knob("wide_records", 0)
    knob("exact", 1)
    exact_t, _ = hip_table(b, o, k)
    assert_tables_equal(exact_t, wide_t, "compact exact vs wide")
    for key in ("distinct", "n_out", "purged", "count_sum"):
        assert st_c[key] == st_w[key], key


@pytest.mark.parametrize("k", [21, 63])
def test_distinct_sketch_estimate(k):
    """The HyperLogLog sketch that sizes the fine partition is within 12 % of the true distinct count."""
    b, o = synth_set(40000, 2_000_000, 41)
    _, st = hip_table(b, o, k)
    assert st["distinct"] > 0
    assert abs(st["distinct_estimate"] - st["distinct"]) <= 0.12 * st["distinct"], (st["distinct_estimate"], st["distinct"])


# ---- round 2: host chunks, stream ordering, dmin at finish, overflow guard ----------------------------


@pytest.mark.parametrize("nib", [0, 1, 2])
@pytest.mark.parametrize("k,chunk", [(21, 700), (63, 1000), (33, 100000)])
def test_host_chunks_equal_oracle(k, chunk, nib, knob):
    """mhmkc_add_reads copies a host batch in chunks of whole reads, each extracted as a slice view (an aligned
    byte base plus a head offset) as soon as it lands: ragged reads (empty, shorter than k, N runs, poly-A)
    over many chunk boundaries give the oracle's table, with the bases sent as bytes (nib 0) or as nibbles that the
    device expands back (nib 1 with u32 offset distances, 2 with u64 offsets: odd chunk starts and ends split nibble
    pairs)."""
    knob("chunk_bytes", chunk)
    knob("h2d_nib", nib)
    b, o = edge_case_set(seed=17 + k)
    with m.KmerCounter(k) as c:
        c.add_packed_reads(b, o)
        c.finish()
        got, st = c.fetch(), c.stats()
    assert st["h2d_chunks"] >= (2 if chunk < 10000 else 1)
    if nib:  # nibbles, and the offsets as u32 distances from each chunk's first byte (2: as they are, u64)
        offs_bytes = (4 if nib == 1 else 8) * (o.size - 1 + st["h2d_chunks"])
        assert int(o[-1]) // 2 <= st["h2d_bytes"] - offs_bytes <= (int(o[-1]) + st["h2d_chunks"]) // 2
    else:
        assert st["h2d_bytes"] == int(o[-1]) + 8 * (o.size - 1) + 8 * st["h2d_chunks"]
    assert_tables_equal(got, oracle_table(b, o, k), f"host chunks k={k} nib={nib}")
    check_stats(st)


@pytest.mark.parametrize("qcut", [0, 1, 19, 20, 31, 32])
def test_host_nibbles_quality_cutoffs(qcut, knob):
    """The nibble H2D keeps one quality bit, q >= cutoff, per base: for cutoffs at both ends of the accepted [0, 32]
    and around the default, the table equals the oracle's and the byte H2D's, with the codes A, C, G, T, N and every
    quality 0-31 in the input (codes 5-7 are an input error: test_host_nibbles_bad_code_reported)."""
    b, o = synth_set(600, 20000, 71)
    rng = np.random.default_rng(qcut + 3)
    b = ((b & 7) | (rng.integers(0, 32, b.size, dtype=np.uint8) << 3)).astype(np.uint8)
    knob("chunk_bytes", 3001)
    tabs = []
    for nib in (1, 0):
        knob("h2d_nib", nib)
        got, st = hip_table(b, o, 21, qual_cutoff=qcut)
        check_stats(st)
        tabs.append(got)
    assert_tables_equal(tabs[0], oracle_table(b, o, 21, qual_cutoff=qcut), f"nibbles qcut={qcut}")
    assert_tables_equal(tabs[0], tabs[1], f"nibbles vs bytes qcut={qcut}")


def test_host_nibbles_empty_read_runs(knob):
    """Chunks are also cut at a read count (chunk_bytes / 32, at least 64): runs of hundreds of empty reads make chunks
    with no bases at all between ordinary ones."""
    b, o = synth_set(400, 20000, 73)
    lens = np.diff(o.astype(np.int64))
    lens = np.concatenate([lens[:150], np.zeros(700, np.int64), lens[150:300], np.zeros(130, np.int64), lens[300:]])
    o2 = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    knob("chunk_bytes", 2048)
    knob("h2d_nib", 1)
    got, st = hip_table(b, o2, 21)
    assert st["h2d_chunks"] >= 15
    assert_tables_equal(got, oracle_table(b, o2, 21), "empty read runs")


@pytest.mark.parametrize("k", [21, 63])
def test_host_local_rounds_equal_oracle(k, knob):
    """One rank, a host batch in many chunks (local rounds, the default): the chunks' slabs are fine-partitioned as
    they land (the incremental layout of DESIGN.md §3.5f, set once they hold 40 % of the windows) and finish only
    counts; the table equals the CPU restatement's and the one partitioned at finish (local_rounds 0)."""
    b, o = synth_set(200000, 2_000_000, 74)
    knob("local_rounds", 1)
    knob("chunk_bytes", 8 << 20)  # (the first chunk, 2 MB, samples >= 4096 records of one coarse bucket also at k = 63)
    knob("h2d_nib", 1)
    got, st = hip_table(b, o, k)
    inc = {key: st[key] for key in ("inc_rounds", "inc_fallbacks", "inc_redone_coarse", "h2d_chunks", "slabs")}
    assert st["inc_rounds"] >= 4 and st["inc_fallbacks"] == 0 and st["inc_redone_coarse"] == 0, inc
    check_stats(st)
    exp = O.kcount_mt(b, o, k)
    assert_tables_equal(got, m.KmerTable(k, *exp.fetch()), f"local rounds k={k}")
    knob("local_rounds", 0)
    ref, st0 = hip_table(b, o, k)
    assert st0["inc_rounds"] == 0
    assert_tables_equal(got, ref, f"local rounds vs at finish k={k}")


def test_host_local_rounds_hot_kmer_redo(knob):
    """Local rounds with a skewed batch: 800 poly-A reads at its end, after 120k random reads. The poly-A k-mer's fine
    bucket overflows its capped segment; that coarse bucket alone is counted again with exact sizes at finish."""
    b, o = hot_set(n_reads=120000, genome_len=400000, n_poly=800, seed=4)
    knob("local_rounds", 1)
    knob("chunk_bytes", 5 << 20)
    knob("h2d_nib", 1)
    got, st = hip_table(b, o, 21)
    inc = {key: st[key] for key in ("inc_rounds", "inc_fallbacks", "inc_redone_coarse", "h2d_chunks", "slabs")}
    assert st["inc_rounds"] >= 3 and st["inc_fallbacks"] == 0 and st["inc_redone_coarse"] == 1, inc
    assert_tables_equal(got, oracle_table(b, o, 21), "local rounds, hot k-mer")


@pytest.mark.parametrize("adapt", [1, 2])
def test_host_nibbles_mixed_raw_chunks(adapt, knob):
    """From pinned host memory a chunk goes as PackedRead bytes when the wire has drained while the host packed
    (h2d_adapt 1; 2 forces every other chunk): raw and nibble chunks in one batch, odd chunk boundaries, every quality,
    give the oracle's table."""
    torch = pytest.importorskip("torch")
    b, o = synth_set(3000, 20000, 75)
    rng = np.random.default_rng(76)
    b = ((b & 7) | (rng.integers(0, 32, b.size, dtype=np.uint8) << 3)).astype(np.uint8)
    hb = torch.from_numpy(b).pin_memory().numpy()
    knob("chunk_bytes", 7001)
    knob("h2d_nib", 1)
    knob("h2d_adapt", adapt)
    with m.KmerCounter(21) as c:
        c.add_packed_reads(hb, o)
        c.finish()
        got, st = c.fetch(), c.stats()
    assert st["h2d_raw_chunks"] >= (st["h2d_chunks"] // 2 if adapt == 2 else 1), (st["h2d_raw_chunks"], st["h2d_chunks"])
    if adapt == 2:
        assert st["h2d_raw_chunks"] < st["h2d_chunks"]
    assert_tables_equal(got, oracle_table(b, o, 21), f"raw and nibble chunks, adapt={adapt}")


def test_host_nibbles_bad_code_reported(knob):
    """A byte with code 5-7 sent as a nibble still reaches the device's input check (error, no table)."""
    b, o = synth_set(200, 5000, 72)
    b = b.copy()
    b[int(o[100]) + 7] = (b[int(o[100]) + 7] & 0xF8) | 6
    knob("h2d_nib", 1)
    with m.KmerCounter(21) as c:
        c.add_packed_reads(b, o)
        with pytest.raises(m.MhmkcError) as e:
            c.finish()
        assert e.value.code == -6


def test_device_input_ordered_after_torch_stream():
    """Tensors written by an asynchronous copy on torch's current stream and handed over at once: the counter
    orders its stream after torch's (mhmkc_wait_stream), no torch.cuda.synchronize() needed."""
    torch = pytest.importorskip("torch")
    b, o = synth_set(3000, 20000, 52)
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        bt = torch.from_numpy(b).pin_memory().cuda(non_blocking=True)
        ot = torch.from_numpy(o.astype(np.int64)).pin_memory().cuda(non_blocking=True)
        with m.KmerCounter(21) as c:
            c.add_tensors(bt, ot, n_bases=int(o[-1]))
            c.finish()
            got = c.fetch()
    assert_tables_equal(got, oracle_table(b, o, 21), "after a torch stream")


def test_device_offsets_checked():
    torch = pytest.importorskip("torch")
    b, o = synth_set(200, 5000, 53)
    oo = o.astype(np.int64).copy()
    oo[50] = oo[51] + 1  # decreasing
    with m.KmerCounter(21) as c:
        with pytest.raises(m.MhmkcError) as e:
            c.add_tensors(torch.from_numpy(b).cuda(), torch.from_numpy(oo).cuda(), n_bases=int(o[-1]))
        assert e.value.code == -1


@pytest.mark.parametrize("k", [21, 63])
def test_analyze_kmers_dmin_thres(k):
    """The Python mirror: KmerDHT built first (dmin unknown), analyze_kmers(..., dmin_thres = 3, ...) decides."""
    b, o = synth_set(1500, 8000, 80 + k)
    dht = m.KmerDHT(k)
    m.analyze_kmers(k, 0, 33, [m.PackedReads.from_arrays(b, o)], 3, [], dht)
    exp = oracle_table(b, o, k, dmin_thres=3)
    assert_tables_equal(dht.table, exp, "analyze_kmers dmin 3")
    # the input must make dmin 3 matter, or the check above could not tell set_dmin_thres from a no-op
    with pytest.raises(AssertionError):
        assert_tables_equal(dht.table, oracle_table(b, o, k, dmin_thres=2), "dmin 3 vs 2")
    dht.counter.close()


def _hot_key_last_bucket(k: int) -> str:
    """A canonical k-mer whose partition hash has the top 19 bits set: the last fine bucket of the last coarse
    bucket for any fine-bit count <= 11 (compact cmix at k <= 21, m2_mix at 33..63, MurmurHash3 otherwise)."""
    rng = np.random.default_rng(k)
    nl = k // 32 + 1
    B = 2 * k
    FK = (0x9E3779, 0x85EBCA, 0xC2B2AE, 0x27D4EB)  # kmer_ops.hpp cunmix (Feistel)

    def f(v, c, n):
        return ((((v ^ (v >> 9)) & 0xffffff) * c & 0xffffffff) >> 11) & ((1 << n) - 1)

    def cunmix(y):  # three rounds
        a, bb = B >> 1, B - (B >> 1)
        R, L = y & ((1 << a) - 1), y >> a
        L ^= f(R, FK[2], bb)
        R ^= f(L, FK[1], a)
        L ^= f(R, FK[0], bb)
        return (L << a) | R

    M2C = (0x9E3779, 0x85EBCB, 0xC2B2AF, 0x27D4EB, 0x165667, 0x3A2659)  # kmer_ops.hpp m2_h
    M32 = 0xffffffff

    def m2_h(v, c1, c2):
        hi = (v >> 32) & M32
        u = (v & M32) ^ (((hi << 7) | (hi >> 25)) & M32)
        u ^= u >> 16
        u = ((u & 0xffffff) * c1) & M32
        u ^= u >> 15
        u = ((u & 0xffffff) * c2) & M32
        return u ^ (u >> 16)

    def m2_unmix(L, R):  # (L', R') -> key words; two rounds
        R ^= m2_h(L, M2C[2], M2C[3])
        L ^= m2_h(R, M2C[0], M2C[1]) << (k - 32)
        x = (L << k) | R  # 2k bits, left-aligned in 128
        x <<= 128 - 2 * k
        return np.array([x >> 64, x & ((1 << 64) - 1)], dtype=np.uint64)

    for _ in range(1 << 22):
        if 33 <= k <= 63:  # m2_unmix of an L' with the top bits set (the mixed two-word records' digits)
            L = (((1 << 19) - 1) << (k - 19)) | int(rng.integers(0, 1 << (k - 19)))
            key = m2_unmix(L, int(rng.integers(0, 1 << 62)) & ((1 << k) - 1))
        elif k <= 21:  # cunmix of a y with the top bits set
            y = (((1 << 19) - 1) << (B - 19)) | int(rng.integers(0, 1 << (B - 19)))
            key = np.array([cunmix(y) << (64 - B)], dtype=np.uint64)
        else:
            key = np.array([int(x) for x in rng.integers(0, 1 << 62, nl)], dtype=np.uint64)
            key[-1] &= np.uint64((~((1 << (64 - 2 * (k - 32 * (nl - 1)))) - 1)) & ((1 << 64) - 1))
            if (O.kmer_hash(key) >> 45) != (1 << 19) - 1:
                continue
        rc = O.kmer_revcomp(key, k)
        if tuple(int(x) for x in key) <= tuple(int(x) for x in rc):
            return O.kmer_to_string(key, k)
    raise AssertionError("no key found")


@pytest.mark.parametrize("k", [21, 33, 63, 77])
def test_capped_overflow_in_last_bucket(k):
    """a hot k-mer in the LAST fine bucket of the LAST coarse bucket overflows its capped
    fine bucket. k_count must not run over the bucket (it returns at once when k_part_scatter flagged the
    overflow); the exact rerun gives the oracle's table."""
    s = _hot_key_last_bucket(k)
    b0, o0 = synth_set(300, 20000, 3 + k)
    hot = m.PackedReads.pack("A" + s + "C", "I" * (k + 2))  # one counted window: the hot k-mer
    reads = [b0[o0[i]:o0[i + 1]] for i in range(300)] + [hot] * 30000
    lens = np.array([x.size for x in reads], dtype=np.uint64)
    o = np.zeros(len(reads) + 1, dtype=np.uint64)
    np.cumsum(lens, out=o[1:])
    b = np.concatenate(reads).astype(np.uint8)
    got, st = hip_table(b, o, k)
    assert st["exact_reruns"] >= 1
    exp = oracle_table(b, o, k)
    assert_tables_equal(got, exp, "hot k-mer in the last bucket")
    nl = k // 32 + 1
    hk = O.kmer_from_string(s, nl)
    row = np.flatnonzero((exp.keys == hk).all(axis=1))
    assert row.size == 1 and exp.counts[row[0]] == 30000


@pytest.mark.slow
@pytest.mark.timeout(1200)
@pytest.mark.parametrize("k", [21, pytest.param(63, marks=pytest.mark.skipif(
    os.environ.get("MHMKC_SCALE_TESTS") != "1", reason="k = 63 at scale: the eight-rank C4 test (8.6e9 occurrences, "
    "all key ranges) supersedes it inside the driver's test window (MHMKC_SCALE_TESTS=1 runs it)")), 99])
def test_c2_full_table_vs_cpu_restatement(k):
    """config C2 at full size (10M x 150 bp, G = 50 Mbp, seed 2) through the host path
    (chunked nibble H2D, local rounds), every row of the table compared with the multi-threaded CPU restatement (oracle/kcount_mt.c,
    itself pinned to the single-threaded oracle and the golden fixtures); k = 21, k = 63 (with MHMKC_SCALE_TESTS=1;
    the eight-rank C4 test covers k = 63 at 8.6e9 occurrences) and k = 99 (mixed four-word records, DESIGN.md
    §3.7c)."""
    g = m.synth_genome(50_000_000, 2)
    b, o = m.synth_reads(g, 10_000_000, 150, 2, threads=16)
    del g
    got, st = hip_table(b, o, k)
    assert st["occurrences"] == 10_000_000 * (150 - k - 1)
    # (one rank, twelve 128 MB chunks: fine-partitioned as they land)
    assert st["inc_rounds"] >= 10 and st["inc_fallbacks"] == 0, (st["inc_rounds"], st["inc_fallbacks"])
    check_stats(st)
    t = O.kcount_mt(b, o, k, threads=16)
    keys, c, l, r = t.fetch()
    ref = m.KmerTable(k, keys, c, l, r)
    rs = t.stats()
    del t
    assert (st["distinct"], st["purged"], st["n_out"]) == (rs["distinct"], rs["purged"], rs["n_out"])
    assert_tables_equal(got, ref, f"C2 k={k}: GPU vs CPU restatement")


def long_ragged_set(k: int, seed: int = 61):
    """Reads of every awkward length for the valid-window list of the two-word extraction: empty, < k + 2,
    k + 2 (one window), k + 3, 150, and reads far longer than a 2048-base tile (a read spanning several
    tiles, starting before the tile it is counted in), concatenated in a random order."""
    rng = np.random.default_rng(seed)
    g = m.synth_genome(400_000, seed)
    lens = [0, 1, k, k + 1, k + 2, k + 3, 150, 151, 2047, 2048, 2049, 4000, 9000]
    reads = []
    for i in range(600):
        L = lens[i % len(lens)] if i % 3 else int(rng.integers(0, 300))
        a = int(rng.integers(0, g.size - L - 1))
        q = np.where(rng.random(L) < 0.03, 5, 31).astype(np.uint8)
        reads.append((g[a:a + L] & 7) | (q << 3))
    rng.shuffle(reads)
    offs = np.zeros(len(reads) + 1, dtype=np.uint64)
    np.cumsum([r.size for r in reads], out=offs[1:])
    return np.concatenate(reads).astype(np.uint8), offs


@pytest.mark.parametrize("k", [33, 47, 63, 77, 99, 21])
def test_valid_window_walk_long_and_ragged_reads(k, knob):
    """Two-word extraction over the listed valid windows == the oracle, for reads of length 0 .. 9000 (reads
    crossing several extraction tiles), whole and as host chunks (slice views with a head offset). At k = 77, 99
    the long reads count nearly every window of a tile, more than the extraction stages at once (kECap: 1024
    records), so their records go out in several rounds."""
    b, o = long_ragged_set(k)
    exp = oracle_table(b, o, k)
    got, st = hip_table(b, o, k)
    assert_tables_equal(got, exp, f"long/ragged reads, k={k}")
    check_stats(st)
    knob("chunk_bytes", 5000)
    got2, _ = hip_table(b, o, k)
    assert_tables_equal(got2, exp, f"long/ragged reads in 5000-byte chunks, k={k}")


@pytest.mark.parametrize("k,nl", [(21, 0), (63, 0), (21, 2), (99, 0), (77, 0), (21, 6)])
def test_fetch_ordered(k, nl):
    """mhmkc_fetch_ordered: the same rows as mhmkc_fetch, ordered by the top 32 bits of mhmkc_map_hash (the slot
    order of the C++ adapter's KmerMap)."""
    b, o = synth_set(2000, 10000, 90 + k)
    with m.KmerCounter(k, n_longs=nl) as c:
        c.add_packed_reads(b, o)
        c.finish()
        plain = c.fetch()
        ordered = c.fetch(ordered=True)
    assert_tables_equal(ordered, plain, "ordered fetch")
    top = np.array([m.kcount.map_hash(row) >> 32 for row in ordered.keys.tolist()], dtype=np.uint64)
    assert len(top) > 1000 and (np.diff(top.astype(np.int64)) >= 0).all()


@pytest.mark.parametrize("k,passes", [(21, "3"), (33, "2"), (63, "5"), (99, "4"), (77, "256"), (19, "7")])
def test_finish_passes_vs_oracle(k, passes, monkeypatch):
    """The owned hash range counted in several finish passes (MHMKC_PASSES: each pass fine-partitions and counts its
    coarse buckets into the same buffer and appends its survivors to the output): the table is the one-pass table."""
    monkeypatch.setenv("MHMKC_PASSES", passes)
    b, o = synth_set(2500, 12000, 600 + k)
    got, st = hip_table(b, o, k, batches=2)
    assert st["finish_passes"] == min(int(passes), 128 if k > 64 else 256)
    assert_tables_equal(got, oracle_table(b, o, k), f"{passes} passes, k={k}")
    check_stats(st)


@pytest.mark.parametrize("k,passes", [(21, "4"), (63, "3"), (99, "2")])
def test_finish_passes_with_contigs(k, passes, monkeypatch):
    """Contig k-mers are folded once and applied in the pass that counts their bucket (CountParams.ctg_base)."""
    monkeypatch.setenv("MHMKC_PASSES", passes)
    b, o, seqs, depths = ctg_set(seed=610 + k)
    got, st = ctg_table(b, o, seqs, depths, k)
    assert st["ctg_kmers"] > 0 and st["finish_passes"] == int(passes)
    assert_tables_equal(got, oracle_ctg_table(b, o, seqs, depths, k), f"contigs over {passes} passes, k={k}")


@pytest.mark.parametrize("k,passes,exact", [(21, "1", False), (21, "3", False), (63, "2", True), (99, "1", False)])
def test_output_overflow_redoes_the_pass(k, passes, exact, monkeypatch, knob):
    """An output sized too small (the test knob out_cap: rows) fills: the pass writes nothing past it, the output grows to
    the rows its cursor counted (the earlier passes' rows kept) and the pass is redone; the table is unchanged."""
    monkeypatch.setenv("MHMKC_PASSES", passes)
    knob("out_cap", 100)
    if exact:
        knob("exact", 1)
    b, o = synth_set(2500, 12000, 620 + k)
    got, st = hip_table(b, o, k)
    assert st["out_reruns"] >= 1
    assert_tables_equal(got, oracle_table(b, o, k), f"output overflow, {passes} passes, k={k}")
    check_stats(st)
    assert st["device_bytes_peak"] >= st["device_bytes"] > 0


@pytest.mark.parametrize("k,pinned", [(21, False), (63, True)])
def test_fetch_into_existing_buffers(k, pinned):
    """fetch(out=...) fills the caller's arrays (larger than the table; pinned host memory is reached by one DMA,
    pageable memory through the staging buffers): the rows equal a plain fetch's, ordered or not."""
    torch = pytest.importorskip("torch")
    b, o = synth_set(2000, 10000, 95 + k)
    with m.KmerCounter(k) as c:
        c.add_packed_reads(b, o)
        n = c.finish()
        plain = c.fetch()
        nl, rows = c.n_longs, n + 100
        if pinned:
            arrs = [torch.empty(s, dtype=t, pin_memory=True).numpy() for s, t in
                    (((rows, nl), torch.int64), (rows, torch.int16), (rows, torch.uint8), (rows, torch.uint8))]
            out = m.KmerTable(k, arrs[0].view(np.uint64), arrs[1].view(np.uint16), arrs[2], arrs[3])
        else:
            out = m.KmerTable(k, np.zeros((rows, nl), np.uint64), np.zeros(rows, np.uint16), np.zeros(rows, np.uint8),
                              np.zeros(rows, np.uint8))
        for ordered in (False, True):
            got = c.fetch(ordered=ordered, out=out)
            assert len(got) == n
            assert_tables_equal(got, plain, f"fetch into existing buffers, ordered={ordered}")


@pytest.mark.parametrize("chunk", [257, 258, 259, 1000, 4099])
def test_fetch_staged_chunk_tails(chunk, knob):
    """A fetch into pageable memory goes through pinned staging chunks, each copied out by four host threads. With
    staging chunks of 257-259 bytes (quarters of 64.25-64.75 bytes) and other odd sizes, every byte of every array
    (keys, counts, left, right; plain and ordered) arrives: the quarter split once rounded down and dropped a chunk's
    last 1-3 bytes (the last two rows' left/right bytes of a C4 rank's 65,094,658-row table)."""
    b, o = synth_set(2000, 10000, 1234)
    with m.KmerCounter(63) as c:
        c.add_packed_reads(b, o)
        n = c.finish()
        ref, ref_o = c.fetch(), c.fetch(ordered=True)  # small arrays: one DMA straight into them
        assert n >= 2 * chunk  # (every array goes through the staging chunks)
        knob("d2h_chunk", chunk)
        got, got_o = c.fetch(), c.fetch(ordered=True)
    for a, e in ((got, ref), (got_o, ref_o)):
        assert np.array_equal(a.keys, e.keys) and np.array_equal(a.counts, e.counts)
        assert np.array_equal(a.left, e.left) and np.array_equal(a.right, e.right)
    assert np.isin(got.left.view(np.uint8), np.frombuffer(b"ACGTXF", np.uint8)).all()
