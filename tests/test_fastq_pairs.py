"""Read-pair merging (merge_reads, src/merge_reads.cpp:237-588) on the device, against the C restatement
(oracle/merge_reads.c), which is itself cross-checked here against an independent string-level restatement
(tests/ref_merge_literal.py). Parity unpinned by reference outputs: the reference's merge_reads needs UPC++
and its CI data is downloaded; the two restatements and review against the cited lines pin
it. Compared: merge_reads' PackedReads (bytes and offsets, merged read + "N" mate or both mates), the merge
statistics, errors where the reference DIEs, and the count table of the merged reads."""
from __future__ import annotations

import re

import numpy as np
import pytest

import common as c
import oracle_lib as O
import ref_merge_literal as R

VARIANTS = {
    "default": {},
    "many_n": {"n_rate": 0.02, "seed": 3},           # N / IUPAC in most pairs: the quality-scratch path
    "no_iupac": {"iupac": False, "seed": 4},
    "long_frag": {"frag_mean": 330, "frag_sd": 60, "seed": 5},   # most pairs do not overlap
    "short_frag": {"frag_mean": 120, "frag_sd": 30, "seed": 6},  # mate 2 runs past mate 1's start
    "noisy": {"subst": 0.04, "low_q": 0.15, "seed": 7},
    "long_reads": {"read_len": 900, "frag_mean": 1500, "frag_sd": 300, "seed": 8},
    "qoff64": {"qual_offset": 64, "seed": 9},
}


def _text(v, n=1500):
    kw = dict(VARIANTS[v])
    return c.paired_fastq_text(n, **kw), kw.get("qual_offset", 33)


def _bad(name):
    good = c.paired_fastq_text(6, seed=11)
    recs = good.split(b"\n")
    if name == "pair_name":
        recs[4] = b"@other/2"  # record 1 (mate 2 of pair 0)
    elif name == "pair_number":
        recs[4] = recs[0]      # record 1 carries mate 1's name
    elif name == "char2":
        recs[5] = b"X" + recs[5][1:]
    elif name == "char1":
        recs[1] = b"X" + recs[1][1:]
    elif name == "qual":       # pair 0 overlaps fully with one mismatch whose mate-1 quality is below the offset
        rng = np.random.default_rng(1)
        s1 = bytes(rng.choice(list(b"ACGT"), size=100).astype(np.uint8))
        comp = bytes.maketrans(b"ACGT", b"TGCA")
        s2 = bytearray(s1.translate(comp)[::-1])
        s2[40] = ord("A") if s2[40] != ord("A") else ord("C")  # mate-1 base 59 mismatches
        q1 = bytearray(b"I" * 100)
        q1[59] = 0x1f
        recs[0:8] = [b"@bad/1", s1, b"+", bytes(q1), b"@bad/2", bytes(s2), b"+", b"I" * 100]
    return b"\n".join(recs)


# --------------------------------------------------------------------------------------------------
# CPU: the two restatements agree


@pytest.mark.parametrize("variant", sorted(VARIANTS))
def test_oracle_merge_equals_literal(variant):
    t, qoff = _text(variant, 300)
    b, o, st = O.merge_fastq(t, qoff)
    b2, o2, st2 = R.merge_fastq(t, qoff)
    assert st == st2
    assert list(o) == o2 and b.tobytes() == b2


def test_oracle_merge_merges_and_keeps_pairs():
    t, _ = _text("default", 1000)
    b, o, st = O.merge_fastq(t)
    assert st["pairs"] == 1000 and 0.4 * 1000 < st["merged"] < 1000
    lens = np.diff(o)
    assert len(lens) == 2000
    assert (lens[1::2] == 1).sum() == st["merged"]  # a dummy "N" mate per merged pair
    assert (b[o[1::2][lens[1::2] == 1]] == 4).all()


def test_oracle_merge_odd_and_empty():
    b, o, st = O.merge_fastq(b"")
    assert list(o) == [0] and st["pairs"] == 0
    t = c.paired_fastq_text(3, seed=2)
    last = t.rstrip(b"\n").rsplit(b"\n", 4)[0] + b"\n"  # drop the last record: pair 2 has no mate 2
    b, o, st = O.merge_fastq(last)
    assert st["pairs"] == 2 and len(o) == 5


@pytest.mark.parametrize("name", ["pair_name", "pair_number", "char2", "char1", "qual"])
def test_oracle_merge_errors(name):
    with pytest.raises(O.FastqError) as e:
        O.merge_fastq(_bad(name))
    assert e.value.record in (0, 1)


# --------------------------------------------------------------------------------------------------
# GPU: the device merge through the C ABI against the oracle

ERRS = {"pair_name": ("MHMKC_EINVAL", "mismatched pair names"), "pair_number": ("MHMKC_EINVAL", "pair numbers"),
        "char2": ("MHMKC_EBADCHAR", "record 1"), "char1": ("MHMKC_EBADCHAR", "record 0"),
        "qual": ("MHMKC_EINVAL", "invalid quality")}


@pytest.mark.gpu
@pytest.mark.parametrize("variant", sorted(VARIANTS))
def test_gpu_merge_equals_oracle(variant):
    import mhm2_proxy_amd as m
    t, qoff = _text(variant, 4000)
    pb, po, pst = O.merge_fastq(t, qoff)
    with m.KmerCounter(21, device=0, qual_offset=qoff) as cnt:
        cnt.add_fastq_pairs(t)
        gb, go = cnt.fastq_packed()
        st = cnt.stats()
    assert len(go) == len(po) and (go == po).all()
    assert (gb == pb).all()
    for key in ("pairs", "merged", "ambiguous", "overlap_bases"):
        assert st["fq_" + key] == pst[key], key


@pytest.mark.gpu
def test_gpu_merge_mixed_lengths():
    """Short and long pairs in one batch: mates around the short-pair limit of k_fq_merge's small-staging instance
    (504 bases, fastq.hip MG_SHORT - 8; unequal mate lengths, so some pairs have one mate on each side), interleaved
    with 150-base and 900-base pairs. The long ones go through the second, 2048-byte instance."""
    import mhm2_proxy_amd as m
    parts = [c.paired_fastq_text(1500, seed=21),
             c.paired_fastq_text(300, seed=22, read_len=506, frag_mean=800, frag_sd=120),
             c.paired_fastq_text(300, seed=23, read_len=900, frag_mean=1500, frag_sd=300),
             c.paired_fastq_text(300, seed=24, read_len=503, frag_mean=700, frag_sd=100),
             c.paired_fastq_text(800, seed=25)]
    t = b"".join(parts)
    pb, po, pst = O.merge_fastq(t, 33)
    with m.KmerCounter(21, device=0) as cnt:
        cnt.add_fastq_pairs(t)
        gb, go = cnt.fastq_packed()
        st = cnt.stats()
    assert len(go) == len(po) and (go == po).all()
    assert (gb == pb).all()
    for key in ("pairs", "merged", "ambiguous", "overlap_bases"):
        assert st["fq_" + key] == pst[key], key
    assert pst["merged"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("k", [21, 63])
def test_gpu_merged_reads_count_equals_oracle(k):
    """End to end: paired FASTQ -> device merge -> count == the oracle's count of the oracle's merge."""
    import mhm2_proxy_amd as m
    t, _ = _text("default", 6000)
    pb, po, _ = O.merge_fastq(t)
    with m.KmerCounter(k, device=0) as cnt:
        cnt.add_fastq_pairs(t)
        cnt.finish()
        got = cnt.fetch().sorted()
    keys, counts, left, right = O.kcount(pb, po, k).fetch()
    assert (got.keys == keys).all() and (got.counts == counts).all()
    assert (got.left == left).all() and (got.right == right).all()


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(ERRS))
def test_gpu_merge_errors(name):
    import mhm2_proxy_amd as m
    code, what = ERRS[name]
    with m.KmerCounter(21, device=0) as cnt:
        with pytest.raises(m.MhmkcError) as got:
            cnt.add_fastq_pairs(_bad(name))
    msg = str(got.value)
    assert msg.startswith(code) and what in msg, msg


@pytest.mark.gpu
def test_gpu_merge_odd_empty_and_device_text():
    import torch

    import mhm2_proxy_amd as m
    t = c.paired_fastq_text(2001, seed=12)
    odd = t.rstrip(b"\n").rsplit(b"\n", 4)[0] + b"\n"
    pb, po, pst = O.merge_fastq(odd)
    with m.KmerCounter(33, device=0) as cnt:
        cnt.add_fastq_pairs(b"")
        gb, go = cnt.fastq_packed()
        assert gb.size == 0 and list(go) == [0]
        cnt.add_fastq_pairs(odd)
        gb, go = cnt.fastq_packed()
        assert (go == po).all() and (gb == pb).all() and cnt.stats()["fq_pairs"] == 2000
        d = torch.from_numpy(np.frombuffer(t, dtype=np.uint8).copy()).cuda()
        cnt.reset()
        cnt.add_fastq_tensor(d, pairs=True)
        gb, go = cnt.fastq_packed()
    pb2, po2, _ = O.merge_fastq(t)
    assert (go == po2).all() and (gb == pb2).all()
