"""FASTQ file ingest with the file I/O overlapped (mhmkc_add_fastq_file / mhmkc_add_fastq_pairs_file, SURVEY.md
§8(f) row 3): the file is read in blocks, each block's last record (pair) is cut and carried into the next one,
and the blocks are parsed, merged and counted on the device. Small blocks (MHMKC_FQ_BLOCK) force many cuts,
including cuts inside every line kind, CRLF line ends, a missing final newline and records longer than a block.
The table must equal the oracle's count of the oracle's parse of the whole file (parity as in test_fastq.py and
test_fastq_pairs.py: pinned by the restatements, not by reference outputs)."""
from __future__ import annotations

import re

import pytest

import common as c
import oracle_lib as O


def _write(tmp_path, name: str, text: bytes):
    p = tmp_path / name
    p.write_bytes(text)
    return p


def _assert_table(got, pb, po, k):
    keys, counts, left, right = O.kcount(pb, po, k).fetch()
    assert (got.keys == keys).all() and (got.counts == counts).all()
    assert (got.left == left).all() and (got.right == right).all()


@pytest.mark.gpu
@pytest.mark.parametrize("k,block,variant", [
    (21, 4093, dict(crlf_every=3, trailing_ws=True, iupac=True, seed=31)),
    (63, 20011, dict(final_newline=False, seed=32)),
    (21, 1 << 28, dict(seed=33)),  # one block: the whole file
])
def test_gpu_fastq_file_equals_oracle(tmp_path, monkeypatch, k, block, variant):
    import mhm2_proxy_amd as m
    b, o = c.synth_set(6000, 60000, 30 + k)
    t = c.fastq_text(b, o, **variant)
    path = _write(tmp_path, "reads.fq", t)
    pb, po = O.fastq_pack(t)
    monkeypatch.setenv("MHMKC_FQ_BLOCK", str(block))
    with m.KmerCounter(k, device=0) as cnt:
        cnt.add_fastq_file(path)
        st = cnt.stats()
        gb, go = cnt.fastq_packed()  # every block's PackedReads, appended
        cnt.finish()
        got = cnt.fetch().sorted()
    assert (go == po).all() and (gb == pb).all()
    assert st["reads"] == len(po) - 1 and st["bases"] == int(po[-1])
    assert st["fq_file_blocks"] >= (len(t) // block if block < len(t) else 1)
    _assert_table(got, pb, po, k)


@pytest.mark.gpu
def test_gpu_fastq_file_record_longer_than_block(tmp_path, monkeypatch):
    """A block that holds no complete record grows until one fits (reads of 1500 bases, 1 KB blocks)."""
    import mhm2_proxy_amd as m
    b, o = c.synth_set(40, 60000, 35, read_len=1500)
    t = c.fastq_text(b, o, seed=35)
    assert len(t) > 40 * 3000
    path = _write(tmp_path, "long.fq", t)
    pb, po = O.fastq_pack(t)
    monkeypatch.setenv("MHMKC_FQ_BLOCK", "1024")
    with m.KmerCounter(33, device=0) as cnt:
        cnt.add_fastq_file(path)
        cnt.finish()
        got = cnt.fetch().sorted()
    _assert_table(got, pb, po, 33)


@pytest.mark.gpu
@pytest.mark.parametrize("block", [7001, 1 << 28])
def test_gpu_fastq_pairs_file_equals_oracle(tmp_path, monkeypatch, block):
    """Interleaved pairs: blocks are cut at pair boundaries, the pair statistics sum over the blocks."""
    import mhm2_proxy_amd as m
    t = c.paired_fastq_text(3000, seed=36)
    path = _write(tmp_path, "pairs.fq", t)
    pb, po, pst = O.merge_fastq(t)
    monkeypatch.setenv("MHMKC_FQ_BLOCK", str(block))
    with m.KmerCounter(21, device=0) as cnt:
        cnt.add_fastq_file(path, pairs=True)
        st = cnt.stats()
        gb, go = cnt.fastq_packed()
        cnt.finish()
        got = cnt.fetch().sorted()
    for key in ("pairs", "merged", "ambiguous", "overlap_bases"):
        assert st["fq_" + key] == pst[key], key
    assert len(go) == len(po) and (go == po).all() and (gb == pb).all()
    _assert_table(got, pb, po, 21)


@pytest.mark.gpu
def test_gpu_fastq_file_errors(tmp_path, monkeypatch):
    import mhm2_proxy_amd as m
    monkeypatch.setenv("MHMKC_FQ_BLOCK", "3000")
    with m.KmerCounter(21, device=0) as cnt:
        with pytest.raises(m.MhmkcError) as e:
            cnt.add_fastq_file(tmp_path / "missing.fq")
        assert str(e.value).startswith("MHMKC_EINVAL")
    b, o = c.synth_set(200, 20000, 37)
    lines = c.fastq_text(b, o, seed=37).split(b"\n")[:-1]
    bad = list(lines)
    bad[4 * 150 + 1] = b"X" + bad[4 * 150 + 1][1:]  # an illegal base in record 150 (a later block)
    with m.KmerCounter(21, device=0) as cnt:
        with pytest.raises(m.MhmkcError) as e:
            cnt.add_fastq_file(_write(tmp_path, "bad.fq", b"\n".join(bad) + b"\n"))
        assert str(e.value).startswith("MHMKC_EBADCHAR"), str(e.value)
        # the message locates the failing block in the file, and the round that holds the earlier
        # blocks refuses to finish until reset
        assert re.search(r"FASTQ file block [1-9]\d*, whose text starts at file byte [1-9]\d*", str(e.value)), str(e.value)
        with pytest.raises(m.MhmkcError) as e2:
            cnt.finish()
        assert str(e2.value).startswith("MHMKC_ESTATE"), str(e2.value)
        cnt.reset()
        cnt.add_fastq_file(_write(tmp_path, "good.fq", b"\n".join(lines) + b"\n"))
        cnt.finish()
        from common import assert_tables_equal, oracle_table
        assert_tables_equal(cnt.fetch(), oracle_table(b, o, 21), "after reset")
    trunc =b"\n".join(lines[:-2]) + b"\n"  # the last record lacks its '+' and quality lines
    with m.KmerCounter(21, device=0) as cnt:
        with pytest.raises(m.MhmkcError) as e:
            cnt.add_fastq_file(_write(tmp_path, "trunc.fq", trunc))
        assert str(e.value).startswith("MHMKC_EINVAL") and re.search(r"ends inside record", str(e.value))


@pytest.mark.gpu
@pytest.mark.parametrize("fail_block", [1, 2])
def test_gpu_fastq_file_read_failure_after_first_block(tmp_path, monkeypatch, fail_block, knob):
    """the background read of a later block fails (a file that shrinks or turns unreadable mid-call,
    injected with the test knob fq_read_fail): the earlier blocks' reads are already in the round, so the call fails
    with MHMKC_EINVAL and finish refuses the round (MHMKC_ESTATE) until reset."""
    import mhm2_proxy_amd as m
    b, o = c.synth_set(400, 20000, 38)
    t = c.fastq_text(b, o, seed=38)
    path = _write(tmp_path, "reads.fq", t)
    monkeypatch.setenv("MHMKC_FQ_BLOCK", "5000")
    assert len(t) > 4 * 5000
    knob("fq_read_fail", fail_block)
    with m.KmerCounter(21, device=0) as cnt:
        with pytest.raises(m.MhmkcError) as e:
            cnt.add_fastq_file(path)
        assert str(e.value).startswith("MHMKC_EINVAL") and "read error" in str(e.value), str(e.value)
        with pytest.raises(m.MhmkcError) as e2:
            cnt.finish()
        assert str(e2.value).startswith("MHMKC_ESTATE"), str(e2.value)
        knob("fq_read_fail", -1)
        cnt.reset()
        cnt.add_fastq_file(path)
        cnt.finish()
        from common import assert_tables_equal, oracle_table
        assert_tables_equal(cnt.fetch(), oracle_table(b, o, 21), "after reset")
