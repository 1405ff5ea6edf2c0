"""FASTQ ingest: FASTQ text -> PackedRead bytes on the device (mhmkc_add_fastq).

The checker is oracle/kcount_oracle.c orc_fastq_pack, a restatement of FastqReader::get_next_fq_record
(src/fastq.cpp:504-551, rtrim :67-71, get_fq_name :73-122) and the PackedRead constructor
(src/packed_reads.cpp:73-109). It is cross-checked here against a second, literal string-level restatement
(`literal_pack`). The reference holds no FASTQ fixtures (its CI downloads arctic_sample_0.fq), so this row is
pinned by the two restatements and review against the cited lines, not by reference-generated vectors.
"""
from __future__ import annotations

import re

import numpy as np
import pytest

import common as c
import oracle_lib as O

K = 21


# --------------------------------------------------------------------------------------------------
# literal restatement (strings, as the reference code reads)

def _rtrim(s: str) -> str:  # fastq.cpp:67-71 (an all-whitespace line: UB there, "" here)
    return s.rstrip(" \t\n\v\f\r")


def _get_fq_name(header: str) -> bool:  # fastq.cpp:73-122, verdict only
    if not header or header[0] != "@":
        return False
    header = _rtrim(header[1:])
    n = len(header)
    if n >= 3 and header[n - 2] != "/":
        if header[n - 2] == "R":
            return True
        end_pos = header.find("\t")
        if end_pos < 0:
            end_pos = header.find(" ")
            if end_pos < 0:
                return True
        if end_pos > 3 and header[end_pos - 2] == "/" and header[end_pos - 1] in "12":
            return True
        if (n < end_pos + 7 or header[end_pos + 2] != ":" or header[end_pos + 4] != ":"
                or header[end_pos + 6] != ":" or header[end_pos + 1] not in "12"):
            return False
    return True


_CODE = {"A": 0, "C": 1, "G": 2, "T": 3, **{ch: 4 for ch in "NURYKMSWBDHV"}}  # packed_reads.cpp:87-105


def literal_pack(text: bytes, qual_offset: int = 33):
    lines = text.decode("latin-1").split("\n")
    if text.endswith(b"\n"):
        lines.pop()
    out, offs = [], [0]
    for r in range(0, len(lines) // 4 * 4, 4):
        ident, seq, plus, quals = lines[r:r + 4]
        ident, seq, quals = _rtrim(ident), _rtrim(seq), _rtrim(quals)
        if not ident or ident[0] != "@":
            raise O.FastqError("id", r // 4)
        if not plus or plus[0] != "+":
            raise O.FastqError("plus", r // 4)
        if not _get_fq_name(ident):
            raise O.FastqError("name", r // 4)
        if len(seq) != len(quals):
            raise O.FastqError("len", r // 4)
        for ch, q in zip(seq, quals):
            if ch not in _CODE:
                raise O.FastqError("char", r // 4)
            qv = min(ord(q) - qual_offset, 31)
            out.append((_CODE[ch] | ((qv & 0xFF) << 3)) & 0xFF)
        offs.append(len(out))
    if len(lines) % 4:
        raise O.FastqError("trunc", len(lines) // 4)
    return np.array(out, dtype=np.uint8), np.array(offs, dtype=np.uint64)


def _odd_quals(text: bytes, seed: int) -> bytes:
    """Replace every quality line by random printable quality characters ('!'..'~', incl. q - 33 > 31)."""
    rng = np.random.default_rng(seed)
    lines = text.split(b"\n")
    for i in range(3, len(lines), 4):
        body = lines[i].rstrip(b"\r")
        q = rng.integers(0x21, 0x7F, size=len(body)).astype(np.uint8).tobytes()
        lines[i] = q + lines[i][len(body):]
    return b"\n".join(lines)


VARIANTS = {
    "plain": dict(),
    "crlf_ws_iupac": dict(crlf_every=2, trailing_ws=True, iupac=True, seed=1),
    "no_final_newline": dict(final_newline=False, seed=2),
}

# malformed inputs: (mutation of record 3 of a small valid file, expected kind)
BAD = {
    "id": (lambda L: L.__setitem__(12, b"read3"), "id"),
    "plus": (lambda L: L.__setitem__(14, b"-"), "plus"),
    "name": (lambda L: L.__setitem__(12, b"@pair3 x:N:0:1"), "name"),
    "len": (lambda L: L.__setitem__(15, L[15][:-1]), "len"),
    "char": (lambda L: L.__setitem__(13, L[13][:40] + b"a" + L[13][41:]), "char"),
    "long": (lambda L: (L.__setitem__(13, b"A" * 2046), L.__setitem__(15, b"I" * 2046)), "long"),
    "trunc": (lambda L: L.__delitem__(slice(len(L) - 3, len(L))), "trunc"),
}


def _bad_text(name: str) -> bytes:
    b, o = c.synth_set(8, 5000, 4)
    lines = c.fastq_text(b, o, seed=4).split(b"\n")[:-1]
    BAD[name][0](lines)
    return b"\n".join(lines) + b"\n"


# --------------------------------------------------------------------------------------------------
# CPU: the oracle against the literal restatement and the round trip

@pytest.mark.parametrize("variant", sorted(VARIANTS))
def test_oracle_fastq_roundtrip(variant):
    b, o = c.synth_set(3000, 30000, 11)
    t = c.fastq_text(b, o, **VARIANTS[variant])
    pb, po = O.fastq_pack(t)
    assert (po == o).all() and (pb == b).all()
    lb, lo = literal_pack(t)
    assert (lo == o).all() and (lb == b).all()


@pytest.mark.parametrize("qoff", [33, 64])
def test_oracle_fastq_quality_range(qoff):
    b, o = c.synth_set(500, 10000, 12)
    t = _odd_quals(c.fastq_text(b, o, seed=5), 5)
    pb, po = O.fastq_pack(t, qoff)
    lb, lo = literal_pack(t, qoff)
    assert (po == lo).all() and (pb == lb).all()


@pytest.mark.parametrize("name", sorted(BAD))
def test_oracle_fastq_errors(name):
    t = _bad_text(name)
    with pytest.raises(O.FastqError) as e1:
        O.fastq_pack(t)
    want_rec = 7 if name == "trunc" else 3
    assert e1.value.kind == BAD[name][1] and e1.value.record == want_rec
    if name != "long":  # the literal restatement has no fgets buffer
        with pytest.raises(O.FastqError) as e2:
            literal_pack(t)
        assert (e2.value.kind, e2.value.record) == (e1.value.kind, e1.value.record)


def test_oracle_fastq_empty():
    pb, po = O.fastq_pack(b"")
    assert pb.size == 0 and list(po) == [0]


# --------------------------------------------------------------------------------------------------
# GPU: the device parser against the oracle, through the C ABI

ERR_CODE = {"id": "MHMKC_EINVAL", "plus": "MHMKC_EINVAL", "name": "MHMKC_EINVAL", "len": "MHMKC_EINVAL",
            "trunc": "MHMKC_EINVAL", "char": "MHMKC_EBADCHAR", "long": "MHMKC_EUNSUPPORTED"}


@pytest.mark.gpu
@pytest.mark.parametrize("variant", sorted(VARIANTS))
def test_gpu_fastq_pack_matches_oracle(variant):
    import mhm2_proxy_amd as m
    b, o = c.synth_set(20000, 200000, 21)
    t = c.fastq_text(b, o, **VARIANTS[variant])
    pb, po = O.fastq_pack(t)
    with m.KmerCounter(K, device=0) as cnt:
        cnt.add_fastq(t)
        gb, go = cnt.fastq_packed()
    assert (go == po).all() and (gb == pb).all()


@pytest.mark.gpu
@pytest.mark.parametrize("qoff", [33, 64])
def test_gpu_fastq_quality_range(qoff):
    import mhm2_proxy_amd as m
    b, o = c.synth_set(3000, 30000, 22)
    t = _odd_quals(c.fastq_text(b, o, seed=6, crlf_every=3), 6)
    pb, po = O.fastq_pack(t, qoff)
    with m.KmerCounter(K, device=0, qual_offset=qoff) as cnt:
        cnt.add_fastq(t)
        gb, go = cnt.fastq_packed()
    assert (go == po).all() and (gb == pb).all()


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(BAD))
def test_gpu_fastq_errors(name):
    import mhm2_proxy_amd as m
    t = _bad_text(name)
    with pytest.raises(O.FastqError) as want:
        O.fastq_pack(t)
    with m.KmerCounter(K, device=0) as cnt:
        with pytest.raises(m.MhmkcError) as got:
            cnt.add_fastq(t)
    msg = str(got.value)
    assert msg.startswith(ERR_CODE[name]), msg
    assert int(re.search(r"record (\d+)", msg).group(1)) == want.value.record, msg


@pytest.mark.gpu
def test_gpu_fastq_empty_and_tiny():
    import mhm2_proxy_amd as m
    with m.KmerCounter(K, device=0) as cnt:
        cnt.add_fastq(b"")
        gb, go = cnt.fastq_packed()
        assert gb.size == 0 and list(go) == [0]
        cnt.add_fastq(b"@r0\nACGTN\n+\nIIIII")  # one record, no final newline
        gb, go = cnt.fastq_packed()
        assert list(go) == [0, 5] and list(gb) == [0 | 31 << 3, 1 | 31 << 3, 2 | 31 << 3, 3 | 31 << 3, 4 | 31 << 3]


@pytest.mark.gpu
@pytest.mark.parametrize("k", [21, 63])
def test_gpu_fastq_count_matches_oracle(k):
    """End to end: FASTQ text -> device pack -> count, equal to the oracle's count of the oracle's pack."""
    import mhm2_proxy_amd as m
    b, o = c.synth_set(20000, 100000, 23)
    t = c.fastq_text(b, o, crlf_every=5, trailing_ws=True, iupac=True, seed=7)
    pb, po = O.fastq_pack(t)
    with m.KmerCounter(k, device=0) as cnt:
        cnt.add_fastq(t)
        cnt.finish()
        got = cnt.fetch().sorted()
    keys, counts, left, right = O.kcount(pb, po, k).fetch()
    assert (got.keys == keys).all() and (got.counts == counts).all()
    assert (got.left == left).all() and (got.right == right).all()


@pytest.mark.gpu
def test_gpu_fastq_device_text_large():
    """HBM-resident text (mhmkc_add_fastq_device), 400k reads: the round trip to the generator's bytes is
    the size-independent check; the occurrence count closes the loop."""
    import torch
    import mhm2_proxy_amd as m
    b, o = c.synth_set(400_000, 2_000_000, 24)
    t = c.fastq_text(b, o, seed=8)
    tt = torch.frombuffer(bytearray(t), dtype=torch.uint8).to("cuda:0")
    with m.KmerCounter(K, device=0) as cnt:
        cnt.add_fastq_tensor(tt)
        gb, go = cnt.fastq_packed()
        cnt.finish()
        st = cnt.stats()
    assert (go == o).all() and (gb == b).all()
    assert st["occurrences"] == st["count_sum"] == 400_000 * (150 - K - 1)


@pytest.mark.gpu
def test_gpu_fastq_ragged_reads():
    """Reads of every length 0..150 (empty records are undefined behaviour in the reference's rtrim; both
    sides read them as empty), all-N and low-quality reads: every output misalignment and partial dword of
    k_fq_pack, against the oracle, then counted."""
    import mhm2_proxy_amd as m
    b, o = c.edge_case_set(seed=31, n=3000)
    t = c.fastq_text(b, o, seed=3, crlf_every=7, iupac=True)
    pb, po = O.fastq_pack(t)
    assert (po == o).all() and (pb == b).all()
    with m.KmerCounter(K, device=0) as cnt:
        cnt.add_fastq(t)
        gb, go = cnt.fastq_packed()
        cnt.finish()
        got = cnt.fetch().sorted()
    assert (go == po).all() and (gb == pb).all()
    keys, counts, left, right = O.kcount(pb, po, K).fetch()
    assert (got.keys == keys).all() and (got.counts == counts).all()
    assert (got.left == left).all() and (got.right == right).all()


def test_oracle_fastq_ragged_reads():
    b, o = c.edge_case_set(seed=31, n=600)
    t = c.fastq_text(b, o, seed=3, crlf_every=7, iupac=True)
    pb, po = O.fastq_pack(t)
    lb, lo = literal_pack(t)
    assert (po == o).all() and (pb == b).all() and (lo == o).all() and (lb == b).all()
