"""Host-side logic without a GPU: PackedReads mirror, k-mer helpers, synthetic generator, dump format."""
from __future__ import annotations

import gzip

import numpy as np
import pytest

import mhm2_proxy_amd as m
import oracle_lib as O
from common import synth_set


def test_packed_read_encoding_matches_reference_ctor():
    # src/packed_reads.cpp:73-109: ACGTN -> 0..4, IUPAC -> 4, quality min(q - off, 31) << 3
    b = m.PackedReads.pack("ACGTNRYK", "!+5?I~II")
    assert list(b & 7) == [0, 1, 2, 3, 4, 4, 4, 4]
    assert list(b >> 3) == [0, 10, 20, 30, 31, 31, 31, 31]
    with pytest.raises(ValueError):
        m.PackedReads.pack("ACGX", "IIII")


def test_packed_reads_roundtrip():
    pr = m.PackedReads(33)
    pr.add_read("@r1/1", "ACGTN", "II#+I")
    pr.add_read("@r2/1", "TTT", "III")
    assert pr.get_local_num_reads() == 2 and pr.get_bases() == 8
    _, seq, quals = pr.get_read(0)
    assert seq == "ACGTN" and quals == "@@#+@"  # qualities are capped at Q31 ('@') as the reference stores them
    assert list(pr.offsets) == [0, 5, 8]


def test_kmer_helpers_match_oracle():
    rng = np.random.default_rng(1)
    for k in (5, 21, 33, 63, 99):
        nl = m.n_longs_for(k)
        for _ in range(20):
            s = "".join(rng.choice(list("ACGT"), size=k))
            longs = m.kmer_from_string(s, nl)
            assert list(longs) == [int(x) for x in O.kmer_from_string(s, nl)]
            assert m.kmer_to_string(longs, k) == s
            assert m.keys_to_strings(np.array([longs], dtype=np.uint64), k) == [s]


def test_target_rank_matches_oracle():
    rng = np.random.default_rng(2)
    for k in (21, 33, 55):
        nl = m.n_longs_for(k)
        for _ in range(30):
            s = "".join(rng.choice(list("ACGT"), size=k))
            longs = m.kmer_from_string(s, nl)
            for n in (1, 3, 8):
                assert m.get_kmer_target_rank(longs, k, n) == O.target_rank(np.array(longs, np.uint64), k, n)


def test_synth_deterministic_and_shardable():
    g = m.synth_genome(20000, 3)
    b1, o1 = m.synth_reads(g, 1000, 150, 3, threads=1)
    b4, o4 = m.synth_reads(g, 1000, 150, 3, threads=4)
    assert (b1 == b4).all() and (o1 == o4).all()
    bs, _ = m.synth_reads(g, 300, 150, 3, first_read=500)
    assert (bs == b1[500 * 150:800 * 150]).all()


def test_synth_rates():
    b, _ = synth_set(20000, 100000, 4)
    codes, q = b & 7, b >> 3
    assert abs((codes == 4).mean() - 0.0002) < 0.0001
    assert abs((q == 10).mean() - 0.02) < 0.003
    assert abs((q == 2).mean() - 0.0025) < 0.0008
    assert set(np.unique(q)) <= {2, 10, 31}


def test_table_lines_dump_format(tmp_path):
    t = m.KmerTable(5, np.array([m.kmer_from_string("ACGTA", 1)], dtype=np.uint64), np.array([7], np.uint16),
                    np.array([ord("A")], np.uint8), np.array([ord("F")], np.uint8))
    assert list(t.lines()) == ["ACGTA 7 A F"]
    p = tmp_path / "x.gz"
    with gzip.open(p, "wt") as f:
        f.write("\n".join(t.lines()) + "\n")
    assert gzip.open(p, "rt").read() == "ACGTA 7 A F\n"


def test_mixed_record_bijection_and_flatness(tmp_path):
    """kmer_ops.hpp cmix / m2_mix / mx_mix and their inverses (mixed records): round
    trips at every k in 10..21, 33..63 and 65..127 (k % 32 != 0),
    and flat bucket digits and home groups over the consecutive (correlated) canonical windows of one sequence."""
    import shutil
    import subprocess
    from pathlib import Path

    if not shutil.which("g++"):
        pytest.skip("g++ missing")
    src = Path(__file__).parent / "cpp" / "mix_check.cpp"
    exe = tmp_path / "mix_check"
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wno-unknown-pragmas", str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), "2000000"], capture_output=True, text=True, check=True).stdout
    assert "roundtrip ok" in out
    rows = [ln.split() for ln in out.splitlines() if ln.startswith("k ")]
    assert len(rows) == 11
    for r in rows:
        coarse, fine, group = float(r[3]), float(r[5]), float(r[7])
        # 256 coarse bins of ~7800 windows, up to 2^17 fine bins of ~15 (Poisson max), 1000 groups of 2000
        assert coarse < 1.08 and group < 1.12 and fine < 3.0, r


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_nibble_packing(mode):
    """The nibble H2D's host packing (mhmkc_host.cpp nib_pack) against a numpy restatement: every
    byte value, odd lengths and unaligned starts, cutoffs across [0, 32]; two nibbles per byte, the first low."""
    import ctypes as C

    from mhm2_proxy_amd import _native as N

    rng = np.random.default_rng(mode + 11)
    for n, off, qcut in [(0, 0, 20), (1, 0, 20), (7, 3, 0), (63, 0, 1), (64, 0, 31), (65, 5, 32), (1000, 32, 20),
                         (4099, 1, 19), (100_000, 0, 20), (100_001, 17, 7)]:
        buf = np.zeros(n + 64, np.uint8)
        src = buf[off:off + n]
        src[:] = rng.integers(0, 256, n, dtype=np.uint8)
        if n >= 256:
            src[:256] = np.arange(256, dtype=np.uint8)
        out = np.full((n + 1) // 2 + 64, 0xAB, np.uint8)
        rc = N.lib().mhmkc_debug_nib_pack(src.ctypes.data, n, out.ctypes.data, qcut, mode)
        if rc == -7 and mode == 2:  # MHMKC_EUNSUPPORTED: no AVX2 on this CPU
            pytest.skip("no AVX2")
        assert rc == 0
        nib = (src & 7) | np.where((src >> 3) >= min(max(qcut, 0), 32), 8, 0).astype(np.uint8)
        if n & 1:
            nib = np.concatenate([nib, np.zeros(1, np.uint8)])
        exp = (nib[0::2] | (nib[1::2] << 4)).astype(np.uint8)
        assert np.array_equal(out[:(n + 1) // 2], exp), (n, off, qcut)
        assert (out[(n + 1) // 2:] == 0xAB).all()  # nothing written past the packed bytes
