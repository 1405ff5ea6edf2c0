"""The count table's consumer and multi-k end to end:
include/mhmkc_dbjg.hpp restates traverse_debruijn_graph at one rank (src/dbjg_traversal.cpp:569-596) over the
KmerMap that the C++ adapter fills; tests/cpp/dbjg_test.cpp runs contigging rounds k1, k2, ... (count with the
previous round's contigs, traverse, hand the contigs on; src/contigging.cpp:93-158).

Parity unpinned: the reference's traversal needs UPC++, so the contig sets are compared between the GPU counts
and the CPU oracle's counts through the same restated traversal, not against reference output.
"""
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

import mhm2_proxy_amd as m
import oracle_lib as O
from common import synth_set

ROOT = Path(__file__).resolve().parents[1]


def build(tmp: Path) -> Path:
    if not shutil.which("g++"):
        pytest.skip("g++ missing")
    from mhm2_proxy_amd import build as b

    b.build_lib()
    b.build_oracle()
    exe = tmp / "dbjg_test"
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", f"-I{ROOT / 'include'}", str(ROOT / "tests/cpp/dbjg_test.cpp"),
                    f"-L{ROOT / 'mhm2_proxy_amd'}", "-lmhmkc", f"-L{ROOT / 'oracle'}", "-loracle", "-lz",
                    f"-Wl,-rpath,{ROOT / 'mhm2_proxy_amd'}", f"-Wl,-rpath,{ROOT / 'oracle'}", "-o", str(exe)],
                   check=True)
    return exe


def reads_file(tmp: Path, b, o) -> Path:
    pr = m.PackedReads.from_arrays(b, o)
    path = tmp / "reads.txt"
    with open(path, "w") as f:
        for i in range(pr.get_local_num_reads()):
            _, s, q = pr.get_read(i)
            f.write(f"{s} {q}\n")
    return path


def rounds(text: str) -> dict:
    out, k = {}, None
    for line in text.splitlines():
        parts = line.split()
        if parts[0] == "K":
            k = int(parts[1])
            out[k] = []
        else:
            out[k].append((parts[0], float(parts[1])))
    return out


def revcomp(s: str) -> str:
    return s[::-1].translate(str.maketrans("ACGT", "TGCA"))


def test_traversal_walks_the_unique_chains(tmp_path):
    """CPU: the restated traversal over the oracle's table emits every k-mer with unique extensions on both
    sides exactly once, in chains that follow those extensions."""
    exe = build(tmp_path)
    b, o = synth_set(3000, 20000, 5)
    out = subprocess.run([str(exe), "oracle", str(reads_file(tmp_path, b, o)), "21"], capture_output=True, text=True,
                         check=True, env={"MHMKC_NO_TORCH": "1"}).stdout
    ctgs = rounds(out)[21]
    keys, counts, left, right = O.kcount(b, o, 21).fetch()
    strs = m.keys_to_strings(keys, 21)
    table = {s_: (chr(l_), chr(r_)) for s_, l_, r_ in zip(strs, left, right)}
    uu = {s_ for s_, (l_, r_) in table.items() if l_ in "ACGT" and r_ in "ACGT"}
    seen = set()
    for seq, depth in ctgs:
        assert len(seq) >= 21 and depth > 0
        for i in range(len(seq) - 20):
            km = seq[i:i + 21]
            c = min(km, revcomp(km))
            assert c in uu, "a contig k-mer must be UU"
            assert c not in seen, "a k-mer in two contigs"
            seen.add(c)
    assert seen == uu or len(uu - seen) < 0.01 * len(uu)  # only cycles' and conflicts' k-mers may be left out
    assert max(len(s_) for s_, _ in ctgs) > 3000


@pytest.mark.gpu
@pytest.mark.parametrize("ks,seed,n_reads,genome", [("21,33,55", 5, 3000, 20000), ("21,33,55,77,99", 9, 6000, 40000),
                                                    ("33,63", 13, 4000, 30000)])
def test_multik_gpu_equals_oracle(tmp_path, ks, seed, n_reads, genome):
    """Multi-k contigging: every round's contig set from GPU counts (with the contig pass fed by the previous
    round's contigs) equals the one from the oracle's counts; the contig pass is exercised from round 2 on."""
    exe = build(tmp_path)
    b, o = synth_set(n_reads, genome, seed)
    rf = reads_file(tmp_path, b, o)
    gpu = subprocess.run([str(exe), "gpu", str(rf), ks], capture_output=True, text=True, check=True).stdout
    ora = subprocess.run([str(exe), "oracle", str(rf), ks], capture_output=True, text=True, check=True,
                         env={"MHMKC_NO_TORCH": "1"}).stdout
    rg, ro = rounds(gpu), rounds(ora)
    assert list(rg) == [int(x) for x in ks.split(",")]
    for k in rg:
        assert rg[k] == ro[k], f"k={k}: {len(rg[k])} vs {len(ro[k])} contigs"
        assert len(rg[k]) > 0
