"""The reference-shaped C++ adapter (include/mhmkc_kcount.hpp) over the C ABI."""
import gzip
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
SRC = ROOT / "tests" / "cpp" / "adapter_test.cpp"
GOLDEN = ROOT / "tests" / "golden"


def build(tmp: Path) -> Path:
    if not shutil.which("g++"):
        pytest.skip("g++ missing")
    exe = tmp / "adapter_test"
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", f"-I{ROOT / 'include'}", str(SRC),
                    f"-L{ROOT / 'mhm2_proxy_amd'}", "-lmhmkc", "-lz", f"-Wl,-rpath,{ROOT / 'mhm2_proxy_amd'}",
                    "-o", str(exe)], check=True)
    return exe


def test_adapter_compiles_and_kmer_kats(tmp_path):
    from mhm2_proxy_amd import build as b

    b.build_lib()
    exe = build(tmp_path)
    out = subprocess.run([str(exe), "kat"], capture_output=True, text=True, env={"MHMKC_NO_TORCH": "1"})
    assert out.stdout.strip() == "KAT OK", out.stdout + out.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("mode,k,setname", [("reads", 21, "s100"), ("reads", 63, "s100"), ("seqs", 33, "s100"),
                                            ("reads", 21, "edge"), ("seqs", 21, "edge")])
def test_adapter_matches_golden(mode, k, setname, tmp_path):
    exe = build(tmp_path)
    reads = tmp_path / "reads.txt"
    reads.write_text(gzip.open(GOLDEN / f"reads_{setname}.txt.gz", "rt").read())
    out = subprocess.run([str(exe), mode, str(k), str(reads)], capture_output=True, text=True, check=True,
                         cwd=tmp_path)
    got = out.stdout.splitlines()
    exp = sorted(gzip.open(GOLDEN / f"table_{setname}_k{k}.tsv.gz", "rt").read().splitlines())
    assert got == exp
    if mode == "reads":  # analyze_kmers(..., dump_kmers = true): the reference's per-rank gzip file
        dump = tmp_path / "per_rank" / "00000000" / "00000000" / f"kmers-{k}.txt.gz"
        assert sorted(gzip.open(dump, "rt").read().splitlines()) == exp


@pytest.mark.gpu
@pytest.mark.parametrize("k", [21, 63])
def test_adapter_dmin_from_analyze_kmers(k, tmp_path):
    """KmerDHT built the reference's way (contigging.cpp:115-116, before dmin is known), then
    analyze_kmers(..., dmin_thres = 3, ...): the finish uses 3 (_dmin_thres, kcount.cpp:145), as the oracle."""
    import sys

    sys.path.insert(0, str(ROOT / "tests"))
    import mhm2_proxy_amd as m
    from common import oracle_table, synth_set

    exe = build(tmp_path)
    b, o = synth_set(1500, 8000, 70 + k)
    pr = m.PackedReads.from_arrays(b, o)
    reads = tmp_path / "reads.txt"
    with open(reads, "w") as f:
        for i in range(pr.get_local_num_reads()):
            _, s_, q = pr.get_read(i)
            f.write(f"{s_} {q}\n")
    out = subprocess.run([str(exe), "reads", str(k), str(reads), "-", "3"], capture_output=True, text=True,
                         check=True, cwd=tmp_path)
    exp3 = sorted(oracle_table(b, o, k, dmin_thres=3).lines())
    assert out.stdout.splitlines() == exp3
    assert exp3 != sorted(oracle_table(b, o, k, dmin_thres=2).lines())  # the threshold matters here


@pytest.mark.gpu
@pytest.mark.parametrize("k", [21, 63])
def test_adapter_contig_pass(k, tmp_path):
    """analyze_kmers with a Contigs list through the C++ adapter equals the oracle's contig pass."""
    import sys

    sys.path.insert(0, str(ROOT / "tests"))
    import mhm2_proxy_amd as m
    from common import ctg_set, oracle_ctg_table

    exe = build(tmp_path)
    b, o, seqs, depths = ctg_set(seed=120 + k)
    pr = m.PackedReads.from_arrays(b, o)
    reads = tmp_path / "reads.txt"
    with open(reads, "w") as f:
        for i in range(pr.get_local_num_reads()):
            _, s_, q = pr.get_read(i)
            f.write(f"{s_} {q}\n")
    ctgs = tmp_path / "ctgs.txt"
    ctgs.write_text("".join(f"{s_} {int(d)}.25\n" for s_, d in zip(seqs, depths)))
    out = subprocess.run([str(exe), "ctgs", str(k), str(reads), str(ctgs)], capture_output=True, text=True, check=True)
    exp = sorted(oracle_ctg_table(b, o, seqs, depths, k).lines())
    assert out.stdout.splitlines() == exp


@pytest.mark.gpu
@pytest.mark.parametrize("k", [21, 63])
def test_adapter_fastq(k, tmp_path):
    """KmerDHT::add_fastq (FASTQ text -> device parse + pack -> count) equals the oracle's count of the oracle's
    pack of the same text."""
    import sys

    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib as O
    from common import fastq_text, oracle_table, synth_set

    exe = build(tmp_path)
    b, o = synth_set(3000, 30000, 130 + k)
    text = fastq_text(b, o, crlf_every=4, trailing_ws=True, iupac=True, seed=k)
    fq = tmp_path / "reads.fq"
    fq.write_bytes(text)
    out = subprocess.run([str(exe), "fastq", str(k), str(fq)], capture_output=True, text=True, check=True)
    assert "fastq reads 3000" in out.stderr
    pb, po = O.fastq_pack(text)
    assert out.stdout.splitlines() == sorted(oracle_table(pb, po, k).lines())


@pytest.mark.parametrize("k,n,chunks,dups", [(21, 400_000, 1, 0), (21, 400_000, 7, 300), (33, 200_000, 3, 50),
                                             (63, 150_000, 1, 20), (99, 100_000, 5, 10), (21, 3000, 2, 5)])
def test_kmermap_parallel_fill(k, n, chunks, dups, tmp_path):
    """KmerMap::fill's threaded placement of rows in mhmkc_fetch_ordered's order (include/mhmkc_kcount.hpp
    chunk_ordered: positions as a running maximum over thread ranges, rows past the last slot wrapped through put), in
    one piece and streamed in chunks as load_ordered feeds it, holds every row with its values, exactly like the
    one-thread insert loop; repeated keys (also across chunk boundaries) keep their first row; unordered rows fall
    back to the loop. --slots: the rows' slots and tags computed as the device computes them for mhmkc_fetch_map_range
    (a prefix maximum of home slot minus row index), placed by KmerMap::fill_chunk_slots, rows past the last slot
    through put."""
    import numpy as np

    from mhm2_proxy_amd import build as b

    tool = b.build_fill()
    rng = np.random.default_rng(k + n + chunks)
    nl = k // 32 + 1
    keys = rng.integers(0, 2 ** 63, size=(n, nl), dtype=np.uint64)
    kk = min(k, 32)
    keys[:, 0] &= np.uint64(((1 << (2 * kk)) - 1) << (64 - 2 * kk))
    if dups:
        keys[n - dups:] = keys[rng.integers(0, n - dups, size=dups)]
    pre = str(tmp_path / "t")
    keys.tofile(pre + ".keys")
    rng.integers(0, 65535, size=n, dtype=np.uint16).tofile(pre + ".counts")
    rng.integers(65, 90, size=n, dtype=np.uint8).tofile(pre + ".left")
    rng.integers(65, 90, size=n, dtype=np.uint8).tofile(pre + ".right")
    for extra in (["4", "--sort", "--chunks", str(chunks)], ["4", "--chunks", str(chunks)],
                  ["4", "--slots", "--chunks", str(chunks)]):
        r = subprocess.run([str(tool), str(k), str(n), pre, *extra], capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr
        import json

        j = json.loads(r.stdout.strip().splitlines()[-1])
        assert j["bad"] == 0 and j["size"] == j["size_one_thread"] == len({tuple(x) for x in keys.tolist()})
