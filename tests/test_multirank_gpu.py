"""libmhmkc's own multi-rank path on one GPU: 2-3 ranks, each a process with its own
counter, exchanging through the host-staged transport over gloo. The union of the owners' tables equals the
oracle's single-rank table of all reads; the owners' key sets are disjoint; bytes sent == bytes received; with
MHMKC_OWNER_MINIMIZER every k-mer ends on KmerDHT::get_kmer_target_rank (src/kcount/kmer_dht.cpp:193-196).
"""
import socket

import numpy as np
import pytest

import mhm2_proxy_amd as m
import oracle_lib as O
from common import assert_tables_equal, ctg_set, oracle_ctg_table, oracle_table, synth_set

pytestmark = pytest.mark.gpu


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_ranks(k, world, tmp_path, **opts):
    import torch.multiprocessing as mp

    import mr_gpu_worker

    mp.spawn(mr_gpu_worker.run, args=(world, free_port(), k, str(tmp_path), opts), nprocs=world, join=True)
    return [dict(np.load(tmp_path / f"rank{r}.npz")) for r in range(world)]


def union(parts, k):
    return m.KmerTable(k, np.concatenate([p["keys"] for p in parts]), np.concatenate([p["counts"] for p in parts]),
                       np.concatenate([p["left"] for p in parts]), np.concatenate([p["right"] for p in parts]))


def check_parts(parts, k, exp, what):
    u = union(parts, k)
    assert_tables_equal(u, exp, what)
    keys = u.keys
    assert len({tuple(r) for r in keys.tolist()}) == len(keys), "owners' key sets overlap"
    assert sum(int(p["bytes_sent"]) for p in parts) == sum(int(p["bytes_recv"]) for p in parts)
    assert sum(int(p["owned"]) for p in parts) == sum(int(p["occurrences"]) for p in parts)
    assert sum(int(p["count_sum"]) for p in parts) == sum(int(p["owned"]) for p in parts) or \
        sum(int(p["ctg_kmers"]) for p in parts) > 0
    if len(parts) > 1:
        assert sum(int(p["bytes_sent"]) for p in parts) > 0


@pytest.mark.parametrize("k,world,seed", [(21, 2, 621), (33, 3, 633), (63, 2, 663), (99, 2, 699)])
def test_ranks_equal_single_rank(k, world, seed, tmp_path):
    parts = run_ranks(k, world, tmp_path, seed=seed)
    b, o = synth_set(1200, 9000, seed)
    check_parts(parts, k, oracle_table(b, o, k), f"union of {world} ranks, k={k}")


@pytest.mark.parametrize("k,world,seed", [(21, 3, 721), (33, 2, 733), (55, 3, 755), (63, 2, 763), (63, 3, 764),
                                          (77, 2, 777), (99, 3, 799)])
def test_minimizer_owner_handoff(k, world, seed, tmp_path):
    """MHMKC_OWNER_MINIMIZER: after finish every k-mer is on its get_kmer_target_rank, as dbjg expects (every
    row checked against the oracle's target rank; m = 15/23/27 and one to four key words)."""
    parts = run_ranks(k, world, tmp_path, seed=seed, minimizer=True)
    b, o = synth_set(1200, 9000, seed)
    check_parts(parts, k, oracle_table(b, o, k), f"minimizer owners, k={k}")
    nl = k // 32 + 1
    L = O.oracle()
    mlen = L.orc_minimizer_len(k)
    for r, p in enumerate(parts):
        keys = np.ascontiguousarray(p["keys"][:, :nl], dtype=np.uint64)
        owner = np.fromiter((L.orc_kmer_target_rank(keys[i].ctypes.data, k, nl, world) for i in range(len(keys))),
                            dtype=np.int64, count=len(keys))
        assert (owner == r).all(), f"rank {r}: {(owner != r).sum()} rows not on their target rank (m={mlen})"
    assert sum(int(p["handoff_sent"]) for p in parts) == sum(int(p["handoff_recv"]) for p in parts) > 0


@pytest.mark.parametrize("k,world", [(21, 2), (33, 3), (63, 2)])
def test_multirank_contig_pass(k, world, tmp_path):
    """Contigs split over the ranks: applied in rank order everywhere, the union equals a single rank given all
    reads and the concatenated contigs (kcount.cpp:100-138, kcount_cpu.cpp:356-406)."""
    seed = 800 + k
    parts = run_ranks(k, world, tmp_path, seed=seed, contigs=True)
    b, o, seqs, depths = ctg_set(seed=seed)
    assert sum(int(p["ctg_kmers"]) for p in parts) > 0
    check_parts(parts, k, oracle_ctg_table(b, o, seqs, depths, k), f"contigs over {world} ranks, k={k}")


def test_multirank_dmin_and_many_chunks(tmp_path):
    """Two ranks, each host batch cut into ~45 H2D chunks (slice views with a head offset), dmin_thres = 3."""
    parts = run_ranks(21, 2, tmp_path, seed=9, dmin=3, n_reads=1200, genome=20000,
                      env={"MHMKC_CHUNK_BYTES": "1000"})
    b, o = synth_set(1200, 20000, 9)
    check_parts(parts, 21, oracle_table(b, o, 21, dmin_thres=3), "2 ranks, dmin 3, many H2D chunks")
