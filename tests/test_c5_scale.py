"""a C5-shaped scale check of the multi-k chain (src/contigging.cpp:93-158 drives, per k, the count
with the previous round's contigs, src/kcount/kcount.cpp:100-138, then the traversal). C5 itself (arcticsynth, 8 x
MI355X) is not available offline; this is its shape on the one test GPU:

  * a synthetic paired set of 1M pairs (tests/common.py paired_fastq_bulk: 150-base mates of 150-360-base fragments
    of a 5 Mbp genome, substitutions, N, low-quality bases) merged on the device (mhmkc_add_fastq_pairs), the merged
    PackedReads checked byte for byte against oracle/merge_reads.c;
  * k = 21, 33, 55, 77, 99 at 4 ranks on the one GPU over libmhmkc's RCCL path (the driver's 8-GPU code path) and
    at 8 ranks over the host transport, with MHMKC_OWNER_MINIMIZER (the record exchange + owner hand-off at k = 21,
    supermers from k = 33); each rank has its shard of the merged reads and its block of the previous round's
    contigs (the contig all-gather and the contig pass at every k after the first);
  * each round's contigs: the restated traversal (include/mhmkc_dbjg.hpp) over the union of the ranks' tables.

Every round's union equals the multi-threaded CPU restatement with the contig pass (oracle/kcount_mt.c
orc_kcount_mt_ctgs_range, pinned to the single-threaded oracle by tests/test_oracle.py) row for row, as sorted 64-bit
row fingerprints, and every row is on its get_kmer_target_rank. Parity unpinned beyond the restatements: the
reference's kcount and traversal need UPC++.
"""
import numpy as np
import pytest

import common as c
import oracle_lib as O


@pytest.mark.gpu
@pytest.mark.slow
@pytest.mark.timeout(1100)
@pytest.mark.parametrize("world,rccl", [(4, True), (8, False)])
def test_c5_shaped_multik_chain(world, rccl, tmp_path):
    import torch.multiprocessing as mp

    import mhm2_proxy_amd as m
    import mr_gpu_worker
    from test_multirank_gpu import free_port

    pairs, genome, ks = 1_000_000, 5_000_000, [21, 33, 55, 77, 99]
    text = c.paired_fastq_bulk(pairs, 55, genome)
    with m.KmerCounter(21, device=0) as cnt:
        cnt.add_fastq_pairs(text)
        gb, go = cnt.fastq_packed()
        st = cnt.stats()
    pb, po, pst = O.merge_fastq(text, 33)
    del text
    assert go.size == po.size and (go == po).all() and (gb == pb).all(), "device merge != oracle/merge_reads.c"
    for key in ("pairs", "merged", "ambiguous", "overlap_bases"):
        assert st["fq_" + key] == pst[key], key
    assert pst["pairs"] == pairs and pst["merged"] > pairs // 2
    del pb, po
    np.savez(tmp_path / "merged.npz", bytes=gb, offs=go)
    print(f"merged {pst['merged']} of {pairs} pairs: {go.size - 1} reads, {gb.size} bases", flush=True)

    mp.spawn(mr_gpu_worker.run_c5, args=(world, free_port(), 0, str(tmp_path),
                                         {"ks": ks, "owner": "minimizer", "rccl": rccl}), nprocs=world, join=True)

    for i, k in enumerate(ks):
        parts = [np.load(tmp_path / f"k{k}_rank{r}.npz") for r in range(world)]
        for r, p in enumerate(parts):
            assert (O.target_ranks(p["keys"], k, world) == r).all(), f"k={k}: rank {r} holds rows of other ranks"
        got = np.sort(np.concatenate([O.row_fingerprints(p["keys"], p["counts"], p["left"], p["right"], k)
                                      for p in parts]))
        if i:
            seqs, depths = mr_gpu_worker.read_ctgs(tmp_path / f"ctgs_k{k}.txt")
            assert sum(int(p["ctg_kmers"]) for p in parts) > 0, f"k={k}: the contig pass saw no k-mers"
        else:
            seqs, depths = [], np.zeros(0, np.uint16)
        blob = "".join(seqs).encode("ascii")
        co = np.zeros(len(seqs) + 1, dtype=np.uint64)
        np.cumsum([len(s) for s in seqs], out=co[1:])
        exp = O.kcount_mt_ctgs(gb, go, blob, co, depths, k, threads=16).fetch()
        ef = np.sort(O.row_fingerprints(*exp, k))
        print(f"k={k}: {got.size} rows over {world} ranks, CPU restatement {ef.size}; {len(seqs)} contigs "
              f"({co[-1]} bases) fed in", flush=True)
        assert got.size == ef.size and np.array_equal(got, ef), f"k={k}: the union differs from the CPU restatement"
