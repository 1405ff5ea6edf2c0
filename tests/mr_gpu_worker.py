"""Worker of the multi-rank GPU tests (TEST INFRASTRUCTURE): one rank of libmhmkc's own multi-GPU path.

Every rank is a process with its own counter on the same GPU. The exchange goes through the host-staged transport
(mhmkc_set_transport, driven by a gloo process group), or with opts["rccl"] through libmhmkc's RCCL path (each rank
with its own NCCL_HOSTID: RCCL refuses two ranks of one communicator on one device otherwise). The rank counts its
shard of the reads (and adds its share of the contigs); mhmkc_finish then runs the real exchange code (exchange(),
the contig all-gather and, with MHMKC_OWNER_MINIMIZER, the owner hand-off or the supermer exchange).
"""
import os
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
sys.path.insert(0, str(HERE.parent))


def shard(n: int, rank: int, world: int):
    return n * rank // world, n * (rank + 1) // world


def rccl_same_gpu_env(rank: int):
    """RCCL refuses two ranks of one communicator on one GPU ("Duplicate GPU detected"), unless the ranks look like
    different hosts: a per-rank NCCL_HOSTID, the socket network transport over loopback, no InfiniBand."""
    os.environ.update(NCCL_HOSTID=f"mhmkc-rehearsal-{rank}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1",
                      NCCL_NET="Socket")


def run(rank: int, world: int, port: int, k: int, out_dir: str, opts: dict):
    import torch
    import torch.distributed as dist

    import mhm2_proxy_amd as m
    from common import ctg_set, synth_set

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from conftest import apply_env

    apply_env(opts.get("env", {}))
    apply_env(opts.get("env_by_rank", {}).get(rank, {}))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    if opts.get("contigs"):
        b, o, seqs, depths = ctg_set(seed=opts["seed"], n_reads=opts.get("n_reads", 300))
    elif opts.get("hot"):  # common.hot_set: random reads first, then the poly-A reads
        from common import hot_set

        b, o = hot_set(**opts.get("hot_args", {}))
        seqs, depths = [], np.zeros(0, np.uint16)
    else:
        b, o = synth_set(opts.get("n_reads", 1200), opts.get("genome", 9000), opts["seed"])
        seqs, depths = [], np.zeros(0, np.uint16)
    if "ctg_seqs" in opts:
        seqs, depths = opts["ctg_seqs"], opts["ctg_depths"]
    n = o.size - 1
    lo, hi = shard(n, rank, world)
    if opts.get("cuts"):  # explicit read ranges: rank r takes [cuts[r], cuts[r + 1])
        lo, hi = opts["cuts"][rank], opts["cuts"][rank + 1]
    idle = opts.get("idle_rank")  # this rank adds nothing; its share goes to the next rank (idle < world - 1)
    if idle is not None and rank == idle:
        lo = hi
    elif idle is not None and rank == idle + 1:
        lo = shard(n, idle, world)[0]
    owner = m.MHMKC_OWNER_MINIMIZER if opts.get("minimizer") else m.MHMKC_OWNER_HASH
    if opts.get("rccl"):
        # libmhmkc's RCCL path (ncclCommInitRank, ncclAllGather, grouped ncclSend/ncclRecv) with the ranks on one GPU:
        # each rank gets its own NCCL_HOSTID, so RCCL sees one GPU per "host" (no duplicate-GPU refusal) and moves
        # the data over its socket transport on loopback
        rccl_same_gpu_env(rank)
        obj = [m.comm_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        c = m.KmerCounter(k, device=0, rank=rank, n_ranks=world, comm_id=obj[0], output_owner=owner,
                          dmin_thres=opts.get("dmin", 2))
    else:
        c = m.KmerCounter(k, device=0, rank=rank, n_ranks=world, transport=m.TorchDistTransport(), output_owner=owner,
                          dmin_thres=opts.get("dmin", 2))
    # two batches per rank: the first from host memory (chunked H2D), the second from device tensors
    mid = (lo + hi) // 2
    c.add_packed_reads(b[int(o[lo]):int(o[mid])], (o[lo:mid + 1] - o[lo]).astype(np.uint64))
    bt = torch.from_numpy(b[int(o[mid]):int(o[hi])].copy()).cuda()
    ot = torch.from_numpy((o[mid:hi + 1] - o[mid]).astype(np.int64)).cuda()
    c.add_tensors(bt, ot)
    if len(seqs):
        a, z = shard(len(seqs), rank, world)
        if opts.get("ctg_rank") is not None:  # all contigs on one rank
            a, z = (0, len(seqs)) if rank == opts["ctg_rank"] else (0, 0)
        c.add_ctgs(seqs[a:z], depths[a:z])
    c.finish()
    t = c.fetch()
    st = c.stats()
    np.savez(Path(out_dir) / f"rank{rank}.npz", keys=t.keys, counts=t.counts, left=t.left, right=t.right,
             bytes_sent=st["bytes_sent"], bytes_recv=st["bytes_recv"], occurrences=st["occurrences"],
             owned=st["owned_records"], count_sum=st["count_sum"], distinct=st["distinct"], purged=st["purged"],
             n_out=st["n_out"], handoff_sent=st["handoff_sent"], handoff_recv=st["handoff_recv"],
             ctg_kmers=st["ctg_kmers"], smer_count=st["smer_count"], smer_words=st["smer_words"],
             xchg_rounds=st["xchg_rounds"], exact_reruns=st["exact_reruns"], inc_rounds=st["inc_rounds"],
             inc_fallbacks=st["inc_fallbacks"], inc_redone_coarse=st["inc_redone_coarse"], inc_slack=st["inc_slack"])
    c.close()
    dist.barrier()
    dist.destroy_process_group()


def run_shared(rank: int, world: int, port: int, k: int, out_dir: str, opts: dict):
    """One host rank of a SharedGpuCounter: world ranks over opts["counters"] counters on the one GPU."""
    import torch.distributed as dist

    import mhm2_proxy_amd as m
    from common import synth_set

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b, o = synth_set(opts.get("n_reads", 1200), opts.get("genome", 9000), opts["seed"])
    lo, hi = shard(o.size - 1, rank, world)
    sc = m.SharedGpuCounter(k, opts["counters"], device=0)
    sc.add_packed_reads(b[int(o[lo]):int(o[hi])], (o[lo:hi + 1] - o[lo]).astype(np.uint64))
    t = sc.finish()
    np.savez(Path(out_dir) / f"rank{rank}.npz", keys=t.keys, counts=t.counts, left=t.left, right=t.right,
             leader=int(sc.counter is not None))
    sc.close()
    dist.barrier()
    dist.destroy_process_group()


def run_share(rank: int, world: int, port: int, k: int, out_dir: str, opts: dict):
    """One rank of a C3 / C4 per-rank share: reads [rank * R, (rank + 1) * R) of the config's global read set
    (genome opts["genome"], seed opts["seed"]) counted with opts["owner"], exchanged over the host transport. The
    owner's part of the table (hundreds of millions of rows) is reduced to its table_digest for the parent."""
    import time

    import torch.distributed as dist

    import mhm2_proxy_amd as m
    from common import table_digest

    t0 = time.time()

    def say(what):
        print(f"[rank {rank} {time.time() - t0:6.1f}s] {what}", flush=True)

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MHMKC_XPIPE=opts.get("xpipe", "1"))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    R = opts["reads_per_rank"]
    g = m.synth_genome(opts["genome"], opts["seed"])
    b, o = m.synth_reads(g, R, 150, opts["seed"], first_read=rank * R)
    del g
    say(f"{R} reads")
    owner = m.MHMKC_OWNER_MINIMIZER if opts.get("owner") == "minimizer" else m.MHMKC_OWNER_HASH
    c = m.KmerCounter(k, device=0, rank=rank, n_ranks=world, transport=m.TorchDistTransport(), output_owner=owner)
    c.add_packed_reads(b, o)
    del b, o
    c.finish()
    say("counted")
    t = c.fetch()
    st = c.stats()
    c.close()
    say(f"fetched {len(t)} rows")
    d = table_digest(t)
    del t
    say(f"digest ({d['keys'].shape[0]} sampled rows)")
    np.savez(Path(out_dir) / f"rank{rank}_digest.npz", **d)
    np.savez(Path(out_dir) / f"rank{rank}_stats.npz", **{key: st[key] for key in ("occurrences", "owned_records", "bytes_sent",
                                                                                 "bytes_recv", "exact_reruns", "smer_count")})
    dist.barrier()
    dist.destroy_process_group()


def run_bad_offsets(rank: int, world: int, port: int, k: int, out_dir: str, opts: dict):
    """a device batch whose offsets do not start at 0 (offs[0] = 16) is refused with MHMKC_EINVAL at the
    add, with and without the pipelined exchange (MHMKC_XPIPE, which cuts the batch into pieces); no collective has
    run, so every rank just records the code."""
    import torch
    import torch.distributed as dist

    import mhm2_proxy_amd as m
    from common import synth_set

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MHMKC_XPIPE=opts["xpipe"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b, o = synth_set(2000, 9000, opts.get("seed", 5))
    c = m.KmerCounter(k, device=0, rank=rank, n_ranks=world, transport=m.TorchDistTransport())
    bt = torch.from_numpy(np.concatenate([np.zeros(16, np.uint8), b])).cuda()
    ot = torch.from_numpy(o.astype(np.int64) + 16).cuda()
    code = 0
    try:
        c.add_tensors(bt, ot, n_bases=int(o[-1]) + 16)
    except m.MhmkcError as e:
        code = e.code
    np.savez(Path(out_dir) / f"rank{rank}.npz", code=code)
    c.close()
    dist.barrier()
    dist.destroy_process_group()


def run_share_full(rank: int, world: int, port: int, k: int, out_dir: str, opts: dict):
    """One rank of C3 / C4 as configured: reads [rank * R, (rank + 1) * R) of the config's 1e8-read
    set (genome opts["genome"], seed opts["seed"]) counted with opts["owner"], exchanged over the host transport, the
    owned range counted in opts["passes"] finish passes. The rank's rows leave as (key-range part, row fingerprint)
    pairs for the parent's part-by-part comparison with the CPU restatement; with the minimizer owner every row is
    first checked to be on its get_kmer_target_rank."""
    import time

    import torch.distributed as dist

    import mhm2_proxy_amd as m
    import oracle_lib as O

    t0 = time.time()

    def say(what):
        print(f"[rank {rank} {time.time() - t0:6.1f}s] {what}", flush=True)

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MHMKC_XPIPE=opts.get("xpipe", "1"))
    if opts.get("passes"):
        os.environ["MHMKC_PASSES"] = str(opts["passes"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    R = opts["reads_per_rank"]
    g = m.synth_genome(opts["genome"], opts["seed"])
    b, o = m.synth_reads(g, R, 150, opts["seed"], first_read=rank * R, threads=2)
    del g
    say(f"{R} reads")
    owner = m.MHMKC_OWNER_MINIMIZER if opts.get("owner") == "minimizer" else m.MHMKC_OWNER_HASH
    if opts.get("rccl"):  # libmhmkc's RCCL path, as the 8-GPU run takes it (per-rank NCCL_HOSTID: rccl_same_gpu_env)
        rccl_same_gpu_env(rank)
        obj = [m.comm_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        c = m.KmerCounter(k, device=0, rank=rank, n_ranks=world, comm_id=obj[0], output_owner=owner)
    else:
        c = m.KmerCounter(k, device=0, rank=rank, n_ranks=world, transport=m.TorchDistTransport(), output_owner=owner)
    dist.barrier()
    t1 = time.time()
    if opts.get("device_batch"):  # one device batch (bench.py's path: cut into MHMKC_XPIECES pipelined slabs)
        import torch

        bt = torch.from_numpy(b).cuda()
        ot = torch.from_numpy(o.view(np.int64)).cuda()
        del b, o
        c.add_tensors(bt, ot)
    else:
        c.add_packed_reads(b, o)
        del b, o
    c.finish()
    t_count = time.time() - t1
    st = c.stats()
    say(f"counted in {t_count:.1f} s: {st['n_out']} rows, {st['finish_passes']} passes, device "
        f"{st['device_bytes'] / 2**30:.1f} GiB (peak {st['device_bytes_peak'] / 2**30:.1f} GiB), sent "
        f"{st['bytes_sent'] / 2**30:.2f} GiB")
    t = c.fetch()
    lr = lr_check(c, t)
    c.close()
    if lr["bad_rows"].size:
        say(f"{lr['bad_rows'].size} rows with left/right outside ACGTXF: {lr}")
    np.savez(Path(out_dir) / f"rank{rank}_lr.npz", **lr)
    if owner == m.MHMKC_OWNER_MINIMIZER:
        off = np.flatnonzero(O.target_ranks(t.keys, k, world) != rank)
        assert off.size == 0, f"rank {rank}: {off.size} rows not on their target rank"
    parts = O.mt_ranges(t.keys, k, opts["n_parts"])
    fps = O.row_fingerprints(t.keys, t.counts, t.left, t.right, k)
    del t
    np.save(Path(out_dir) / f"rank{rank}_parts.npy", parts)
    np.save(Path(out_dir) / f"rank{rank}_fps.npy", fps)
    say(f"{fps.size} row fingerprints saved")
    np.savez(Path(out_dir) / f"rank{rank}_stats.npz", seconds=t_count,
             **{key: st[key] for key in ("occurrences", "owned_records", "bytes_sent", "bytes_recv", "exact_reruns",
                                         "smer_count", "n_out", "distinct", "count_sum", "finish_passes", "out_reruns",
                                         "device_bytes", "device_bytes_peak", "xchg_rounds", "ms_xchg",
                                         "inc_rounds", "inc_fallbacks", "ms_finish_tail", "inc_redone_coarse", "inc_slack")})
    dist.barrier()
    dist.destroy_process_group()


VALID_EXT = np.frombuffer(b"ACGTXF", dtype=np.uint8)


def lr_check(counter, t):
    """Rows of a fetched table whose left / right byte is not one of get_ext's results (A C G T X F): their indices,
    the bytes as fetched, the bytes of a second fetch, and the bytes in device memory read back by a separate small
    copy of just those rows, which tells a transfer that lost bytes from a table written wrong on the device."""
    left, right = np.asarray(t.left).view(np.uint8), np.asarray(t.right).view(np.uint8)
    bad = np.flatnonzero(~(np.isin(left, VALID_EXT) & np.isin(right, VALID_EXT)))
    out = {"bad_rows": bad.astype(np.int64), "n_rows": np.int64(left.size),
           "first_left": left[bad], "first_right": right[bad]}
    if bad.size:
        t2 = counter.fetch()
        out["second_left"] = np.asarray(t2.left).view(np.uint8)[bad]
        out["second_right"] = np.asarray(t2.right).view(np.uint8)[bad]
        import ctypes as C

        import torch

        dev = counter.device_output()
        # the device bytes of the bad rows, one small hipMemcpy each (torch's own copy path, not libmhmkc's d2h)
        hip = C.CDLL("libamdhip64.so")
        hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        dl, dr = np.zeros(bad.size, np.uint8), np.zeros(bad.size, np.uint8)
        for j, i in enumerate(bad[:64]):
            b1, b2 = C.c_uint8(0), C.c_uint8(0)
            hip.hipMemcpy(C.byref(b1), C.c_void_p(dev["left"] + int(i)), 1, 2)
            hip.hipMemcpy(C.byref(b2), C.c_void_p(dev["right"] + int(i)), 1, 2)
            dl[j], dr[j] = b1.value, b2.value
        out["device_left"], out["device_right"] = dl, dr
        torch.cuda.synchronize()
    return out


def read_ctgs(path):
    """The contig file mhmkc_dbjg_traverse writes ("<seq> <uint16 depth>" lines): (seqs, depths)."""
    seqs, depths = [], []
    with open(path) as f:
        for line in f:
            s, d = line.split()
            seqs.append(s)
            depths.append(int(d))
    return seqs, np.array(depths, dtype=np.uint16)


def run_c5(rank: int, world: int, port: int, k_unused: int, out_dir: str, opts: dict):
    """One rank of the C5-shaped multi-k chain (src/contigging.cpp:93-158, src/kcount/kcount.cpp:
    100-138): the merged reads (out_dir/merged.npz, the device merge of the paired set, checked by the parent) sharded
    over the ranks. For every k of opts["ks"] the rank counts its shard plus its block of the previous round's contigs
    (add_ctg_kmers; the blocks in rank order are the traversal's order, the order the contig pass applies them in)
    with opts["owner"] over RCCL (opts["rccl"]) or the host transport, and saves its rows; rank 0 then traverses the
    union of the ranks' tables (the restated dbjg, tools/cpp/dbjg_lib.cpp) into out_dir/ctgs_k<next>.txt."""
    import ctypes as C
    import time

    import torch.distributed as dist

    import mhm2_proxy_amd as m

    t0 = time.time()

    def say(what):
        print(f"[c5 rank {rank} {time.time() - t0:6.1f}s] {what}", flush=True)

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    z = np.load(Path(out_dir) / "merged.npz")
    b, o = z["bytes"], z["offs"]
    lo, hi = shard(o.size - 1, rank, world)
    b, o = b[int(o[lo]):int(o[hi])].copy(), (o[lo:hi + 1] - o[lo]).astype(np.uint64)
    owner = m.MHMKC_OWNER_MINIMIZER if opts.get("owner") == "minimizer" else m.MHMKC_OWNER_HASH
    if opts.get("rccl"):
        rccl_same_gpu_env(rank)
    ks = opts["ks"]
    for i, k in enumerate(ks):
        if opts.get("rccl"):
            obj = [m.comm_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            c = m.KmerCounter(k, device=0, rank=rank, n_ranks=world, comm_id=obj[0], output_owner=owner)
        else:
            c = m.KmerCounter(k, device=0, rank=rank, n_ranks=world, transport=m.TorchDistTransport(),
                              output_owner=owner)
        c.add_packed_reads(b, o)
        if i:
            seqs, depths = read_ctgs(Path(out_dir) / f"ctgs_k{k}.txt")
            a, e = shard(len(seqs), rank, world)
            c.add_ctgs(seqs[a:e], depths[a:e])
        c.finish()
        t = c.fetch()
        st = c.stats()
        c.close()
        nl = k // 32 + 1
        np.savez(Path(out_dir) / f"k{k}_rank{rank}.npz", keys=np.ascontiguousarray(t.keys[:, :nl]), counts=t.counts,
                 left=t.left, right=t.right, ctg_kmers=st["ctg_kmers"], bytes_sent=st["bytes_sent"],
                 xchg_rounds=st["xchg_rounds"], smer_count=st["smer_count"])
        say(f"k={k}: {len(t)} rows, {st['ctg_kmers']} contig k-mers")
        del t
        dist.barrier()
        if rank == 0 and i + 1 < len(ks):
            parts = [np.load(Path(out_dir) / f"k{k}_rank{r}.npz") for r in range(world)]
            keys = np.ascontiguousarray(np.concatenate([p["keys"] for p in parts]), dtype=np.uint64)
            counts = np.ascontiguousarray(np.concatenate([p["counts"] for p in parts]), dtype=np.uint16)
            left = np.ascontiguousarray(np.concatenate([p["left"] for p in parts])).view(np.uint8)
            right = np.ascontiguousarray(np.concatenate([p["right"] for p in parts])).view(np.uint8)
            from mhm2_proxy_amd import build as B

            L = C.CDLL(str(B.DBJG))
            L.mhmkc_dbjg_traverse.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                                              C.c_char_p]
            L.mhmkc_dbjg_traverse.restype = C.c_int64
            n_ctgs = L.mhmkc_dbjg_traverse(k, keys.ctypes.data, counts.ctypes.data, left.ctypes.data,
                                           right.ctypes.data, keys.shape[0],
                                           os.fsencode(str(Path(out_dir) / f"ctgs_k{ks[i + 1]}.txt")))
            assert n_ctgs > 0, f"k={k}: traversal gave {n_ctgs}"
            say(f"k={k}: traversed the union ({keys.shape[0]} rows) into {n_ctgs} contigs")
        dist.barrier()
    dist.destroy_process_group()
