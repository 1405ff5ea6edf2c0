#!/usr/bin/env python3
"""Benchmark of the MI355X-native kcount stage (BASELINE.json metric: k-mers/s, whole node, k=21, 150 bp).

  python bench.py --gpus N --steps K --warmup W
  (N > 1: either under python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 ...,
   or plain: bench.py then starts the N ranks itself as child processes, before it touches the GPU)
  python bench.py --gpus N --transport host ...   N ranks exchanging through the host-staged transport
   (mhmkc_set_transport over gloo); ranks share the visible GPUs round-robin, so N ranks can be rehearsed on one GPU

A step = one full counting round of this rank's resident read shard: extract -> coarse partition ->
RCCL all-to-all (N > 1) -> fine partition -> LDS hash-table count -> finalize + compacted output table,
i.e. mhmkc_add_reads_device + mhmkc_finish. Reads are already in HBM when the timed region starts.
Workloads (--config):
  C2 (default): configs[1] of BASELINE.json per GPU — 10M synthetic 150 bp reads per GPU, genome 50 Mbp x N
      (30x coverage), seed 2, k = 21 (weak scaling: the driver's N = 1, 2, 4, 8 lines);
  C3: configs[2] — 100M reads in total over the N GPUs (100M / N each), genome 500 Mbp, seed 3, k = 21;
  C4: configs[3] — C3 at k = 63.
value = counted k-mer occurrences of all ranks / max-over-ranks time.

Extra JSON fields: roofline (dominant kernel: algorithmic HBM bytes per launch over its HIP-event time against
8 TB/s; k_count also carries its LDS-floor model), cpu_baseline (the multi-threaded CPU restatement on a bounded
sample, rank 0 at N = 1), stages (per-stage device ms per step), h2d_inclusive (BASELINE.md's window: the same step
from reads in pinned host memory, timed from the first H2D, median of 5 after 3 warm-ups), d2h_fetch (copying the
finished table to the host), kmermap (the streamed hand-off into the C++ adapter's KmerMap).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
# Random-address LDS throughput on MI355X, whole chip, lane-ops/s (tools/micro/lds_atomics.hip,
# profiles/r01_lds_microbench.txt): the cost model of k_count's LDS floor.
LDS_RATE = {"ds_read_b128": 1593.28e9, "ds_add_u32": 5507.50e9, "ds_cmpst_rtn_b32": 3347.90e9,
            "ds_read_b64": 5656.04e9, "ds_write_b32": 6066.34e9}
CONFIGS = {  # reads in total (None: per GPU), genome (per GPU for C2), seed, k
    "C2": dict(reads_per_gpu=10_000_000, reads_total=None, genome=50_000_000, genome_scales=True, seed=2, k=21),
    "C3": dict(reads_per_gpu=None, reads_total=100_000_000, genome=500_000_000, genome_scales=False, seed=3, k=21),
    "C4": dict(reads_per_gpu=None, reads_total=100_000_000, genome=500_000_000, genome_scales=False, seed=3, k=63),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="C2")
    ap.add_argument("--k", type=int, default=None, help="override the config's k")
    ap.add_argument("--reads-per-gpu", type=int, default=None, help="override (C2: reads per GPU)")
    ap.add_argument("--reads-total", type=int, default=None, help="override (C3/C4: reads over all GPUs)")
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--cpu-sample-reads", type=int, default=10_000_000)
    ap.add_argument("--cpu-threads", type=int, default=16, help="CPU baseline threads (the box's CPU share)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--h2d-steps", type=int, default=5,
                    help="timed steps of the H2D-inclusive leg, after 3 warm-ups (BASELINE.md: median of 5; 0: skip)")
    ap.add_argument("--input", choices=("packed", "fastq", "fastq-pairs", "fastq-file"), default="packed",
                    help="packed: PackedRead bytes in HBM (the headline); fastq: FASTQ text in HBM, parsed and "
                         "packed on the device inside every step (mhmkc_add_fastq_device); fastq-pairs: interleaved "
                         "paired FASTQ (reads_per_gpu / 2 pairs), parsed, pair-merged and packed on the device "
                         "(mhmkc_add_fastq_pairs_device); fastq-file: the FASTQ text as a file (page cache), read "
                         "in blocks into pinned memory, each block parsed and counted while the next is read "
                         "(mhmkc_add_fastq_file): the step includes the file read and the H2D")
    ap.add_argument("--no-profile-events", action="store_true")
    ap.add_argument("--profile-level", type=int, choices=(1, 2), default=None,
                    help="stage events: 1 every stage, 2 the heavy stages (default for packed input)")
    ap.add_argument("--no-k63", dest="k63", action="store_false",
                    help="N = 1, C2: skip the second leg, C2's reads at k = 63 (C4's two-word Kmer<> path)")
    ap.add_argument("--no-kmermap", dest="kmermap", action="store_false",
                    help="skip timing the hand-off into the C++ adapter's KmerMap")
    ap.add_argument("--transport", choices=("rccl", "host", "rccl-same-gpu"), default="rccl",
                    help="exchange between ranks (N > 1): rccl = one rank per GPU, RCCL grouped send/recv over xGMI; "
                         "host = mhmkc_set_transport over a gloo process group (pinned D2H, gloo, H2D), ranks share "
                         "the visible GPUs round-robin (a rehearsal of the multi-rank path on one GPU); rccl-same-gpu = "
                         "libmhmkc's RCCL path with the ranks sharing the visible GPUs (a per-rank NCCL_HOSTID makes "
                         "RCCL accept them and move the data over its socket transport on loopback: a rehearsal of the "
                         "8-GPU run's code path, not of its speed)")
    ap.add_argument("--owner", choices=("hash", "minimizer"), default="hash",
                    help="N > 1: where a finished k-mer lives: hash = the counting hash range (record exchange); "
                         "minimizer = the reference's get_kmer_target_rank (k >= 33: supermer exchange, DESIGN.md "
                         "§3.5b; k <= 31: record exchange + hand-off)")
    ap.add_argument("--pmc-json", default=str(ROOT / "profiles" / "pmc_traffic.json"),
                    help="per-kernel HBM bytes per launch from rocprofv3 --pmc passes (profiles/), if present")
    return ap.parse_args()


def algorithmic_bytes(stage: str, st: dict, k: int) -> float:
    """Algorithmic HBM bytes of one launch of a stage."""
    nl = k // 32 + 1
    rec, frec = st["coarse_record_bytes"], st["fine_record_bytes"]  # 5 / 4 B compact (k <= 21), else 8 * nl (+1)
    occ, owned, bases = st["occurrences"], st["owned_records"], st["bases"]
    out = st["n_out"] * (8 * nl + 4)
    return {
        "extract_hist": bases,
        "extract_scatter": bases + occ * rec,
        "part_hist": owned * rec,
        "part_scatter": owned * (rec + frec),
        "count": owned * frec + out,
        "exchange": st["bytes_sent"] + st.get("bytes_recv", 0),
    }.get(stage, 0.0)


def lds_floor_seconds(st: dict, k: int) -> tuple:
    """k_count's LDS time floor: its table operations priced at the measured whole-chip
    random-address LDS rates. Per record: the home-group read (one ds_read_b128 of four 32-bit keys; two for
    64-bit keys) and the count add; per extension add one ds_add; per phase-B record (not in its home group)
    one more group read, a CAS and a miss-list write + read. Returns (seconds, LDS bytes)."""
    nl = k // 32 + 1
    g_reads = 1 if st["fine_record_bytes"] == 4 else 2 * nl  # b128 reads per group lookup
    recs, miss, ext = st["owned_records"], st["lds_misses"], st["lds_ext_adds"]
    r = LDS_RATE
    t = (recs * (g_reads / r["ds_read_b128"] + 1 / r["ds_add_u32"]) + ext / r["ds_add_u32"] +
         miss * (g_reads / r["ds_read_b128"] + 1 / r["ds_cmpst_rtn_b32"] + 2 * nl / r["ds_write_b32"] +
                 nl / r["ds_read_b64"]))
    b = recs * (16 * g_reads + 4) + ext * 4 + miss * (16 * g_reads + 4 + 16 * nl)
    return t, b


def handoff_ms(counter, k: int, threads: int, runs: int = 3):
    """The hand-off into the C++ adapter's KmerMap, timed in this process on the finished device table (SURVEY.md
    §8(d)): tools/bin/libmhmkc_handoff.so runs include/mhmkc_kcount.hpp's load_ordered on the counter's handle, which
    is what HashTableInserter::insert_into_local_hashtable does after mhmkc_finish (the device sort into the map's slot
    order, chunked D2H on a helper thread, the parallel fill of a fresh map; src/kcount/kcount_cpu.cpp:503-522). The
    first run includes the device sort (ms_cold); later runs reuse the sorted rows (the sort is ~1.5 ms at C2). Every
    run fills a fresh map (its page faults included); a sample of the rows is looked up after every run (untimed)."""
    import ctypes as C

    lib_path = ROOT / "tools" / "bin" / "libmhmkc_handoff.so"
    if not lib_path.exists():
        return None
    lib = C.CDLL(str(lib_path))
    from mhm2_proxy_amd import _native as N

    abi = N.lib().mhmkc_abi_version()
    if not hasattr(lib, "mhmkc_handoff_abi") or lib.mhmkc_handoff_abi() != abi:
        return {"error": f"tools/bin/libmhmkc_handoff.so was built for another libmhmkc ABI than {abi}: run build()"}
    lib.mhmkc_handoff_ms.restype = C.c_double
    lib.mhmkc_handoff_ms.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_uint64, C.POINTER(C.c_uint64),
                                     C.POINTER(C.c_uint64), C.POINTER(C.c_double)]
    ms, size, bad, parts = [], C.c_uint64(0), C.c_uint64(0), []
    for _ in range(runs):
        pa = (C.c_double * 5)()
        t = lib.mhmkc_handoff_ms(counter._h, k, threads, 0, C.byref(size), C.byref(bad), pa)
        if t < 0:
            return {"error": "library error in the hand-off"}
        ms.append(t)
        parts.append({n_: round(v, 1) for n_, v in zip(("first_fetch_incl_sort", "fill", "wait_fetch", "begin", "end"),
                                                        pa)})
    return {"ms": round(sorted(ms)[len(ms) // 2], 1), "statistic": f"median of {runs} runs",
            "ms_cold": round(ms[0], 1), "runs_ms": [round(x, 1) for x in ms], "rows": counter.n_out,
            "map_size": int(size.value), "sample_rows_bad": int(bad.value), "threads": threads, "parts_ms": parts,
            "kind": "C++ adapter load_ordered (HashTableInserter::insert_into_local_hashtable): device sort by KmerMap "
                    "slot, 4M-row chunks D2H on a helper thread overlapped with the parallel fill of a fresh "
                    "KmerMap<MAX_K> (tools/cpp/handoff.cpp)"}


def survey_model_bytes(st: dict, k: int, n_reads: int, read_len: int) -> float:
    """SURVEY.md §8(d) B_alg of one step on one GPU: the reference's DRAM-table traffic model (2-bit read
    stream, one S_slot read + write per occurrence, compacted output), without its capacity-dependent
    finalize-scan term. It prices the work the reference's hash table does; this design keeps that table
    in LDS, so the figure is a path-level yardstick, not the HBM bytes moved."""
    nl = k // 32 + 1
    s_slot = 8 * nl + 20
    return n_reads * ((3 * read_len + 7) // 8) + st["occurrences"] * 2 * s_slot + st["n_out"] * (8 * nl + 4)


def fastq_text(b, o, read_len: int):
    """FASTQ text of fixed-length packed reads, vectorised: '@r%010d', sequence, '+', quality (q + 33)."""
    import numpy as np

    n = len(o) - 1
    L = read_len
    rec = 13 + (L + 1) + 2 + (L + 1)
    t = np.empty((n, rec), dtype=np.uint8)
    t[:, 0], t[:, 1] = ord("@"), ord("r")
    idx = np.arange(n, dtype=np.int64)
    for p in range(10):
        t[:, 11 - p] = ord("0") + (idx // 10 ** p) % 10
    t[:, 12] = ord("\n")
    bb = b.reshape(n, L)
    t[:, 13:13 + L] = np.frombuffer(b"ACGTNNNN", dtype=np.uint8)[bb & 7]
    t[:, 13 + L], t[:, 14 + L], t[:, 15 + L] = ord("\n"), ord("+"), ord("\n")
    t[:, 16 + L:16 + 2 * L] = (bb >> 3) + 33
    t[:, 16 + 2 * L] = ord("\n")
    return t.reshape(-1)


def paired_fastq_text(genome, n_pairs: int, read_len: int, seed: int, frag_mean: int = 250, frag_sd: int = 25):
    """Interleaved paired FASTQ, vectorised: fragment F ~ N(frag_mean, frag_sd) at a uniform start, mate 1 =
    its first L bases, mate 2 = the reverse complement of its last L bases ('@p%010d/1' and '/2'), 0.5 %
    substitutions at quality '#', 2 % of bases at quality '+', the rest 'I'. Most pairs overlap by 2L - F."""
    import numpy as np

    rng = np.random.default_rng(seed)
    L = read_len
    G = genome.size
    rec = 15 + (L + 1) + 2 + (L + 1)  # '@p' + 10 digits + '/m' + '\n', sequence, '+\n', qualities
    out = np.empty((2 * n_pairs, rec), dtype=np.uint8)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    step = 1 << 18
    for c0 in range(0, n_pairs, step):
        n = min(step, n_pairs - c0)
        F = np.clip(rng.normal(frag_mean, frag_sd, size=n), L, 2 * L + 100).astype(np.int64)
        a = (rng.random(n) * (G - F)).astype(np.int64)
        pos1 = a[:, None] + np.arange(L)[None, :]
        pos2 = (a + F - 1)[:, None] - np.arange(L)[None, :]
        m1 = genome[pos1]
        m2 = 3 - genome[pos2]  # complement of the reversed end
        for m in (m1, m2):
            sub = rng.random(m.shape) < 0.005
            m[sub] = (m[sub] + rng.integers(1, 4, size=int(sub.sum()))) & 3
        t = out[2 * c0:2 * (c0 + n)].reshape(n, 2, rec)
        idx = np.arange(c0, c0 + n, dtype=np.int64)
        t[:, :, 0], t[:, :, 1] = ord("@"), ord("p")
        for d in range(10):
            t[:, :, 11 - d] = (ord("0") + (idx // 10 ** d) % 10)[:, None]
        t[:, :, 12] = ord("/")
        t[:, 0, 13], t[:, 1, 13] = ord("1"), ord("2")
        t[:, :, 14] = ord("\n")
        for j, m in enumerate((m1, m2)):
            t[:, j, 15:15 + L] = acgt[m]
            q = np.full(m.shape, ord("I"), dtype=np.uint8)
            q[rng.random(m.shape) < 0.02] = ord("+")
            t[:, j, 18 + L:18 + 2 * L] = q
        t[:, :, 15 + L], t[:, :, 16 + L], t[:, :, 17 + L] = ord("\n"), ord("+"), ord("\n")
        t[:, :, 18 + 2 * L] = ord("\n")
    return out.reshape(-1)


def cpu_baseline(b, o, k, n_reads, threads):
    """The CPU restatement (oracle/kcount_mt.c: the reference's read-pass rules, hash-partitioned over T
    threads like the reference's ranks) timed on this host on the first n_reads reads."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib as O

    n = min(n_reads, o.size - 1)
    bb, oo = b[: int(o[n])], o[: n + 1]
    t0 = time.perf_counter()
    t = O.kcount_mt(bb, oo, k, threads=threads)
    dt = time.perf_counter() - t0
    occ = t.stats()["occurrences"]
    return {"value": occ / dt, "unit": "k-mers/s", "cores": threads, "kind": "port",
            "sample": f"first {n} reads of this rank's shard ({occ} k-mers), oracle/kcount_mt.c, {threads} threads, "
                      f"{dt:.1f} s"}


def launch_ranks(n: int) -> int:
    """--gpus N > 1 without torch.distributed.run: start the N ranks as child processes of this one (this process
    never touches the GPU: no exec from a GPU process), with the env torchrun would give them (RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_ADDR=127.0.0.1, a free MASTER_PORT). The first rank to fail ends the others; the exit code
    is the first non-zero one."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MHMKC_BENCH_CHILD="1")
        procs.append(subprocess.Popen([sys.executable, "-u", str(Path(__file__).resolve()), *sys.argv[1:]], env=env))
    rc, live = 0, list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0 and rc == 0:
                rc = r if r > 0 else 128 - r
                print(f"bench.py: rank {procs.index(p)} exited with {r}; stopping the other ranks", file=sys.stderr,
                      flush=True)
                for q in live:
                    q.terminate()
        time.sleep(0.1)
    return rc


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(launch_ranks(args.gpus))
    import numpy as np
    import torch

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    host_xp = world > 1 and args.transport == "host"
    same_gpu = world > 1 and args.transport == "rccl-same-gpu"
    if same_gpu:  # before anything initialises RCCL in this process
        os.environ.update(NCCL_HOSTID=f"mhmkc-rehearsal-{rank}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1",
                          NCCL_NET="Socket")
    # the pipelined record exchange: a step goes from its adds to finish with no other collective
    # in between, which is the contract MHMKC_XPIPE asks for (MHMKC_XPIPE=0 in the environment: one exchange at finish)
    if world > 1:
        os.environ.setdefault("MHMKC_XPIPE", "1")
    n_dev = torch.cuda.device_count()
    if n_dev < 1:
        raise SystemExit("bench.py: no GPU visible")
    shared = host_xp or same_gpu  # ranks share the visible GPUs round-robin
    if not shared and local >= n_dev:
        raise SystemExit(f"bench.py: rank {rank} needs GPU {local} (one rank per GPU, RCCL), but {n_dev} visible; "
                         "use --transport host to run several ranks on one GPU")
    local_dev = local % n_dev if shared else local
    torch.cuda.set_device(local_dev)
    dist = None
    cdev = torch.device("cpu") if shared else torch.device("cuda", local_dev)  # where the timing reductions run
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if shared:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local_dev))
    local = local_dev

    import mhm2_proxy_amd as m
    from mhm2_proxy_amd.build import source_build_id

    cf = dict(CONFIGS[args.config])
    k = args.k or cf["k"]
    seed = args.seed if args.seed is not None else cf["seed"]
    L = args.read_len
    if args.reads_total or cf["reads_total"]:
        total = args.reads_total or cf["reads_total"]
        first, R = total * rank // world, total * (rank + 1) // world - total * rank // world
        G = cf["genome"]
    else:
        R = args.reads_per_gpu or cf["reads_per_gpu"]
        total, first = R * world, rank * R
        G = cf["genome"] * world
    threads = max(1, min(16, (os.cpu_count() or 8) // max(1, world)))
    t0 = time.perf_counter()
    genome = m.synth_genome(G, seed)
    b, o = m.synth_reads(genome, R, L, seed, first_read=first, threads=threads)
    del genome
    gen_s = time.perf_counter() - t0
    dev = torch.device("cuda", local)
    if args.input == "fastq-pairs":
        genome = m.synth_genome(G, seed)
        text = paired_fastq_text(genome, R // 2, L, seed)
        del genome
        tt = torch.zeros(int(text.size) + 16, dtype=torch.uint8, device=dev)
        tt[: text.size].copy_(torch.from_numpy(text))
        text_bytes = int(text.size)
        del text
    elif args.input == "fastq-file":
        import tempfile

        text = fastq_text(b, o, L)
        fq_dir = Path("/dev/shm") if Path("/dev/shm").is_dir() else Path(tempfile.gettempdir())
        fq_path = fq_dir / f"mhmkc_bench_{os.getpid()}_{rank}.fq"
        text.tofile(str(fq_path))
        text_bytes = int(text.size)
        del text
    elif args.input == "fastq":
        text = fastq_text(b, o, L)
        tt = torch.zeros(int(text.size) + 16, dtype=torch.uint8, device=dev)  # 4+ bytes of padding (mhmkc.h)
        tt[: text.size].copy_(torch.from_numpy(text))
        text_bytes = int(text.size)
        del text
    else:
        bt = torch.from_numpy(b).to(dev)
        ot = torch.from_numpy(o.view(np.int64)).to(dev)
    n_bases = int(o[-1])
    torch.cuda.synchronize()

    cid = None
    if world > 1 and not host_xp:
        obj = [m.comm_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        cid = obj[0]
    counter = m.KmerCounter(k, device=local, rank=rank, n_ranks=world, comm_id=cid,
                            transport=m.TorchDistTransport() if host_xp else None,
                            output_owner=m.MHMKC_OWNER_MINIMIZER if args.owner == "minimizer" else m.MHMKC_OWNER_HASH)
    # events around the heavy stages only (each event record is a marker the next launch waits behind: all stages
    # measured 0.07-0.2 ms per step slower than none)
    # (FASTQ inputs time their ingest as stage "other": every stage)
    counter.set_profiling(0 if args.no_profile_events else args.profile_level if args.profile_level is not None
                          else 1 if args.input != "packed" else 2)

    def step():
        counter.reset()
        if args.input == "fastq-file":
            counter.add_fastq_file(fq_path)
        elif args.input == "fastq":
            counter.add_fastq_tensor(tt, n_bytes=text_bytes)
        elif args.input == "fastq-pairs":
            counter.add_fastq_tensor(tt, n_bytes=text_bytes, pairs=True)
        else:
            counter.add_tensors(bt, ot, n_bases=n_bases)
        counter.finish()

    for _ in range(args.warmup):
        step()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    stage_ms = {}
    launches = {}
    occ_total = 0
    st = None
    step_s = []
    for _ in range(args.steps):
        t_s = time.perf_counter()
        step()
        st = counter.stats()
        step_s.append(time.perf_counter() - t_s)
        occ_total += st["occurrences"]
        for s_, v in st["ms_kernel"].items():
            stage_ms[s_] = stage_ms.get(s_, 0.0) + v
            launches[s_] = launches.get(s_, 0) + st["launches"][s_]
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        c = torch.tensor([occ_total], dtype=torch.float64, device=cdev)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        occ_total = int(c.item())

    value = occ_total / elapsed
    steps = max(1, args.steps)
    per_step = {s_: v / steps for s_, v in stage_ms.items()}
    dom = max((s_ for s_ in per_step if s_ not in ("other", "tileidx")), key=lambda s_: per_step[s_], default=None)
    roofline = None
    pmc = {}
    if Path(args.pmc_json).exists():
        try:
            pmc = json.loads(Path(args.pmc_json).read_text())
        except Exception:
            pmc = {}
    # measured for this workload only (the config's own sizes)
    pmc = {} if (args.reads_per_gpu or args.reads_total) else pmc.get("configs", {}).get(f"{args.config}/k{k}", {})
    def roofline_of(stage, stage_ms=stage_ms, launches=launches, st=st, k=k, pmc=pmc):
        """The roofline object of one stage's kernel: algorithmic HBM bytes per launch over the launch's HIP-event
        time, against the 8 TB/s HBM peak (k_count also carries its LDS-floor model)."""
        ms_launch = stage_ms[stage] / launches[stage]
        alg = algorithmic_bytes(stage, st, k) / max(1, launches[stage] // steps)
        hbm = {"achieved": round(alg / (ms_launch * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
               "frac": round(alg / (ms_launch * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4), "algorithmic_bytes": int(alg)}
        traffic = pmc.get("per_launch_bytes", {}).get(stage)
        extra = {}
        if stage == "count":
            # k_count keeps its hash table in LDS: beside its HBM roofline, the LDS time floor of its
            # table operations at the measured random-access LDS rates (a model, not a hardware peak)
            t_floor, lds_b = lds_floor_seconds(st, k)
            extra = {"lds_model": {"floor_ms": round(t_floor * 1e3, 4), "frac": round(t_floor / (ms_launch * 1e-3), 4),
                                   "lds_TBps": round(lds_b / (ms_launch * 1e-3) / 1e12, 3),
                                   "ops": {"records": st["owned_records"], "phase_b_records": st["lds_misses"],
                                           "ext_adds": st["lds_ext_adds"]}}}
        # the issue roofline beside it: the fraction of the kernel's cycles its SIMDs spent issuing VALU instructions
        # (PMC, tools/pmc_traffic.py); at k = 21 about half of the extraction's and 40 % of k_count's cycles
        valu = pmc.get("valu_issue_frac", {}).get(stage)
        if valu is not None:
            extra["valu_issue_frac"] = valu
        return {"bound": "hbm", "kernel": "k_" + stage, "achieved": hbm["achieved"], "peak": HBM_PEAK_GBPS,
                "unit": "GB/s", "frac": hbm["frac"], "traffic": traffic, "traffic_source": pmc.get("source"),
                "algorithmic_bytes": int(alg), "avg_launch_ms": round(ms_launch, 4), **extra}

    if dom and launches.get(dom):
        roofline = roofline_of(dom)
    # every main kernel's roofline (at k = 21 extraction and counting take about the same time, so the dominant one
    # changes from run to run)
    rooflines = {s_: roofline_of(s_) for s_ in ("extract_scatter", "part_scatter", "count") if launches.get(s_)}

    # D2H of the finished table (the KmerMap fill starts from it), into host arrays that exist already (their first
    # touch is the caller's allocation, not the transfer): pageable (numpy) and pinned (torch pin_memory) ones;
    # median of 3 each
    def timed_fetch(ordered, out):
        ts = []
        for _ in range(3):
            t1 = time.perf_counter()
            counter.fetch(ordered=ordered, out=out)
            ts.append((time.perf_counter() - t1) * 1e3)
        return sorted(ts)[1]

    # the hand-off into the adapter's KmerMap first: its first run includes the device sort into slot order
    kmermap = handoff_ms(counter, k, threads) if rank == 0 and args.kmermap else None
    n_rows = counter.n_out
    row_b = 8 * counter.n_longs + 4
    table = m.KmerTable(k, np.ones((n_rows, counter.n_longs), np.uint64), np.ones(n_rows, np.uint16),
                        np.ones(n_rows, np.uint8), np.ones(n_rows, np.uint8))
    d2h_ms = timed_fetch(False, table)
    d2h = {"ms": round(d2h_ms, 2), "rows": n_rows, "bytes": int(n_rows * row_b),
           "GBps": round(n_rows * row_b / (d2h_ms * 1e-3) / 1e9, 2) if d2h_ms else None,
           "ordered_ms": round(timed_fetch(True, table), 2),
           "into": "existing pageable host arrays (numpy)"}
    try:
        pin = [torch.empty(a.shape, dtype=t, pin_memory=True) for a, t in
               ((table.keys, torch.int64), (table.counts, torch.int16), (table.left, torch.uint8),
                (table.right, torch.uint8))]
        ptab = m.KmerTable(k, pin[0].numpy().view(np.uint64), pin[1].numpy().view(np.uint16), pin[2].numpy(),
                           pin[3].numpy())
        d2h["pinned_ms"] = round(timed_fetch(False, ptab), 2)
        d2h["pinned_ordered_ms"] = round(timed_fetch(True, ptab), 2)
        d2h["pinned_GBps"] = round(n_rows * row_b / (d2h["pinned_ms"] * 1e-3) / 1e9, 2)
        del ptab, pin
    except RuntimeError:
        pass
    del table

    # the same step from reads in pinned host memory: chunked H2D on a copy stream, each chunk extracted as
    # soon as it lands (mhmkc_add_reads); the timed region starts at the first H2D
    h2d = None
    if args.h2d_steps and args.input == "packed":
        hb = torch.from_numpy(b).pin_memory().numpy()
        ho = torch.from_numpy(o.view(np.int64)).pin_memory().numpy().view(np.uint64)
        counter.set_profiling(False)
        ts, h2d_ms, pack_ms, raw_chunks = [], [], [], []
        for i in range(args.h2d_steps + 3):
            if dist:
                dist.barrier()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            counter.reset()
            counter.add_packed_reads(hb, ho)
            counter.finish()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t1
            if dist:
                tt_ = torch.tensor([dt], dtype=torch.float64, device=cdev)
                dist.all_reduce(tt_, op=dist.ReduceOp.MAX)
                dt = float(tt_.item())
            if i >= 3:  # three warm-ups (pinned staging, chunk events), BASELINE.md:74
                ts.append(dt)
                h2d_ms.append(counter.stats()["ms_h2d"])
                pack_ms.append(counter.stats()["ms_h2d_pack"])
                raw_chunks.append(counter.stats()["h2d_raw_chunks"])
        tmed = sorted(ts)[len(ts) // 2]
        stt = counter.stats()
        hbytes = stt["h2d_bytes"]
        h2d = {"value": round(occ_total / steps * 1.0 / tmed, 1), "unit": "k-mers/s", "ms_per_step": round(tmed * 1e3, 3),
               "h2d_ms": round(sorted(h2d_ms)[len(h2d_ms) // 2], 3), "h2d_bytes_per_gpu": int(hbytes),
               "host_pack_ms": round(sorted(pack_ms)[len(pack_ms) // 2], 3), "raw_chunks_per_step": raw_chunks,
               "h2d_GBps": round(hbytes / (sorted(h2d_ms)[len(h2d_ms) // 2] * 1e-3) / 1e9, 1) if h2d_ms[0] else None,
               "chunks": int(stt["h2d_chunks"]), "steps": len(ts), "warmup": 3, "statistic": "median",
               "input": "PackedRead bytes + offsets in pinned host memory (torch pin_memory)",
               "wire": "bases as nibbles (code, q >= cutoff), packed by host threads" if hbytes < int(o[-1])
               else "PackedRead bytes",
               "window": "BASELINE.md:74-75: from the first H2D of the reads to the finished device table"}
        del hb, ho

    # C4's one-GPU figure: the same resident reads counted at k = 63, the two-word Kmer<> path
    # (mixed 16-byte records, two-word LDS table), timed like the headline leg; not `value`
    k63 = None
    if world == 1 and args.k63 and args.config == "C2" and args.input == "packed" and k != 63 and not args.reads_per_gpu:
        c63 = m.KmerCounter(63, device=local)
        c63.set_profiling(0 if args.no_profile_events else 2)

        def step63():
            c63.reset()
            c63.add_tensors(bt, ot, n_bases=n_bases)
            c63.finish()

        for _ in range(args.warmup):
            step63()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        sm63, la63, occ63, st63 = {}, {}, 0, None
        for _ in range(args.steps):
            step63()
            st63 = c63.stats()
            occ63 += st63["occurrences"]
            for s_, v in st63["ms_kernel"].items():
                sm63[s_] = sm63.get(s_, 0.0) + v
                la63[s_] = la63.get(s_, 0) + st63["launches"][s_]
        torch.cuda.synchronize()
        el63 = time.perf_counter() - t1
        pmc63 = {}
        if Path(args.pmc_json).exists():
            try:
                pmc63 = json.loads(Path(args.pmc_json).read_text()).get("configs", {}).get("C2/k63", {})
            except Exception:
                pmc63 = {}
        k63 = {"workload": f"C2's reads ({R} x {L} bp, genome {G} bp, seed {seed}) at k = 63: C4's two-word path on one GPU",
               "value": round(occ63 / el63, 1), "unit": "k-mers/s", "ms_per_step": round(el63 / steps * 1e3, 3),
               "steps": args.steps, "warmup": args.warmup,
               "stages_ms_per_step": {**{s_: round(v / steps, 3) for s_, v in sm63.items() if la63.get(s_)},
                                      "rest": round(el63 / steps * 1e3 - sum(v / steps for s_, v in sm63.items()
                                                                               if la63.get(s_)), 3)},
               "rooflines": {s_: roofline_of(s_, sm63, la63, st63, 63, pmc63)
                             for s_ in ("extract_scatter", "part_scatter", "count") if la63.get(s_)},
               "n_out": st63["n_out"], "distinct": st63["distinct"]}
        c63.close()

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(b, o, k, args.cpu_sample_reads, args.cpu_threads)

    if rank == 0:
        launched = [s_ for s_ in per_step if launches.get(s_)]
        line = {
            "metric": f"k-mers/s (whole node), k={k} {L}bp reads",
            "value": round(value, 1),
            "unit": "k-mers/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / steps * 1e3, 3),
            "ms_per_step_median": round(sorted(step_s)[len(step_s) // 2] * 1e3, 3) if step_s else None,
            "higher_is_better": True,
            "scaling": "weak" if args.config == "C2" else "strong",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (SURVEY.md §8(d) generator: splitmix64 genome + reads, 0.5% subst, 0.02% N, 2% Q10)",
            "config": {"workload": (f"{args.config}: {total} x {L}bp synthetic reads ({R} on rank 0), k={k}, genome "
                                    f"{G} bp, seed {seed}"),
                       "k": k, "reads_total": total, "reads_per_gpu": R, "read_len": L, "genome_len": G,
                       "occurrences_per_step": occ_total // steps, "parallelism": f"hash-range x{world}",
                       "transport": args.transport if world > 1 else None,
                       "physical_gpus": min(world, n_dev) if shared else world},
            "roofline": roofline,
            "rooflines": rooflines,
            "cpu_baseline": cpu,
            # (events around the heavy stages only, mhmkc_set_profiling level 2: "rest" is the step's time outside
            # them: the tile index, layouts, small copies and the host's turns between launches)
            "stages_ms_per_step": {**{s_: round(v, 3) for s_, v in per_step.items() if launches.get(s_)},
                                   "rest": round(elapsed / steps * 1e3 - sum(v for s_, v in per_step.items()
                                                                            if launches.get(s_)), 3)},
            "achieved_measured_GBps_whole_step": round(
                sum(pmc["per_launch_bytes"][s_] * launches[s_] / steps for s_ in launched
                    if s_ not in ("other", "tileidx")) / (elapsed / steps) / 1e9, 1)
            if pmc.get("per_launch_bytes") and all(s_ in pmc["per_launch_bytes"] for s_ in launched
                                                   if s_ not in ("other", "tileidx")) else None,
            "l2_hit": pmc.get("l2_hit"),
            "achieved_alg_GBps_whole_step": round(
                sum(algorithmic_bytes(s_, st, k) * launches[s_] / steps for s_ in launched) / (elapsed / steps) / 1e9,
                1) if st else None,
            "survey_model": {
                "bytes_per_step_per_gpu": int(survey_model_bytes(st, k, R, L)),
                "GBps_per_gpu": round(survey_model_bytes(st, k, R, L) / (elapsed / steps) / 1e9, 1),
                "frac_of_hbm_peak": round(survey_model_bytes(st, k, R, L) / (elapsed / steps) / 1e9 / HBM_PEAK_GBPS, 4),
            } if st else None,
            "h2d_inclusive": h2d,
            "d2h_fetch": d2h,
            "kmermap": kmermap,
            "k63": k63,
            "d2h_kmermap_ms": kmermap["ms"] if kmermap and "ms" in kmermap else None,
            "distinct_per_gpu": st["distinct"] if st else None,
            "n_out_per_gpu": st["n_out"] if st else None,
            "bytes_sent_rank0": st["bytes_sent"] if st else None,
            "exchange": ({"transport": ("host-staged (mhmkc_set_transport over gloo: pinned D2H, gloo all-to-all-v, "
                                        f"H2D), {world} ranks on {min(world, n_dev)} physical GPU(s)")
                          if host_xp else
                          (f"RCCL grouped ncclSend/ncclRecv, {world} ranks on {min(world, n_dev)} physical GPU(s) "
                           "(per-rank NCCL_HOSTID: RCCL's socket transport on loopback)") if same_gpu else
                          "RCCL grouped ncclSend/ncclRecv over xGMI, one rank per GPU",
                          "ms_per_step_rank0": round(per_step.get("exchange", 0.0), 3),
                          "bytes_sent_per_step_rank0": st["bytes_sent"], "bytes_recv_per_step_rank0": st["bytes_recv"],
                          "bytes_sent_per_occurrence": round(st["bytes_sent"] / max(1, st["occurrences"]), 3),
                          "owner": args.owner,
                          "wire": ("supermers (2-bit codes + extension bits in 32-base words + a descriptor)"
                                   if st["smer_count"] else "records"),
                          "handoff_rows_sent_rank0": st["handoff_sent"],
                          "pipelined": bool(st["xchg_rounds"]),
                          "rounds_rank0": st["xchg_rounds"],
                          # pipelined: device time of the rounds' transfers, and the part of it after the last
                          # extraction ended (the rest overlapped extraction)
                          "ms_transfers_rank0": round(st["ms_xchg"], 3) if st["xchg_rounds"] else None,
                          "ms_exposed_rank0": round(st["ms_xchg_exposed"], 3) if st["xchg_rounds"] else None,
                          # the incremental fine partition: rounds partitioned as they landed, and
                          # the device time from the last transfer's end to the finished table
                          "inc_rounds_rank0": st["inc_rounds"], "inc_fallbacks_rank0": st["inc_fallbacks"],
                          "inc_redone_coarse_rank0": st["inc_redone_coarse"], "inc_slack_rank0": round(st["inc_slack"], 3),
                          "ms_finish_tail_rank0": round(st["ms_finish_tail"], 3),
                          "GBps_rank0": round(st["bytes_sent"] / (per_step["exchange"] * 1e-3) / 1e9, 2)
                          if per_step.get("exchange") else None}
                         if world > 1 and st else None),
            "synth_seconds": round(gen_s, 2),
            "build_id": m._native.build_id(),
            "build_id_matches_tree": m._native.build_id() == source_build_id(),
        }
        if args.input == "fastq-file":
            line["config"]["workload"] = line["config"]["workload"].replace("synthetic reads", "FASTQ records")
            line["config"]["input"] = (f"FASTQ file ({text_bytes} bytes/GPU, {fq_path.parent}) read in "
                                       f"{st['fq_file_blocks'] if st else '?'} blocks into pinned memory, "
                                       "parsed + packed + counted on the device (file read and H2D in the step)")
        if args.input == "fastq":
            # FASTQ ingest (stage "other": k_fq_count/lines/records/pack + scans): text read twice, 8 B per
            # newline written and read, sequence + quality read and the packed byte written per base
            ing_ms = per_step.get("other", 0.0)
            n_lines = 4 * R
            ing_bytes = 2 * text_bytes + 16 * n_lines + 3 * R * L
            line["config"]["workload"] = line["config"]["workload"].replace("synthetic reads", "FASTQ records")
            line["config"]["input"] = f"FASTQ text in HBM ({text_bytes} bytes/GPU), parsed + packed on the device"
            line["ingest"] = {"ms_per_step": round(ing_ms, 3), "text_GBps": round(text_bytes / (ing_ms * 1e-3) / 1e9, 1)
                              if ing_ms else None, "algorithmic_bytes": ing_bytes,
                              "achieved_GBps": round(ing_bytes / (ing_ms * 1e-3) / 1e9, 1) if ing_ms else None}
        print(json.dumps(line), flush=True)
    counter.close()
    if args.input == "fastq-file":
        fq_path.unlink(missing_ok=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
