#!/usr/bin/env python3
"""Benchmark of the MI355X-native kcount stage (BASELINE.json metric: k-mers/s, whole node, k=21, 150 bp).

  python bench.py --gpus N --steps K --warmup W
  (N > 1: python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 ... bench.py)

A step = one full counting round of this rank's resident read shard: extract -> coarse partition ->
RCCL all-to-all (N > 1) -> fine partition -> LDS hash-table count -> finalize + compacted output table,
i.e. mhmkc_add_reads_device + mhmkc_finish. Reads are already in HBM when the timed region starts.
Workload (weak scaling): configs[1] of BASELINE.json per GPU — 10M synthetic 150 bp reads per GPU, genome
50 Mbp x N (30x coverage), k = 21. value = counted k-mer occurrences of all ranks / max-over-ranks time.

Extra JSON fields: roofline (dominant kernel, algorithmic bytes / its HIP-event time), cpu_baseline (the
CPU oracle on a bounded sample, rank 0 at N = 1), stages (per-stage device ms per step).
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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--k", type=int, default=21)
    ap.add_argument("--reads-per-gpu", type=int, default=10_000_000)
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--genome-per-gpu", type=int, default=50_000_000)
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--cpu-sample-reads", type=int, default=400_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--input", choices=("packed", "fastq"), default="packed",
                    help="packed: PackedRead bytes in HBM (the headline); fastq: FASTQ text in HBM, parsed and "
                         "packed on the device inside every step (mhmkc_add_fastq_device)")
    ap.add_argument("--no-profile-events", action="store_true")
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
        "exchange": st["bytes_sent"],
    }.get(stage, 0.0)


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


def cpu_baseline(b, o, k, n_reads):
    """The CPU oracle (oracle/kcount_oracle.c, single thread) on the first n_reads reads."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib as O

    n = min(n_reads, o.size - 1)
    bb, oo = b[: int(o[n])], o[: n + 1]
    t0 = time.perf_counter()
    t = O.kcount(bb, oo, k)
    dt = time.perf_counter() - t0
    occ = t.stats()["occurrences"]
    return {"value": occ / dt, "unit": "k-mers/s", "cores": 1, "kind": "port",
            "sample": f"first {n} reads of this rank's C2 shard ({occ} k-mers), oracle/kcount_oracle.c, 1 thread, "
                      f"{dt:.1f} s"}


def main():
    args = parse()
    import numpy as np
    import torch

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one rank per GPU)")
        world = args.gpus if world == 1 else world
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))

    import mhm2_proxy_amd as m

    k, L, R = args.k, args.read_len, args.reads_per_gpu
    G = args.genome_per_gpu * world
    threads = max(1, min(16, (os.cpu_count() or 8) // max(1, world)))
    t0 = time.perf_counter()
    genome = m.synth_genome(G, args.seed)
    b, o = m.synth_reads(genome, R, L, args.seed, first_read=rank * R, threads=threads)
    del genome
    gen_s = time.perf_counter() - t0
    dev = torch.device("cuda", local)
    if args.input == "fastq":
        text = fastq_text(b, o, L)
        tt = torch.from_numpy(text).to(dev)
        text_bytes = int(text.size)
        del text
    else:
        bt = torch.from_numpy(b).to(dev)
        ot = torch.from_numpy(o.view(np.int64)).to(dev)
    torch.cuda.synchronize()

    cid = None
    if world > 1:
        obj = [m.comm_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        cid = obj[0]
    counter = m.KmerCounter(k, device=local, rank=rank, n_ranks=world, comm_id=cid)
    counter.set_profiling(not args.no_profile_events)

    def step():
        counter.reset()
        if args.input == "fastq":
            counter.add_fastq_tensor(tt)
        else:
            counter.add_tensors(bt, ot)
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
    for _ in range(args.steps):
        step()
        st = counter.stats()
        occ_total += st["occurrences"]
        for s, v in st["ms_kernel"].items():
            stage_ms[s] = stage_ms.get(s, 0.0) + v
            launches[s] = launches.get(s, 0) + st["launches"][s]
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        c = torch.tensor([occ_total], dtype=torch.float64, device=dev)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        occ_total = int(c.item())

    value = occ_total / elapsed
    steps = max(1, args.steps)
    per_step = {s: v / steps for s, v in stage_ms.items()}
    dom = max((s for s in per_step if s not in ("other", "tileidx")), key=lambda s: per_step[s], default=None)
    roofline = None
    if dom and launches.get(dom):
        ms_launch = stage_ms[dom] / launches[dom]
        alg = algorithmic_bytes(dom, st, k) / max(1, launches[dom] // steps)
        achieved = alg / (ms_launch * 1e-3) / 1e9
        traffic = None
        pmc = Path(args.pmc_json)
        if pmc.exists():
            try:
                traffic = json.loads(pmc.read_text()).get("per_launch_bytes", {}).get(dom)
            except Exception:
                traffic = None
        roofline = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                    "algorithmic_bytes": int(alg), "avg_launch_ms": round(ms_launch, 4)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(b, o, k, args.cpu_sample_reads)

    if rank == 0:
        line = {
            "metric": f"k-mers/s (whole node), k={args.k} {args.read_len}bp reads",
            "value": round(value, 1),
            "unit": "k-mers/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (SURVEY.md §8(d) generator: splitmix64 genome + reads, 0.5% subst, 0.02% N, 2% Q10)",
            "config": {"workload": f"C2 per GPU: {R} x {L}bp synthetic reads/GPU, k={k}, genome {G} bp "
                                   f"(30x), seed {args.seed}", "k": k, "reads_per_gpu": R, "read_len": L,
                       "genome_len": G, "occurrences_per_step": occ_total // steps, "parallelism": f"hash-range x{world}"},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "stages_ms_per_step": {s: round(v, 3) for s, v in per_step.items()},
            "achieved_alg_GBps_whole_step": round(
                sum(algorithmic_bytes(s, st, k) for s in per_step) / (elapsed / steps) / 1e9, 1) if st else None,
            "survey_model": {
                "bytes_per_step_per_gpu": int(survey_model_bytes(st, k, R, L)),
                "GBps_per_gpu": round(survey_model_bytes(st, k, R, L) / (elapsed / steps) / 1e9, 1),
                "frac_of_hbm_peak": round(survey_model_bytes(st, k, R, L) / (elapsed / steps) / 1e9 / HBM_PEAK_GBPS, 4),
            } if st else None,
            "distinct_per_gpu": st["distinct"] if st else None,
            "n_out_per_gpu": st["n_out"] if st else None,
            "synth_seconds": round(gen_s, 2),
        }
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
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
