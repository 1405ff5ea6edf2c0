"""Multi-k back to back on one GPU (the read passes of BASELINE config C5, k in {21,33,55,77,99}).

C5 also runs the contig pass between rounds with contigs from dbjg traversal, which is out of scope here
(DESIGN.md §5). This tool times only the read passes, on the C2 synthetic reads. One counter per k stays
alive. Each step counts every k in turn from the same HBM-resident reads. Prints one JSON line.
  python tools/bench_multik.py [--ks 21,33,55,77,99] [--steps 3] [--warmup 1]
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ks", default="21,33,55,77,99")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--reads", type=int, default=10_000_000)
    args = ap.parse_args()
    import numpy as np
    import torch

    import mhm2_proxy_amd as m

    ks = [int(x) for x in args.ks.split(",")]
    g = m.synth_genome(50_000_000, 2)
    b, o = m.synth_reads(g, args.reads, 150, 2, threads=16)
    del g
    bt = torch.from_numpy(b).cuda()
    ot = torch.from_numpy(o.view(np.int64)).cuda()
    counters = {k: m.KmerCounter(k, device=0) for k in ks}
    for c in counters.values():
        c.set_profiling(True)

    per_k_ms = {k: 0.0 for k in ks}
    occ = {k: 0 for k in ks}

    def step(timed):
        for k in ks:
            c = counters[k]
            c.reset()
            c.add_tensors(bt, ot)
            c.finish()
            if timed:
                st = c.stats()
                per_k_ms[k] += st["ms_total"]
                occ[k] += st["occurrences"]

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    total = sum(occ.values())
    print(json.dumps({
        "metric": "k-mers/s, multi-k read passes back to back (C5 read passes, no contig pass), 1 GPU",
        "value": round(total / el, 1), "unit": "k-mers/s", "n_gpus": 1, "steps": args.steps,
        "ms_per_step": round(el / args.steps * 1e3, 3),
        "config": {"workload": f"{args.reads} x 150bp synthetic reads (C2 generator, seed 2), k in {ks}"},
        "per_k": {str(k): {"ms": round(per_k_ms[k] / args.steps, 3), "occurrences": occ[k] // args.steps,
                           "G_kmers_per_s": round(occ[k] / (per_k_ms[k] * 1e-3) / 1e9, 2)} for k in ks},
    }), flush=True)
    for c in counters.values():
        c.close()


if __name__ == "__main__":
    main()
