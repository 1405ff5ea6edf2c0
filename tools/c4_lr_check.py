"""The eight-rank C4 run of tests/test_multirank_gpu.py (8 ranks of 12.5M reads on one GPU, k = 63, supermer exchange,
4 finish passes) repeated, without the CPU comparison: after each run every rank's fetched table is checked for
left / right bytes outside get_ext's results (tests/mr_gpu_worker.lr_check), which is how the one-row C4 mismatch
showed (a row with its count right and left = right = 0). TEST TOOL.

  python tools/c4_lr_check.py [--runs 3] [--passes 4] [--k 63]
"""
import argparse
import socket
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--passes", type=int, default=4)
    ap.add_argument("--k", type=int, default=63)
    ap.add_argument("--reads-per-rank", type=int, default=12_500_000)
    a = ap.parse_args()
    import torch.multiprocessing as mp

    import mr_gpu_worker

    world = 8
    owner = "minimizer" if a.k >= 33 else "hash"
    tot_bad = 0
    for run in range(a.runs):
        t0 = time.time()
        with tempfile.TemporaryDirectory() as d:
            s = socket.socket()
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
            s.close()
            opts = {"reads_per_rank": a.reads_per_rank, "genome": 500_000_000, "seed": 3, "owner": owner,
                    "passes": a.passes, "n_parts": 8}
            mp.spawn(mr_gpu_worker.run_share_full, args=(world, port, a.k, d, opts), nprocs=world, join=True)
            for r in range(world):
                z = dict(np.load(Path(d) / f"rank{r}_lr.npz"))
                st = dict(np.load(Path(d) / f"rank{r}_stats.npz"))
                nb = int(z["bad_rows"].size)
                tot_bad += nb
                line = (f"run {run} rank {r}: {int(z['n_rows'])} rows, {nb} with bad left/right; count_sum - owned "
                        f"{int(st['count_sum']) - int(st['owned_records'])}")
                if nb:
                    line += (f"; rows {z['bad_rows'][:8].tolist()} first L/R {z['first_left'][:8].tolist()}/"
                             f"{z['first_right'][:8].tolist()} second {z['second_left'][:8].tolist()}/"
                             f"{z['second_right'][:8].tolist()} device {z['device_left'][:8].tolist()}/"
                             f"{z['device_right'][:8].tolist()}")
                print(line, flush=True)
        print(f"run {run}: {time.time() - t0:.1f} s", flush=True)
    print(f"{a.runs} runs: {tot_bad} rows with bad left/right in all", flush=True)


if __name__ == "__main__":
    main()
