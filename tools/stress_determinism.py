"""Run-to-run determinism of the whole count (TEST TOOL): the same reads counted again and again by one KmerCounter on
cuda:0, each run's table reduced to an order-independent digest of its row fingerprints (row count, sum, xor). A
table differing from the first run's in any row changes the digest; the differing rows (key words, count, left,
right of both runs) are printed. Used to find the C4 one-row mismatch ("the two-word claim race").

  python tools/stress_determinism.py --k 63 --iters 30 [--passes 4] [--reads 10000000]
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def digest(fps):
    return int(fps.size), int(np.bitwise_xor.reduce(fps)), int(fps.sum(dtype=np.uint64))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=63)
    ap.add_argument("--reads", type=int, default=10_000_000)
    ap.add_argument("--genome", type=int, default=50_000_000)
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--passes", type=int, default=0)
    ap.add_argument("--seconds", type=float, default=0, help="stop after this many seconds")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    if a.passes:
        os.environ["MHMKC_PASSES"] = str(a.passes)
    import torch

    import mhm2_proxy_amd as m
    import oracle_lib as O

    t0 = time.time()
    g = m.synth_genome(a.genome, a.seed)
    b, o = m.synth_reads(g, a.reads, 150, a.seed, threads=16)
    del g
    bt = torch.from_numpy(b).cuda()
    ot = torch.from_numpy(o.view(np.int64)).cuda()
    n_bases = int(o[-1])
    del b, o
    c = m.KmerCounter(a.k, device=0)
    ref = None
    res = []
    for it in range(a.iters):
        c.reset()
        c.add_tensors(bt, ot, n_bases=n_bases)
        c.finish()
        t = c.fetch()
        st = c.stats()
        fps = O.row_fingerprints(t.keys, t.counts, t.left, t.right, a.k)
        d = digest(fps)
        rec = {"iter": it, "rows": d[0], "xor": d[1], "sum": d[2], "distinct": int(st["distinct"]),
               "count_sum": int(st["count_sum"]), "occurrences": int(st["occurrences"]),
               "finish_passes": int(st["finish_passes"]), "sweeps": int(st["overflow_sweeps"]),
               "misses": int(st["lds_misses"])}
        res.append(rec)
        same = ref is None or d == ref[0]
        print(f"[{time.time() - t0:6.1f}s] iter {it}: rows {d[0]} distinct {rec['distinct']} count_sum-occ "
              f"{rec['count_sum'] - rec['occurrences']} sweeps {rec['sweeps']} {'same' if same else 'DIFFERS'}",
              flush=True)
        if ref is None:
            ref = (d, np.sort(fps), t)
        elif not same:
            s = np.sort(fps)
            only_now, only_ref = np.setdiff1d(s, ref[1]), np.setdiff1d(ref[1], s)
            print(f"  {only_now.size} rows only in this run, {only_ref.size} only in run 0", flush=True)
            for name, tab, fp_all, bad in (("now", t, fps, only_now[:8]),
                                           ("run0", ref[2], None, only_ref[:8])):
                fa = fp_all if fp_all is not None else O.row_fingerprints(tab.keys, tab.counts, tab.left, tab.right,
                                                                           a.k)
                for i in np.flatnonzero(np.isin(fa, bad)):
                    print(f"  {name}: key {[hex(int(x)) for x in tab.keys[i]]} count {int(tab.counts[i])} "
                          f"L {chr(int(tab.left[i]))} R {chr(int(tab.right[i]))}", flush=True)
            rec["only_now"], rec["only_ref"] = int(only_now.size), int(only_ref.size)
        if a.seconds and time.time() - t0 > a.seconds:
            break
    c.close()
    bad = sum(1 for r in res if (r["rows"], r["xor"], r["sum"]) != ref[0])
    print(f"{len(res)} runs, {bad} differ from run 0", flush=True)
    if a.out:
        Path(a.out).write_text(json.dumps({"args": vars(a), "runs": res, "differing": bad}, indent=1))


if __name__ == "__main__":
    main()
