"""Performance probe (not a test): the C2 reads at one k counted with test-only knobs set (include/mhmkc_debug.h),
one configuration after the other in one process, so that they share the box: per configuration the median step and
stage times of 7 steps (2 warm-ups), the fine buckets and the output rows (which must agree).
    python tools/knob_ab.py K "" "cb0_2=9" "cb0_2=9,fine_bits=9" ...   ("" = the defaults)
"""
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import mhm2_proxy_amd as m  # noqa: E402
from mhm2_proxy_amd import _native as N  # noqa: E402


def main():
    k = int(sys.argv[1])
    cfgs = sys.argv[2:] or [""]
    g = m.synth_genome(50_000_000, 2)
    b, o = m.synth_reads(g, 10_000_000, 150, 2, threads=16)
    bt = torch.from_numpy(b).cuda()
    ot = torch.from_numpy(o.view(np.int64)).cuda()
    n_bases = int(o[-1])
    for rnd in range(2):  # every configuration twice, interleaved (drift on a shared box)
        for cfg in cfgs:
            N.debug_reset()
            for kv in filter(None, cfg.split(",")):
                key, val = kv.split("=")
                N.debug_set(key, int(val))
            rows = []
            with m.KmerCounter(k, device=0) as c:
                c.set_profiling(2)
                for rep in range(9):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    c.reset()
                    c.add_tensors(bt, ot, n_bases=n_bases)
                    c.finish()
                    torch.cuda.synchronize()
                    dt = (time.perf_counter() - t0) * 1e3
                    st = c.stats()
                    if rep >= 2:
                        rows.append((dt, st["ms_kernel"], st["fine_buckets"], st["n_out"]))
            rows.sort(key=lambda r: r[0])
            dt, kern, nfb, n_out = rows[len(rows) // 2]
            ks = " ".join(f"{s_}={v:.3f}" for s_, v in kern.items() if v)
            print(f"round {rnd} k={k} [{cfg or 'defaults'}]: step {dt:.3f} ms  {ks}  fine_buckets={nfb} n_out={n_out}",
                  flush=True)
    N.debug_reset()


if __name__ == "__main__":
    main()
