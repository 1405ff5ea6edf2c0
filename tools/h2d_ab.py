"""Performance probe (not a test): the C2 reads counted from pinned host memory (mhmkc_add_reads, the bench's
h2d_inclusive window) under test-only knobs (include/mhmkc_debug.h), the configurations interleaved in one process:
per configuration the median window (reset + add + finish, synchronised), the copy stream's span and bytes, the host
packing and slot-wait times, the rounds fine-partitioned as they landed, and the output (which must agree).
    python tools/h2d_ab.py K STEPS "h2d_nib=0" "h2d_nib=1" "h2d_nib=1,h2d_threads=8" "h2d_nib=1,local_rounds=0" ...
(every configuration has its own counter, created with its knobs set: local_rounds is read at creation)
"""
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import mhm2_proxy_amd as m  # noqa: E402
from mhm2_proxy_amd import _native as N  # noqa: E402


def knobs(cfg):
    N.debug_reset()
    for kv in filter(None, cfg.split(",")):
        key, val = kv.split("=")
        N.debug_set(key, int(val))


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 21
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    cfgs = sys.argv[3:] or ["h2d_nib=0", "h2d_nib=1"]
    g = m.synth_genome(50_000_000, 2)
    b, o = m.synth_reads(g, 10_000_000, 150, 2, threads=16)
    hb = torch.from_numpy(b).pin_memory().numpy()
    ho = torch.from_numpy(o.view(np.int64)).pin_memory().numpy().view(np.uint64)
    counters = {}
    for cfg in cfgs:
        knobs(cfg)
        counters[cfg] = m.KmerCounter(k, device=0)
    res = {cfg: [] for cfg in cfgs}
    ref = None
    for rep in range(steps + 2):
        for cfg in cfgs:
            knobs(cfg)
            c = counters[cfg]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            c.reset()
            c.add_packed_reads(hb, ho)
            c.finish()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) * 1e3
            st = c.stats()
            sig = (st["n_out"], st["count_sum"], st["distinct"])
            if ref is None:
                ref = sig
            assert sig == ref, (cfg, sig, ref)
            if rep >= 2:
                res[cfg].append((dt, st["ms_h2d"], st["h2d_bytes"], st["h2d_chunks"], st["ms_h2d_pack"],
                                 st["ms_h2d_wait"], st["inc_rounds"], st["ms_finish_tail"], st["ms_h2d_rounds"], st["h2d_raw_chunks"]))
    N.debug_reset()
    for cfg, rows in res.items():
        rows.sort()
        dt, h2d, hb_, ch, pk, wt, ir, tail, rms, raw = rows[len(rows) // 2]
        print(f"k={k} [{cfg}]: window {dt:.2f} ms (min {rows[0][0]:.2f})  copy span {h2d:.2f} ms  "
              f"{hb_ / 1e9:.3f} GB in {ch} chunks, {raw} raw ({hb_ / h2d / 1e6:.1f} GB/s)  host packing {pk:.2f} ms  "
              f"slot waits {wt:.2f} ms  rounds partitioned as they landed {ir} (host {rms:.2f} ms)  "
              f"finish tail {tail:.2f} ms  "
              f"n_out={ref[0]}", flush=True)
    for c in counters.values():
        c.close()


if __name__ == "__main__":
    main()
