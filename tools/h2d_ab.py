"""Performance probe (not a test): the C2 reads counted from pinned host memory (mhmkc_add_reads, the bench's
h2d_inclusive window) with the bases sent as bytes (h2d_nib 0) and as nibbles with u32 (1) or u64 (2) offsets, interleaved in one process:
per mode the median window (reset + add + finish, synchronised), the copy stream's span and bytes, and the output rows
and count sum (which must agree).
    python tools/h2d_ab.py [K] [steps]
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
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 21
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    g = m.synth_genome(50_000_000, 2)
    b, o = m.synth_reads(g, 10_000_000, 150, 2, threads=16)
    hb = torch.from_numpy(b).pin_memory().numpy()
    ho = torch.from_numpy(o.view(np.int64)).pin_memory().numpy().view(np.uint64)
    res = {0: [], 1: [], 2: []}
    ref = None
    with m.KmerCounter(k, device=0) as c:
        for rep in range(steps + 2):
            for nib in (0, 1, 2):
                N.debug_set("h2d_nib", nib)
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
                assert sig == ref, (nib, sig, ref)
                if rep >= 2:
                    res[nib].append((dt, st["ms_h2d"], st["h2d_bytes"], st["h2d_chunks"], st["ms_h2d_pack"],
                                     st["ms_h2d_wait"]))
    N.debug_reset()
    for nib, rows in res.items():
        rows.sort()
        dt, h2d, hb_, ch, pk, wt = rows[len(rows) // 2]
        print(f"k={k} h2d_nib={nib}: window {dt:.2f} ms (min {rows[0][0]:.2f})  copy span {h2d:.2f} ms  "
              f"{hb_ / 1e9:.3f} GB in {ch} chunks  ({hb_ / h2d / 1e6:.1f} GB/s)  host packing {pk:.2f} ms, "
              f"slot waits {wt:.2f} ms  n_out={ref[0]}", flush=True)


if __name__ == "__main__":
    main()
