"""Performance probe (not a test): the C2 reads at one k counted with forced fine bits (the test-only knob of
include/mhmkc_debug.h), to see where k_count's per-bucket overhead and its table load balance.
    python tools/fine_bits_probe.py K FB [FB ...]   -> one line per fine-bits value: stage ms (median of 5 finishes)
"""
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import mhm2_proxy_amd as m  # noqa: E402
from mhm2_proxy_amd import _native as N  # noqa: E402


def main():
    k = int(sys.argv[1])
    fbs = [int(x) for x in sys.argv[2:]] or [-1]
    g = m.synth_genome(50_000_000, 2)
    b, o = m.synth_reads(g, 10_000_000, 150, 2, threads=16)
    bt = torch.from_numpy(b).cuda()
    ot = torch.from_numpy(o.view(np.int64)).cuda()
    for fb in fbs:
        N.debug_reset()
        if fb >= 0:
            N.debug_set("fine_bits", fb)
        rows = []
        with m.KmerCounter(k, device=0) as c:
            c.set_profiling(True)
            for rep in range(6):
                c.reset()
                c.add_tensors(bt, ot)
                c.finish()
                st = c.stats()
                if rep:
                    rows.append((st["ms_total"], st["ms_kernel"], st["fine_buckets"], st["table_slots"],
                                 st["distinct"]))
        rows.sort(key=lambda r: r[0])
        ms, kern, nfb, slots, distinct = rows[len(rows) // 2]
        per = distinct / max(1, nfb)
        print(f"k={k} fine_bits={fb}: {ms:.2f} ms, stages { {s_: round(v, 2) for s_, v in kern.items() if v > 0.01} }, {nfb} fine buckets, {per:.0f} distinct per bucket "
              f"(load {per / slots:.2f})", flush=True)


if __name__ == "__main__":
    main()
