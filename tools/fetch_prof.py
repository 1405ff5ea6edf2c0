"""Time mhmkc_fetch / mhmkc_fetch_ordered on the C2 table (run under rocprofv3 --kernel-trace --stats for the kernels)."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mhm2_proxy_amd as m  # noqa: E402

g = m.synth_genome(50_000_000, 2)
b, o = m.synth_reads(g, 10_000_000, 150, 2)
bt = torch.from_numpy(b).cuda()
ot = torch.from_numpy(o.view(np.int64)).cuda()
with m.KmerCounter(21, device=0) as c:
    c.add_tensors(bt, ot)
    c.finish()
    torch.cuda.synchronize()
    for what in ("plain", "ordered", "ordered", "plain"):
        t0 = time.perf_counter()
        t = c.fetch(ordered=what == "ordered")
        print(what, round((time.perf_counter() - t0) * 1e3, 2), "ms", len(t), flush=True)
