"""Print the counter statistics of one C2 counting round (diagnostics for performance work)."""
import sys, json
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np, torch
import mhm2_proxy_amd as m
g = m.synth_genome(50_000_000, 2)
b, o = m.synth_reads(g, 10_000_000, 150, 2, threads=16)
bt = torch.from_numpy(b).cuda(); ot = torch.from_numpy(o.view(np.int64)).cuda()
c = m.KmerCounter(21, device=0)
c.set_profiling(True)
for _ in range(2):
    c.reset(); c.add_tensors(bt, ot); c.finish()
st = c.stats()
print(json.dumps({k: v for k, v in st.items() if k not in ("launches",)}, default=str))
