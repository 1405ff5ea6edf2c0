"""Probe: which HIP runtime ends up in the process, and does torch + libmhmkc work in either load order."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
order = sys.argv[1]


def maps():
    return sorted({l.split()[-1] for l in open("/proc/self/maps") if "amdhip64" in l or "hsa-runtime" in l or "rccl" in l})


import numpy as np

if order == "torch_first":
    import torch
    print("torch devices", torch.cuda.device_count(), torch.cuda.is_available())
    x = torch.ones(4, device="cuda")
import mhm2_proxy_amd as m

g = m.synth_genome(5000, 1)
b, o = m.synth_reads(g, 200, 150, 1)
with m.KmerCounter(21) as c:
    c.add_packed_reads(b, o)
    print("n_out", c.finish())
if order == "lib_first":
    import torch
    print("torch devices", torch.cuda.device_count(), torch.cuda.is_available())
    x = torch.ones(4, device="cuda")
    print("torch ok", x.sum().item())
print("\n".join(maps()))
