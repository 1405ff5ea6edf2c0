"""Summarise rocprofv3 --pmc passes (gpurun_out/<tag>/p*/run_counter_collection.csv) per kernel."""
import collections
import csv
import glob
import json
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "pmc"
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(lambda: collections.defaultdict(set))
for f in sorted(glob.glob(f"gpurun_out/{tag}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("mhm::", "")
        if name.startswith("__amd"):
            continue
        agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[name][r["Counter_Name"]].add(r["Dispatch_Id"])
out = {}
for name, d in agg.items():
    out[name] = {c: v / max(1, len(disp[name][c])) for c, v in d.items()}
json.dump(out, open(f"gpurun_out/{tag}_summary.json", "w"), indent=1)
for name, d in out.items():
    print(name)
    for c, v in sorted(d.items()):
        print(f"   {c:36s} {v:.4g}")
