"""One step's device timeline from a rocprofv3 --kernel-trace [--memory-copy-trace] run: every kernel and copy of the
last bench step in start order, with the idle gap before it (where the device waited for the host).
  python tools/timeline.py <rocprof output dir> [first kernel name of a step, default k_tile_first_read]
"""
import csv
import glob
import sys


def rows(pattern):
    out = []
    for f in glob.glob(f"{sys.argv[1]}/**/{pattern}", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name") or r.get("Direction") or r.get("Operation") or "copy"
            out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    return out


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("mhm::", "")
    return ("rocprim " + n.split("detail::")[-1][:30]) if "rocprim" in n else n.split("(")[0][-48:]


ev = sorted(rows("*kernel_trace.csv") + rows("*memory_copy_trace.csv"))
first = sys.argv[2] if len(sys.argv) > 2 else "k_tile_first_read"
starts = [i for i, e in enumerate(ev) if first in e[2]]
if len(starts) < 2:
    sys.exit("fewer than two steps in the trace")
a, b = starts[-2], starts[-1]  # the last complete step
t0, prev_end, busy = ev[a][0], ev[a][0], 0
for s, e, n in ev[a:b]:
    gap = max(0, s - prev_end)
    print(f"{(s - t0) / 1e3:9.1f} us  gap {gap / 1e3:7.1f}  dur {(e - s) / 1e3:8.1f}  {short(n)}")
    busy += e - max(s, prev_end) if e > prev_end else 0
    prev_end = max(prev_end, e)
span = prev_end - t0
print(f"step span {span / 1e3:.1f} us, device busy {busy / 1e3:.1f} us, idle {(span - busy) / 1e3:.1f} us")
