"""Print a rocprofv3 kernel_stats.csv (the directory a --stats run wrote) as name / calls / average ms."""
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:int(sys.argv[2]) if len(sys.argv) > 2 else 16]:
    n = r["Name"]
    n = n.replace("(anonymous namespace)::", "").replace("mhm::", "")
    n = ("rocprim " + n.split("detail::")[-1][:40]) if "rocprim" in n else n.split("(")[0][-70:]
    print(f"{n:72s} {r['Calls']:>5} {float(r['AverageNs']) / 1e6:8.3f}")
