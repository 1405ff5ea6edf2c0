"""Per-launch HBM traffic of each stage from a PMC summary (tools/pmc_summary.py output) ->
profiles/pmc_traffic.json, which bench.py reports as roofline.traffic.

traffic = (FETCH_SIZE * 2 + WRITE_SIZE) * 1024 bytes per launch: rocprofv3 reports both in KiB, and on
gfx950 FETCH_SIZE counts half the bytes of wide streaming reads (MI355X_MICROARCH.md, HBM section); the
counts kernel's 8-byte loads match its algorithmic read volume under the same correction (within 0.2 %).
  python tools/pmc_traffic.py <tag> <config key, e.g. C2/k21>
Entries are kept per workload (bench.py reports one only for its own config and k).
"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
tag = sys.argv[1] if len(sys.argv) > 1 else "pmc"
key = sys.argv[2] if len(sys.argv) > 2 else "C2/k21"
summ = json.loads((ROOT / "gpurun_out" / f"{tag}_summary.json").read_text())
stage_of = {"k_extract_scatter": "extract_scatter", "k_extract_hist": "extract_hist", "k_part_scatter": "part_scatter",
            "k_part_hist": "part_hist", "k_count": "count"}
out, l2, valu = {}, {}, {}
N_SIMD, N_XCD = 256 * 4, 8  # MI355X: 256 CUs x 4 SIMDs; GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles
for kern, c in summ.items():
    base = kern.split("<")[0]
    if base in stage_of and "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        out[stage_of[base]] = int((c["FETCH_SIZE"] * 2 + c["WRITE_SIZE"]) * 1024)
    # VALU issue: a wave64 VALU instruction issues over 2 cycles on gfx950 (MI355X_MICROARCH.md), so
    # SQ_INSTS_VALU * 2 / N_SIMD is the cycles an average SIMD spent issuing VALU, against the kernel's cycles
    if base in stage_of and "SQ_INSTS_VALU" in c and "GRBM_GUI_ACTIVE" in c and c["GRBM_GUI_ACTIVE"] > 0:
        valu[stage_of[base]] = round(c["SQ_INSTS_VALU"] * 2 / N_SIMD / (c["GRBM_GUI_ACTIVE"] / N_XCD), 3)
    if base in stage_of and "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
        l2[stage_of[base]] = round(c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 3)
path = ROOT / "profiles" / "pmc_traffic.json"
doc = json.loads(path.read_text()) if path.exists() else {}
doc = {"formula": "(FETCH_SIZE*2 + WRITE_SIZE) * 1024", "configs": doc.get("configs", {})}
doc["configs"][key] = {"per_launch_bytes": out, "l2_hit": l2, "valu_issue_frac": valu,
                       "source": f"profiles/{tag}_summary.json"}
path.write_text(json.dumps(doc, indent=1) + "\n")
print(json.dumps(doc, indent=1))
