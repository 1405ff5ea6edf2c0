"""Per-kernel PMC digest of tools/pmc_summary.py output: traffic (FETCH_SIZE*2 + WRITE_SIZE, KiB -> GB), L2 hit,
instruction mix and wait ratios, for the kcount kernels.   python tools/pmc_report.py <tag> [...]"""
import json
import sys

for tag in sys.argv[1:]:
    d = json.load(open(f"gpurun_out/{tag}_summary.json"))
    for k, v in d.items():
        if not k.startswith(("k_", "void k_")) and "k_" not in k[:12]:
            continue
        f, w = v.get("FETCH_SIZE", 0) * 2 * 1024 / 1e9, v.get("WRITE_SIZE", 0) * 1024 / 1e9
        if f + w < 0.05:
            continue
        hit = v.get("TCC_HIT_sum", 0) / max(1, v.get("TCC_HIT_sum", 0) + v.get("TCC_MISS_sum", 0))
        wc = max(1, v.get("SQ_WAVE_CYCLES", 1))
        print(f"{tag:14s} {k[:34]:34s} read {f:6.2f} write {w:6.2f} GB  L2hit {hit:.3f}  VALU {v.get('SQ_INSTS_VALU', 0):.3g} "
              f"SALU {v.get('SQ_INSTS_SALU', 0):.3g} LDS {v.get('SQ_INSTS_LDS', 0):.3g}  wait/wave {v.get('SQ_WAIT_ANY', 0) / wc:.2f} "
              f"bank/lds {v.get('SQ_LDS_BANK_CONFLICT', 0) / max(1, v.get('SQ_ACTIVE_INST_LDS', 1)):.2f}")
