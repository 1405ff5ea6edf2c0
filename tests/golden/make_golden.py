"""Regenerate the golden fixtures of tests/golden/ (run from the repo root: python tests/golden/make_golden.py).

Inputs are 'seq qual' lines (BASELINE.md's input format; qualities in Phred+33, capped at Q31 as
PackedRead stores them). Expected tables are produced by the CPU oracle (oracle/kcount_oracle.c, the
restatement of the reference kcount read pass pinned as described in DESIGN.md §2) and written in the
reference's dump_kmers line format "KMER count L R" (src/kcount/kmer_dht.cpp:243-266), sorted by k-mer.
"""
import gzip
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
sys.path.insert(0, str(HERE.parents[1]))

import numpy as np  # noqa: E402

import mhm2_proxy_amd as m  # noqa: E402
from common import edge_case_set, hot_set, oracle_table, synth_set  # noqa: E402

SETS = {
    "s100": (lambda: synth_set(2000, 10000, 100), [21, 33, 55, 63, 77, 99]),
    "edge": (lambda: edge_case_set(), [21, 33, 63]),
    "hot": (lambda: hot_set(), [21]),
}


def write_reads(path, b, o):
    with gzip.open(path, "wt", compresslevel=9) as f:
        for i in range(o.size - 1):
            r = b[int(o[i]):int(o[i + 1])]
            seq = "".join("ACGTN"[x & 7] for x in r)
            qual = "".join(chr(33 + (int(x) >> 3)) for x in r)
            f.write(f"{seq} {qual}\n")


def main():
    for name, (make, ks) in SETS.items():
        b, o = make()
        write_reads(HERE / f"reads_{name}.txt.gz", b, o)
        for k in ks:
            t = oracle_table(b, o, k).sorted()
            with gzip.open(HERE / f"table_{name}_k{k}.tsv.gz", "wt", compresslevel=9) as f:
                for line in t.lines():
                    f.write(line + "\n")
            print(name, k, len(t))


if __name__ == "__main__":
    main()
