"""Summarise rocprofv3 --pmc CSVs per kernel (median over dispatches).

    python tools/pmc_summary.py gpurun_out/pmc [kernel-substring]
"""

from __future__ import annotations

import csv
import glob
import statistics
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "ginet_graph_kernel"
    vals = defaultdict(lambda: defaultdict(float))  # (pass, dispatch) -> counter -> value
    for path in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
        with open(path) as f:
            for row in csv.DictReader(f):
                if pat not in row["Kernel_Name"]:
                    continue
                key = (path, row["Dispatch_Id"])
                vals[key][row["Counter_Name"]] += float(row["Counter_Value"])
    per = defaultdict(list)
    for d in vals.values():
        for k, v in d.items():
            per[k].append(v)
    out = {k: statistics.median(v) for k, v in per.items()}
    for k in sorted(out):
        print(f"{k:28s} {out[k]:16.1f}   (n={len(per[k])})")
    return out


if __name__ == "__main__":
    main()
