"""Per-kernel HBM traffic table from rocprofv3 --pmc passes (FETCH_SIZE and
WRITE_SIZE in separate passes) plus the kernel-trace stats of the same workload.

    python tools/pmc_per_kernel.py <pmc-dir> [<kernel_stats.csv>] [steps]

For each kernel name: median FETCH_SIZE / WRITE_SIZE per dispatch (KiB), the
gfx950-corrected HBM bytes per dispatch (MI355X_MICROARCH.md: FETCH_SIZE
counts half of wide coalesced reads, bytes = (2*FETCH + WRITE) * 1024), the
dispatches per step, and — with the stats CSV — the average duration and the
achieved traffic bandwidth.
"""

from __future__ import annotations

import csv
import glob
import re
import statistics
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    name = re.sub(r"\(.*$", "", name)  # drop the argument list
    return name.strip()


def main():
    root = sys.argv[1]
    stats = sys.argv[2] if len(sys.argv) > 2 else None
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [value per dispatch]
    for path in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
        disp = defaultdict(lambda: defaultdict(float))
        names = {}
        with open(path) as f:
            for row in csv.DictReader(f):
                key = row["Dispatch_Id"]
                names[key] = short(row["Kernel_Name"])
                disp[key][row["Counter_Name"]] += float(row["Counter_Value"])
        for key, d in disp.items():
            for c, v in d.items():
                per[names[key]][c].append(v)
    dur = {}
    if stats:
        with open(stats) as f:
            for row in csv.DictReader(f):
                dur[short(row["Name"])] = (float(row["AverageNs"]) / 1e3, int(row["Calls"]))
    print(f"{'kernel':60s} {'calls':>6s} {'avg_us':>8s} {'FETCH_KiB':>10s} {'WRITE_KiB':>10s} {'HBM_MB':>8s} {'GB/s':>7s}")
    tot_us = tot_mb = 0.0
    for k in sorted(per, key=lambda k: -dur.get(k, (0, 0))[0]):
        f = statistics.median(per[k]["FETCH_SIZE"]) if per[k]["FETCH_SIZE"] else float("nan")
        w = statistics.median(per[k]["WRITE_SIZE"]) if per[k]["WRITE_SIZE"] else float("nan")
        mb = (2 * f + w) * 1024 / 1e6
        us, calls = dur.get(k, (float("nan"), len(per[k]["FETCH_SIZE"])))
        gbs = mb * 1e6 / (us * 1e-6) / 1e9 if us == us else float("nan")
        print(f"{k[:60]:60s} {calls:6d} {us:8.2f} {f:10.1f} {w:10.1f} {mb:8.3f} {gbs:7.0f}")
        if steps and calls and us == us:
            tot_us += us * calls / steps
            tot_mb += mb * calls / steps
    if steps:
        print(f"per step: {tot_us:.1f} us of kernels, {tot_mb:.2f} MB of HBM traffic")
        # the graph pass's own kernels (model prefixes), without the optimizer and framework kernels
        pre = ("vb_", "vc_", "vanilla_", "ginet_", "fout_", "nc_")
        p_us = p_mb = 0.0
        for k in per:
            if not k.startswith(pre):
                continue
            f = statistics.median(per[k]["FETCH_SIZE"]) if per[k]["FETCH_SIZE"] else 0.0
            w = statistics.median(per[k]["WRITE_SIZE"]) if per[k]["WRITE_SIZE"] else 0.0
            us, calls = dur.get(k, (0.0, 0))
            p_us += us * calls / steps
            p_mb += (2 * f + w) * 1024 / 1e6 * calls / steps
        print(f"per step (graph pass kernels): {p_us:.1f} us, {p_mb:.3f} MB of HBM traffic")


if __name__ == "__main__":
    main()
