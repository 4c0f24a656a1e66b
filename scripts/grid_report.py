#!/usr/bin/env python3
"""Per-(kernel, grid) breakdown of one training step from a rocprofv3 kernel trace: the same kernel name launched at
different shapes (a GEMM at each layer shape) is split by its grid, so per-shape rates can be read off.

    python scripts/grid_report.py <run>_kernel_trace.csv [--match gemm] [--step-marker adam_kernel]
"""
from __future__ import annotations

import argparse
import collections
import csv


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--match", default="", help="kernel-name substring to keep")
    ap.add_argument("--step-marker", default="sgd_kernel", help="kernel that ends a step")
    a = ap.parse_args(argv)
    rows = list(csv.DictReader(open(a.trace)))
    idx = [i for i, r in enumerate(rows) if a.step_marker in r["Kernel_Name"]]
    step = rows[idx[-2] + 1:idx[-1] + 1] if len(idx) >= 2 else rows
    gcols = [c for c in (step[0].keys() if step else []) if c.startswith("Grid_Size")]
    agg = collections.defaultdict(list)
    for r in step:
        if a.match not in r["Kernel_Name"]:
            continue
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        grid = "x".join(r[c] for c in gcols)
        agg[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    tot = sum(sum(v) for v in agg.values())
    print("step kernels matching %r: %.2f ms" % (a.match, tot / 1e3))
    for (name, grid), ts in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print("%8.2f ms  %4d x %8.1f us  grid %-16s %s" % (sum(ts) / 1e3, len(ts), sum(ts) / len(ts), grid, name[:100]))


if __name__ == "__main__":
    main()
