"""Per-dispatch context of selected kernels in a rocprofv3 kernel trace: for every dispatch whose name matches
PATTERN, the dispatches around it (name, grid size, duration), so a stray fill / copy can be traced to its caller.

    python scripts/trace_context.py gpurun_out/prof_llama8b PATTERN [--before 3] [--after 2] [--max 40]
"""
import argparse
import csv
import glob
import os
import re


def load(d):
    path = d if d.endswith(".csv") else sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))[0]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return rows


def short(r):
    name = r["Kernel_Name"]
    name = re.sub(r"\(.*", "", name)[:90]
    grid = "x".join(r.get(k, "?") for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"))
    us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
    return "%-90s grid=%-16s %9.1f us" % (name, grid, us)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("pattern")
    ap.add_argument("--before", type=int, default=3)
    ap.add_argument("--after", type=int, default=2)
    ap.add_argument("--max", type=int, default=40)
    a = ap.parse_args()
    rows = load(a.trace)
    pat = re.compile(a.pattern)
    shown = 0
    for i, r in enumerate(rows):
        if not pat.search(r["Kernel_Name"]):
            continue
        print("---- dispatch %d" % i)
        for j in range(max(0, i - a.before), min(len(rows), i + a.after + 1)):
            print(("=> " if j == i else "   ") + short(rows[j]))
        shown += 1
        if shown >= a.max:
            break


if __name__ == "__main__":
    main()
