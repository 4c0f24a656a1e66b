#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats CSV directory into markdown (per-kernel time share)."""
import csv
import glob
import os
import sys


def main(d, top=40, out=None):
    f = sorted(glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True))
    if not f:
        sys.exit("no kernel_stats.csv under %s" % d)
    rows = list(csv.DictReader(open(f[0])))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    lines = ["| % time | total ms | calls | avg us | kernel |", "|---:|---:|---:|---:|---|"]
    own = 0.0
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        t = float(r["TotalDurationNs"])
        if "k8s_amd" in r["Name"]:
            own += t
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        t = float(r["TotalDurationNs"])
        name = r["Name"].replace("|", "/")[:120]
        lines.append("| %.2f | %.3f | %s | %.1f | `%s` |" % (100 * t / tot, t / 1e6, r["Calls"], float(r["AverageNs"]) / 1e3, name))
    head = "Total GPU kernel time %.3f ms over %d kernel names; k8s_amd HIP kernels: %.1f%%\n\n" % (
        tot / 1e6, len(rows), 100 * own / tot)
    text = head + "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(text)
    print(text)


if __name__ == "__main__":
    main(sys.argv[1], out=sys.argv[2] if len(sys.argv) > 2 else None)
