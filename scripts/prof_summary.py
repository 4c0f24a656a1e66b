#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats CSV directory into markdown (per-kernel time share).

    prof_summary.py DIR [OUT.md] [--steps N --marker SUBSTR]

With ``--steps N`` only the last N training steps of the kernel trace are counted: a step ends with the last
kernel whose name contains ``--marker`` (default ``sgd_kernel``, the optimizer), so warmup, autotuning and
vendor-library tuning kernels are excluded. Also reports the per-step GPU busy time and wall span.
"""
import argparse
import csv
import glob
import os
import sys
from collections import defaultdict


def _table(stats, tot, top):
    lines = ["| % time | total ms | calls | avg us | kernel |", "|---:|---:|---:|---:|---|"]
    for name, (t, n) in sorted(stats.items(), key=lambda kv: -kv[1][0])[:top]:
        lines.append("| %.2f | %.3f | %d | %.1f | `%s` |" % (100 * t / tot, t / 1e6, n, t / n / 1e3,
                                                          name.replace("|", "/")[:120]))
    return lines


def from_stats(d):
    f = sorted(glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True))
    if not f:
        sys.exit("no kernel_stats.csv under %s" % d)
    return {r["Name"]: (float(r["TotalDurationNs"]), int(r["Calls"])) for r in csv.DictReader(open(f[0]))}, ""


def from_trace(d, steps, marker):
    f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))
    if not f:
        sys.exit("no kernel_trace.csv under %s" % d)
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f[0]))]
    rows.sort()
    ends = [e for s, e, n in rows if marker in n]
    # one optimizer launch may be several kernels: collapse markers closer than 1 ms into one step boundary
    bounds = []
    for e in ends:
        if not bounds or e - bounds[-1] > 1_000_000:
            bounds.append(e)
        else:
            bounds[-1] = e
    if len(bounds) < steps + 1:
        sys.exit("trace has %d step boundaries (marker %r), need %d" % (len(bounds), marker, steps + 1))
    lo, hi = bounds[-steps - 1], bounds[-1]
    stats = defaultdict(lambda: [0.0, 0])
    busy = 0
    for s, e, n in rows:
        if lo < s <= hi:
            stats[n][0] += e - s
            stats[n][1] += 1
            busy += e - s
    note = "Window: last %d steps (step boundary = end of `%s`): %.3f ms/step wall, %.3f ms/step summed kernel time\n\n" % (
        steps, marker, (hi - lo) / 1e6 / steps, busy / 1e6 / steps)
    return {k: tuple(v) for k, v in stats.items()}, note


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("out", nargs="?")
    ap.add_argument("--steps", type=int, default=0)
    ap.add_argument("--marker", default="sgd_kernel")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args(argv)
    stats, note = from_trace(a.dir, a.steps, a.marker) if a.steps else from_stats(a.dir)
    tot = sum(t for t, _ in stats.values())
    own = sum(t for n, (t, _) in stats.items() if "k8s_amd" in n)
    head = note + "Total GPU kernel time %.3f ms over %d kernel names; k8s_amd HIP kernels: %.1f%%\n\n" % (
        tot / 1e6, len(stats), 100 * own / tot)
    text = head + "\n".join(_table(stats, tot, a.top)) + "\n"
    if a.out:
        open(a.out, "w").write(text)
    print(text)


if __name__ == "__main__":
    main()
