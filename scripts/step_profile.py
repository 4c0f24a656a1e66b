#!/usr/bin/env python3
"""Per-step kernel breakdown of a rocprofv3 kernel trace: takes the dispatches between the last two
optimizer kernels (one training step) and lists time per kernel name.
    python scripts/step_profile.py gpurun_out/prof/run_kernel_trace.csv [--top 30] [--marker sgd_kernel]"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--marker", default=None, help="kernel-name substring that ends a step (default: optimizer)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    marker = a.marker
    if marker is None:
        marker = "adam_kernel" if any("adam_kernel" in r["Kernel_Name"] for r in rows) else "sgd_kernel"
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    step = rows[idx[-2] + 1:idx[-1] + 1]
    dur = lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"])  # noqa: E731
    tot = sum(dur(r) for r in step)
    ours = sum(dur(r) for r in step if "k8s_amd" in r["Kernel_Name"])
    wall = int(step[-1]["End_Timestamp"]) - int(step[0]["Start_Timestamp"])
    print("step: %d kernels, busy %.2f ms, wall %.2f ms, k8s_amd kernels %.1f%%" % (len(step), tot / 1e6, wall / 1e6,
                                                                                   100.0 * ours / tot))
    agg = collections.defaultdict(lambda: [0, 0])
    for r in step:
        n = r["Kernel_Name"].split("(")[0].replace("void ", "")[:90]
        agg[n][0] += dur(r)
        agg[n][1] += 1
    print("| ms | % | calls | kernel |\n|---:|---:|---:|---|")
    for n, (d, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:a.top]:
        print("| %.3f | %.1f | %d | `%s` |" % (d / 1e6, 100.0 * d / tot, c, n))


if __name__ == "__main__":
    main()
