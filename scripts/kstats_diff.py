"""Compare two rocprofv3 kernel_stats.csv files: per-kernel total time (ms per profiled run) A vs B.

    python scripts/kstats_diff.py A.csv B.csv [--top 30] [--steps N]
"""
import argparse
import csv
import re


def load(p):
    out = {}
    for r in csv.DictReader(open(p)):
        name = re.sub(r"\(.*", "", r["Name"])[:100]
        d = out.setdefault(name, [0.0, 0])
        d[0] += float(r["TotalDurationNs"]) / 1e6
        d[1] += int(r["Calls"])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("a")
    ap.add_argument("b")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--steps", type=float, default=1.0, help="divide totals by this (profiled steps)")
    x = ap.parse_args()
    A, B = load(x.a), load(x.b)
    keys = sorted(set(A) | set(B), key=lambda k: -abs(B.get(k, [0])[0] - A.get(k, [0])[0]))
    ta, tb = sum(v[0] for v in A.values()), sum(v[0] for v in B.values())
    print("total  A %.2f  B %.2f  diff %+.2f ms" % (ta / x.steps, tb / x.steps, (tb - ta) / x.steps))
    for k in keys[:x.top]:
        a, b = A.get(k, [0.0, 0]), B.get(k, [0.0, 0])
        print("%+8.2f  A %8.2f (%4d)  B %8.2f (%4d)  %s" % ((b[0] - a[0]) / x.steps, a[0] / x.steps, a[1], b[0] / x.steps,
                                                        b[1], k))


if __name__ == "__main__":
    main()
