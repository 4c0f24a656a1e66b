#!/usr/bin/env python3
"""Concurrency in a rocprofv3 kernel trace: per hardware queue (and stream) the busy time, and how long kernels of
two different queues actually ran at the same time.

    python scripts/trace_overlap.py <run>_kernel_trace.csv | <run>_results.db [--skip-first-ms 0]

Used for the weight-gradient side-stream experiment (ops/conv.py K8S_AMD_WGRAD_STREAM): if the side stream's
kernels never overlap the compute stream's, the two streams were serialised (same hardware queue, or the dispatcher
never co-schedules them) and any A/B difference is noise.
"""
from __future__ import annotations

import argparse
import csv
from collections import defaultdict


def union(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def inter_len(a, b):
    i = j = 0
    tot = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if e > s:
            tot += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--skip-first-ms", type=float, default=0.0, help="ignore kernels starting this early (warmup)")
    a = ap.parse_args(argv)
    if a.csv.endswith(".db"):  # rocprofv3's default rocpd (SQLite) output
        import sqlite3

        con = sqlite3.connect(a.csv)
        rows = [{"Kernel_Name": n, "Queue_Id": q, "Stream_Id": st, "Start_Timestamp": s, "End_Timestamp": e}
                for n, q, st, s, e in con.execute("select name, queue_id, stream_id, start, end from kernels")]
    else:
        rows = list(csv.DictReader(open(a.csv)))
    t0 = min(int(r["Start_Timestamp"]) for r in rows)
    by_q = defaultdict(list)
    names = defaultdict(lambda: defaultdict(float))
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if (s - t0) / 1e6 < a.skip_first_ms:
            continue
        key = "queue %s / stream %s" % (r.get("Queue_Id", "?"), r.get("Stream_Id", "?"))
        by_q[key].append((s, e))
        names[key][r["Kernel_Name"].split("(")[0][:70]] += (e - s) / 1e6
    keys = sorted(by_q, key=lambda k: -len(by_q[k]))
    unions = {k: union(by_q[k]) for k in keys}
    span = (max(e for k in keys for _, e in by_q[k]) - min(s for k in keys for s, _ in by_q[k])) / 1e6
    print("span %.2f ms" % span)
    for k in keys:
        busy = sum(e - s for s, e in unions[k]) / 1e6
        print("%-32s kernels %6d  busy %9.2f ms" % (k, len(by_q[k]), busy))
        for n, t in sorted(names[k].items(), key=lambda x: -x[1])[:4]:
            print("    %8.2f ms  %s" % (t, n))
    for i in range(len(keys)):
        for j in range(i + 1, len(keys)):
            ov = inter_len(unions[keys[i]], unions[keys[j]]) / 1e6
            print("overlap %s <-> %s: %.2f ms" % (keys[i], keys[j], ov))


if __name__ == "__main__":
    main()
