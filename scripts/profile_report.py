"""Markdown summary of a rocprofv3 kernel_stats.csv (+ optional per-layer roofline JSONL) for profiles/.

    python scripts/profile_report.py STATS.csv --steps 6 [--roofline roofline.jsonl] [--title ...] > profiles/x.md
    python scripts/profile_report.py TRACE_kernel_trace.csv --step-marker adam_kernel ...   (steady state only)

With ``--step-marker`` the input is a kernel TRACE and only the dispatches between the first and the last
dispatch matching the marker (one optimizer launch per step) are counted: start-up work (weight init fills,
first-step copies) stays out of the per-step numbers.

Kernels are grouped into categories (BatchNorm, conv/GEMM forward+dgrad, weight gradient, pooling, optimizer,
vendor/ATen) so the step-time split is visible at a glance; ``k8s_amd::`` share = GPU time in our kernels.
"""
import argparse
import csv
import json
import re

CATS = [
    ("BatchNorm", r"k8s_amd::bn_|relu_mask|pool_bn_bwd"),
    ("weight gradient", r"wgrad_stream|ConvWgB|MNMajorK, k8s_amd::MNMajorK|MNMaj, k8s_amd::g256r::MNMaj|gemm_w4_kernel<true, true>|splitk_reduce|"
                        r"wgrad3x3|wg3_reduce|stem_wgrad|stem_dw"),
    ("conv / GEMM fwd + dgrad", r"gemm_bf16_kernel|gemm256|gemm_w4|gemm_short_kernel|conv3x3_kernel|conv_dgrad_wtrans|stem_conv_fwd|stem_w_s2d"),
    ("pooling", r"pool"),
    ("optimizer / loss", r"sgd_|adam_|xent|sumsq|clip"),
    ("attention / norms / elementwise", r"flash_|norm_|swiglu|rope|gelu|relu_bwd|colsum"),
]


def categorize(name):
    if not name.startswith(("void k8s_amd::", "k8s_amd::")):
        return "vendor / ATen / runtime"
    for cat, pat in CATS:
        if re.search(pat, name):
            return cat
    return "other k8s_amd"


def steady_rows(trace, marker):
    """kernel_stats-shaped rows from the dispatches between the first and last step-marker dispatch."""
    disp = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(disp) if re.search(marker, r["Kernel_Name"])]
    if len(idx) < 2:
        raise SystemExit("need >= 2 dispatches matching %r (found %d)" % (marker, len(idx)))
    agg = {}
    for r in disp[idx[0] + 1:idx[-1] + 1]:
        d = agg.setdefault(r["Kernel_Name"], [0, 0.0])
        d[0] += 1
        d[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    rows = [{"Name": n, "Calls": c, "TotalDurationNs": t, "AverageNs": t / c} for n, (c, t) in agg.items()]
    return rows, float(len(idx) - 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats")
    ap.add_argument("--steps", type=float, help="profiled steps (warmup + timed) in the trace")
    ap.add_argument("--step-marker", help="regex of the one-per-step kernel; input is then a kernel_trace.csv")
    ap.add_argument("--roofline")
    ap.add_argument("--title", default="Kernel profile")
    ap.add_argument("--top", type=int, default=20)
    a = ap.parse_args()
    if a.step_marker:
        rows, a.steps = steady_rows(a.stats, a.step_marker)
    else:
        if a.steps is None:
            ap.error("--steps is required with a kernel_stats.csv")
        rows = list(csv.DictReader(open(a.stats)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    ours = sum(float(r["TotalDurationNs"]) for r in rows if r["Name"].startswith(("void k8s_amd::", "k8s_amd::")))
    print("# %s\n" % a.title)
    print("GPU time per step: **%.2f ms** (%d kernel names, %.0f profiled steps); `k8s_amd::` kernels: **%.1f %%**.\n"
          % (tot / a.steps / 1e6, len(rows), a.steps, 100 * ours / tot))
    cats = {}
    for r in rows:
        c = categorize(r["Name"])
        cats[c] = cats.get(c, 0.0) + float(r["TotalDurationNs"])
    print("| category | ms / step | share |\n|---|---:|---:|")
    for c, v in sorted(cats.items(), key=lambda kv: -kv[1]):
        print("| %s | %.2f | %.1f %% |" % (c, v / a.steps / 1e6, 100 * v / tot))
    print("\n## Top %d kernels\n" % a.top)
    print("| kernel | calls / step | avg us | ms / step | share |\n|---|---:|---:|---:|---:|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:a.top]:
        name = re.sub(r"\(.*", "", r["Name"]).replace("void ", "").replace("|", "/")[:110]
        print("| `%s` | %.1f | %.1f | %.2f | %.1f %% |" % (name, int(r["Calls"]) / a.steps, float(r["AverageNs"]) / 1e3,
                                                        float(r["TotalDurationNs"]) / a.steps / 1e6,
                                                        100 * float(r["TotalDurationNs"]) / tot))
    if a.roofline:
        lines = [json.loads(l) for l in open(a.roofline) if l.strip().startswith("{")]
        layers = [l for l in lines if "layer" in l]
        summ = [l for l in lines if "summary_ms_per_step" in l]
        print("\n## Per-layer roofline (`scripts/layer_roofline.py`, isolated launches)\n")
        if summ:
            print("Sum per step: %s (total %.2f ms).\n" % (", ".join("%s %.2f ms" % kv for kv in
                                                                      summ[0]["summary_ms_per_step"].items()),
                                                          summ[0]["total_ms"]))
        print("| layer | op | count | ms | ms / step | TFLOP/s or TB/s |\n|---|---|---:|---:|---:|---:|")
        for l in sorted(layers, key=lambda l: -l["step_ms"])[:30]:
            rate = ("%.0f TF/s" % l["tflops"]) if "tflops" in l else ("%.2f TB/s" % l["tbps"])
            print("| %s | %s | %d | %.3f | %.3f | %s |" % (l["layer"], l["op"], l["count"], l["ms"], l["step_ms"], rate))


if __name__ == "__main__":
    main()
