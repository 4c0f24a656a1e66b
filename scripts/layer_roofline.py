"""Per-layer roofline of one ResNet-50 training step on our kernels.

Times every unique conv (fwd with the BN-statistics epilogue, weight gradient, data gradient) and every
BatchNorm (forward apply, backward reduce + apply) of ResNet-50 v1.5 at the bench batch, multiplies by how
often the shape occurs per step, and prints one JSON line per (layer, op) with the achieved TFLOP/s (convs) or
TB/s of compulsory HBM traffic (BN), then a summary line. Shapes and dispatch are exactly the trainer's
(``ops/conv.py``, ``ops/nn.py``): the stem is the space-to-depth 4x4 kernel pair of ``stem.hip``, the conv3 layers
of stages 1-2 read their input normalised on load (BN2, ``nn._BnReluConv``: forward and weight gradient with
``xform``; ``nn.ONLOAD_MAXC``), and the identity blocks' conv1 data gradient adds the masked residual gradient in its
epilogue (``nn.MaskedGrad``) -- counted in that row's floor bytes.

    python scripts/layer_roofline.py [--batch 1024] [--reps 5]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_amd.ops import conv  # noqa: E402
from k8s_amd.ops._ext import load  # noqa: E402


def resnet50_layers():
    """[(name, H_in, C_in, K_out, R, stride, count, bn_kind)] per step; bn_kind: relu | res | plain."""
    L = [("stem", 224, 8, 64, 7, 2, 1, "relu")]
    cin = 64
    H = 56
    for si, (nb, w) in enumerate([(3, 64), (4, 128), (6, 256), (3, 512)]):
        s = 1 if si == 0 else 2
        out = 4 * w
        L.append(("s%d.b0.conv1" % si, H, cin, w, 1, 1, 1, "relu"))
        L.append(("s%d.b0.conv2" % si, H, w, w, 3, s, 1, "relu"))
        Ho = H // s
        L.append(("s%d.b0.conv3" % si, Ho, w, out, 1, 1, 1, "res"))
        L.append(("s%d.b0.down" % si, H, cin, out, 1, s, 1, "plain"))
        if nb > 1:
            L.append(("s%d.bx.conv1" % si, Ho, out, w, 1, 1, nb - 1, "relu"))
            L.append(("s%d.bx.conv2" % si, Ho, w, w, 3, 1, nb - 1, "relu"))
            L.append(("s%d.bx.conv3" % si, Ho, w, out, 1, 1, nb - 1, "res"))
        cin, H = out, Ho
    return L


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", default="", help="comma list of ops to time: fwd,wgrad,dgrad,bnf,bnb")
    a = ap.parse_args()
    only = set(a.only.split(",")) if a.only else {"fwd", "wgrad", "dgrad", "bnf", "bnb"}
    C_ = load()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    N = a.batch
    tot = {}
    rows = []
    for (name, H, C, K, R, s, cnt, bnk) in resnet50_layers():
        pad = R // 2
        Ho = (H + 2 * pad - R) // s + 1
        x = torch.randn(N, H, H, C, device=dev, dtype=torch.bfloat16)
        w = (torch.randn(K, R, R, C, device=dev) * (2.0 / (R * R * C)) ** 0.5).bfloat16()
        gy = torch.randn(N, Ho, Ho, K, device=dev, dtype=torch.bfloat16)
        flops = 2.0 * N * Ho * Ho * K * C * R * R
        M = N * Ho * Ho
        res = {}
        # the bench's operand paths (module docstring)
        xf = None
        from k8s_amd.ops import nn as K_nn

        if name.endswith("conv3") and C <= K_nn.ONLOAD_MAXC:  # bn2 on load only up to ONLOAD_MAXC channels (round 6)
            xf = torch.cat([torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1]).contiguous()
        addend = None
        if name.endswith("bx.conv1"):
            from k8s_amd.ops import nn as K_

            addend = K_.MaskedGrad(torch.randn(N, H, H, C, device=dev, dtype=torch.bfloat16),
                                   torch.randint(0, 256, (N * H * H * C // 8,), device=dev, dtype=torch.uint8))
        if name == "stem":
            img = torch.randn(N, 224, 224, 8, device=dev, dtype=torch.bfloat16)
            xs = C_.stem_s2d_input(img, 3)
            w4 = C_.stem_w_s2d(w)
        if "fwd" in only:
            st = torch.zeros(C_.conv_stat_replicas, 2, K, device=dev)
            if name == "stem":
                res["fwd"] = timed(lambda: C_.stem_conv_fwd(xs, w4, st), a.reps)
            else:
                res["fwd"] = timed(lambda: C_.conv_fwd(x, w, s, pad, 1, False, None, 0, st, xform=xf), a.reps)
        if "wgrad" in only:
            dw = torch.empty(K, R, R, C, device=dev)
            if name == "stem":
                dw4 = torch.empty(tuple(w4.shape), device=dev)
                res["wgrad"] = timed(lambda: (C_.stem_wgrad(xs, gy, dw4), C_.stem_dw_s2d(dw4, dw)), a.reps)
            else:
                res["wgrad"] = timed(lambda: conv._wgrad_hip(C_, gy, x, dw, s, pad, False, xf), a.reps)
        if "dgrad" in only and name != "stem":
            if s == 1:
                res["dgrad"] = timed(lambda: conv._dgrad_hip(C_, gy, w, pad, addend), a.reps)
            else:
                res["dgrad"] = timed(lambda: conv._dgrad_strided_hip(C_, gy, w, s, pad, H, H), a.reps)
        # compulsory HBM bytes per op (bf16 activations, fp32 weight gradient) and the speed-of-light floor
        # max(bytes / 8 TB/s, flops / 2.5 PF/s): "sol" = floor / measured.
        xb, yb, wb = N * H * H * C * 2, M * K * 2, K * R * R * C * 2
        # fused operands each form really moves (round 6): the identity blocks' conv1 data
        # gradient also reads the masked residual addend (bf16, dx's shape) and its packed ReLU bits (1 bit / element);
        # the normalize-on-load forms read the same bytes as the plain ones; the statistics outputs are [R][2][K]
        dg_extra = (xb + xb // 16) if addend is not None else 0
        nb = {"fwd": xb + yb + wb, "wgrad": xb + yb + 2 * wb, "dgrad": yb + xb + wb + dg_extra}
        for op in ("fwd", "wgrad", "dgrad"):
            if op in res:
                floor = max(nb[op] / 8e9, flops / 2.5e12)
                rows.append({"layer": name, "op": op, "count": cnt, "batch": N, "ms": round(res[op], 4),
                             "gbytes": round(nb[op] / 1e9, 3), "onload": bool(xf is not None and op != "dgrad"),
                             "step_ms": round(res[op] * cnt, 3), "tflops": round(flops / res[op] / 1e9, 1),
                             "floor_ms": round(floor, 4), "sol": round(floor / res[op], 2),
                             "lost_ms_per_step": round((res[op] - floor) * cnt, 3)})
                tot[op] = tot.get(op, 0.0) + res[op] * cnt
        # BatchNorm of this conv's output y [M, K]
        y = gy
        g = torch.ones(K, device=dev)
        b = torch.zeros(K, device=dev)
        rm, rv = torch.zeros(K, device=dev), torch.ones(K, device=dev)
        sums = torch.zeros(C_.conv_stat_replicas, 2, K, device=dev)
        sums[0, 0] = y.float().sum((0, 1, 2))
        sums[0, 1] = (y.float() ** 2).sum((0, 1, 2))
        resid = torch.randn_like(y) if bnk == "res" else None
        relu = bnk != "plain"
        mask_out = bnk == "res"
        elems = M * K
        if "bnf" in only:
            t = timed(lambda: C_.bn_fwd_from_sums(y, resid, g, b, sums, rm, rv, 0.1, 1e-5, relu, mask_out), a.reps)
            nbytes = elems * (4 + (2 if resid is not None else 0) + (0.125 if mask_out else 0))
            rows.append({"layer": name, "op": "bn_fwd", "count": cnt, "ms": round(t, 4), "step_ms": round(t * cnt, 3),
                         "tbps": round(nbytes / t / 1e9, 2), "sol": round(nbytes / 8e9 / t, 2),
                         "lost_ms_per_step": round((t - nbytes / 8e9) * cnt, 3)})
            tot["bn_fwd"] = tot.get("bn_fwd", 0.0) + t * cnt
        if "bnb" in only:
            out = C_.bn_fwd_from_sums(y, resid, g, b, sums, rm, rv, 0.1, 1e-5, relu, mask_out)
            yy, mean, invstd = out[0], out[1], out[2]
            mask = out[3] if mask_out else None
            dg, db = torch.empty(K, device=dev), torch.empty(K, device=dev)
            relu_x = relu and not mask_out
            t = timed(lambda: C_.bn_bwd(gy, y, None, mean, invstd, g, b, relu_x, dg, db, bnk == "res", mask),
                      a.reps)
            # reduce: dy + x (+ mask); apply: dy + x (+ mask) -> dx (+ dres)
            nbytes = elems * (4 + 4 + 2 + (2 if bnk == "res" else 0) + (0.25 if mask_out else 0))
            rows.append({"layer": name, "op": "bn_bwd", "count": cnt, "ms": round(t, 4), "step_ms": round(t * cnt, 3),
                         "tbps": round(nbytes / t / 1e9, 2), "sol": round(nbytes / 8e9 / t, 2),
                         "lost_ms_per_step": round((t - nbytes / 8e9) * cnt, 3)})
            tot["bn_bwd"] = tot.get("bn_bwd", 0.0) + t * cnt
        for r in rows:
            print(json.dumps(r), flush=True)
        rows = []
        del x, w, gy
        torch.cuda.empty_cache()
    print(json.dumps({"summary_ms_per_step": {k: round(v, 2) for k, v in tot.items()},
                      "total_ms": round(sum(tot.values()), 2), "batch": N}), flush=True)


if __name__ == "__main__":
    main()
