"""Time one K-major x K-major bf16 product per shape (forward form) in this process: A/B of build-time variants
selected by environment (read once per process). Prints one JSON line per shape."""
import json
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from k8s_amd.ops._ext import load  # noqa: E402

C = load()
d = torch.device("cuda")
for spec in sys.argv[1:] or ["4096,28672,4096", "4096,4096,14336", "8192,8192,8192"]:
    M, N, K = (int(v) for v in spec.split(","))
    x = (torch.rand(M, K, device=d) * 2 - 1).bfloat16()
    w = (torch.rand(N, K, device=d) * 2 - 1).bfloat16()
    f = lambda: C.gemm(x, True, w, True, None, False, None, 0, None, False, 1.0, 1)  # noqa: E731
    y = f()
    torch.cuda.synchronize()
    err = ((y.float() - x.float() @ w.float().t()).norm() / (x.float() @ w.float().t()).norm()).item()
    best = 1e9
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            f()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / 10)
    print(json.dumps({"MNK": [M, N, K], "env": {k: v for k, v in os.environ.items() if k.startswith("K8S_AMD_W4")},
                      "us": round(best * 1e3, 1), "tf": round(2.0 * M * N * K / best / 1e9), "relerr": err}), flush=True)
    del x, w, y
