"""Driver for rocprofv3 --pmc passes over ResNet-50's memory-bound 1x1 convolutions at batch 1024 (10 launches
each): s2 conv3 forward (256 -> 1024 channels at 14x14, BN statistics epilogue) and s0 conv3 forward (64 -> 256 at
56x56, the single-buffer K = 64 kernel).

    rocprofv3 --pmc <counters> -d gpurun_out/pmc1 -o p -- python scripts/pmc_1x1.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_amd.ops._ext import load  # noqa: E402

C = load()
dev = torch.device("cuda")
torch.manual_seed(0)
cases = [((1024, 14, 14, 256), 1024), ((1024, 56, 56, 64), 256)]
for shape, K in cases:
    x = torch.randn(*shape, device=dev).bfloat16()
    w = (torch.randn(K, 1, 1, shape[-1], device=dev) * 0.05).bfloat16()
    st = torch.zeros(C.conv_stat_replicas, 2, K, device=dev)
    for _ in range(10):
        C.conv_fwd(x, w, 1, 0, 1, False, None, 0, st)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        C.conv_fwd(x, w, 1, 0, 1, False, None, 0, st)
    e.record()
    e.synchronize()
    print("%s -> %d: %.1f us" % (shape, K, s.elapsed_time(e) * 100), flush=True)
