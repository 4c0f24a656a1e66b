"""Device timer for the A/B and diagnostic scripts under ``scripts/`` ("measure, don't guess")."""
from __future__ import annotations

import torch


def time_ms(fn, reps: int = 3) -> float:
    """Median milliseconds of ``fn()`` over ``reps`` runs (cuda events), after one untimed warm-up call."""
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
