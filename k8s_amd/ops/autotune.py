"""Measured per-shape kernel selection ("measure, don't guess").

For an op with more than one implementation (tile variants of one of our kernels, an experimental
schedule, ...) the first call of a shape times every candidate on the real tensors (cuda events, median
of a few runs) and caches the winner for the process and in a JSON file (``$K8S_AMD_AUTOTUNE_CACHE``,
default ``~/.cache/k8s_amd/autotune-v3.json``; ``none`` disables the file). Candidates must be
side-effect free or write to scratch while tuning. ``K8S_AMD_AUTOTUNE=0`` disables tuning (always the
first candidate).

Since round 2 no shipped op offers a vendor candidate (MIOpen / hipBLASLt): conv and linear always run
our kernels for shapes inside their contract and count + warn on the rest (``conv.STATS``,
``gemm.FALLBACKS``), so the seed tables of round 1 are gone. The A/B scripts under ``scripts/`` use
``_time`` as their timer.
"""
from __future__ import annotations

import json
import os
import sys
import threading
from typing import Callable, Dict, Sequence, Tuple

import torch

_cache: Dict[str, str] = {}
_lock = threading.Lock()
_loaded = False
STATS: Dict[str, Dict[str, int]] = {}


def enabled() -> bool:
    return os.environ.get("K8S_AMD_AUTOTUNE", "1") != "0"


CACHE_VERSION = "v3"  # bump when kernels / candidates change


def cache_path():
    p = os.environ.get("K8S_AMD_AUTOTUNE_CACHE")
    if p is None:
        base = os.environ.get("XDG_CACHE_HOME") or os.path.join(os.path.expanduser("~"), ".cache")
        p = os.path.join(base, "k8s_amd", "autotune-%s.json" % CACHE_VERSION)
    return None if p in ("", "none") else p


def _load_cache():
    global _loaded
    if _loaded:
        return
    _loaded = True
    p = cache_path()
    if p and os.path.exists(p):
        try:
            _cache.update(json.load(open(p)))
        except (ValueError, OSError):
            pass


def _save_cache():
    p = cache_path()
    if not p:
        return
    try:
        os.makedirs(os.path.dirname(p), exist_ok=True)
        tmp = p + ".tmp.%d" % os.getpid()
        with open(tmp, "w") as f:
            json.dump(_cache, f, indent=1, sort_keys=True)
        os.replace(tmp, p)
    except OSError:
        pass  # read-only home: keep the in-process cache


def _time(fn, reps=3) -> float:
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


# Another candidate must beat the default (candidate 0) by this margin: near-ties flip between runs on
# timing noise.
MARGIN = float(os.environ.get("K8S_AMD_AUTOTUNE_MARGIN", "0.03"))


def choose(key: str, candidates: Sequence[Tuple[str, Callable[[], object]]]) -> str:
    """Return the name of the fastest candidate for `key` (tuning on first use)."""
    _load_cache()
    name = _cache.get(key)
    if name is not None and name not in [n for n, _ in candidates]:
        name = None  # stale entry (candidate set changed)
    if name is None:
        if not enabled() or len(candidates) == 1 or not torch.cuda.is_available():
            name = candidates[0][0]
        else:
            times = {}
            for n, fn in candidates:
                try:
                    times[n] = _time(fn, reps=5)
                except RuntimeError:
                    continue
            name = candidates[0][0]
            if times:
                best = min(times, key=times.get)
                ours = times.get(name)
                if ours is None or times[best] < ours * (1.0 - MARGIN):
                    name = best
            with _lock:
                _cache[key] = name
                _save_cache()
            if os.environ.get("K8S_AMD_AUTOTUNE_VERBOSE", "0") != "0":  # progress for long cold-start tuning
                print("autotune %s -> %s %s" % (key, name, {n: round(t, 4) for n, t in times.items()}),
                      file=sys.stderr, flush=True)
    st = STATS.setdefault(key.split("|")[0], {})
    st[name] = st.get(name, 0) + 1
    return name


def choices() -> Dict[str, str]:
    return dict(_cache)
