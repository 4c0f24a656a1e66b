"""Step-phase tracing and the trainer's hang watchdog.

The reference has no tracing at all (glog verbosity only, ``pkg/trainer/training.go:385``). Here:

* ``Tracer.phase(name)`` wraps a step phase (``forward``, ``backward``, ``allreduce``, ``optimizer``, ...) in a
  ROCTx range, so ``rocprofv3 --marker-trace --kernel-trace`` shows which kernels ran in which phase, and
  (``sync=True``) accumulates per-phase wall time measured between device synchronisations -- written to
  the metrics stream as ``phase_ms``. Disabled phases cost one attribute check.
  ROCTx comes from the rocprofiler-sdk library that rocprofv3 records (``librocprofiler-sdk-roctx.so``),
  falling back to ``torch.cuda.nvtx`` (the legacy roctx64 on ROCm builds of PyTorch).
* ``Watchdog``: a collective that never completes (a dead peer, a wedged link) would otherwise leave the
  replica Running forever. If no ``kick()`` arrives within ``timeout`` seconds the process exits with 143
  (>= 128: retryable), so the operator's exit-code contract (``pkg/trainer/training.go:203-238``) restarts it
  and it resumes from the latest checkpoint.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import sys
import threading
import time
from collections import defaultdict
from typing import Callable, Dict, Optional

EXIT_HANG = 143

_roctx = None


def _load_roctx():
    global _roctx
    if _roctx is not None:
        return _roctx
    for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                 "/opt/rocm/lib/librocprofiler-sdk-roctx.so"):
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            _roctx = (lambda s: lib.roctxRangePushA(s.encode()), lib.roctxRangePop)
            return _roctx
        except (OSError, AttributeError):
            continue
    try:
        import torch.cuda.nvtx as nvtx

        _roctx = (nvtx.range_push, nvtx.range_pop)
    except Exception:  # noqa: BLE001  -- no tracer: ranges become no-ops
        _roctx = (lambda s: None, lambda: None)
    return _roctx


class Tracer:
    def __init__(self, enabled: bool = False, sync: bool = False, sync_fn: Optional[Callable[[], None]] = None):
        self.enabled = enabled
        self.sync = sync and enabled
        self.sync_fn = sync_fn or (lambda: None)
        self.totals: Dict[str, float] = defaultdict(float)
        self.counts: Dict[str, int] = defaultdict(int)
        if enabled:
            _load_roctx()

    @classmethod
    def from_env(cls, sync_fn=None) -> "Tracer":
        v = os.environ.get("K8S_AMD_TRACE", "")
        return cls(enabled=v not in ("", "0"), sync=(v == "sync"), sync_fn=sync_fn)

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            yield
            return
        push, pop = _roctx
        if self.sync:
            self.sync_fn()
        t0 = time.perf_counter()
        push(name)
        try:
            yield
        finally:
            if self.sync:
                self.sync_fn()
            pop()
            self.totals[name] += time.perf_counter() - t0
            self.counts[name] += 1

    def summary_ms(self, reset: bool = True) -> Dict[str, float]:
        """Mean milliseconds per occurrence of each phase since the last reset."""
        out = {k: round(1e3 * v / max(self.counts[k], 1), 3) for k, v in self.totals.items()}
        if reset:
            self.totals.clear()
            self.counts.clear()
        return out


class Watchdog:
    """Exit the process (code 143) when ``kick()`` has not been called for ``timeout`` seconds."""

    def __init__(self, timeout: float, on_fire: Optional[Callable[[], None]] = None, poll: float = 1.0,
                 exit_fn: Callable[[int], None] = os._exit):
        self.timeout = timeout
        self.on_fire = on_fire
        self.poll = min(poll, max(timeout / 4, 0.01))
        self.exit_fn = exit_fn
        self._last = time.monotonic()
        self._stop = threading.Event()
        self.fired = False
        self._th = None

    def start(self) -> "Watchdog":
        if self.timeout > 0:
            self._th = threading.Thread(target=self._run, name="k8s_amd-watchdog", daemon=True)
            self._th.start()
        return self

    def kick(self):
        self._last = time.monotonic()

    def stop(self):
        self._stop.set()
        if self._th is not None:
            self._th.join(timeout=5)

    def _run(self):
        while not self._stop.wait(self.poll):
            idle = time.monotonic() - self._last
            if idle > self.timeout:
                self.fired = True
                print("watchdog: no training progress for %.0f s (hung collective?); exiting %d (retryable)"
                      % (idle, EXIT_HANG), file=sys.stderr, flush=True)
                if self.on_fire is not None:
                    try:
                        self.on_fire()
                    except Exception:  # noqa: BLE001
                        pass
                self.exit_fn(EXIT_HANG)
                return
