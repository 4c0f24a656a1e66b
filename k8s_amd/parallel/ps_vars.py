"""PS replicas as the variable store of record.

In the reference's TfJobs the variables live on the ``/job:ps`` tasks
(``replica_device_setter``, `/root/reference/examples/tf_sample/tf_sample/tf_smoke.py:116-118`;
the PS runs ``server.join()``, `/root/reference/grpc_tensorflow_server/grpc_tensorflow_server.py:93-115`):
workers are stateless, and a restarted worker reads the current values back from the PS.

Here the per-step gradient exchange stays on RCCL between the GPU ranks (``parallel/ddp.py`` /
``parallel/ps.py``: pushing every step's gradients through a few PS processes' NICs would cap a
MI355X node at TCP speed). The PS tasks keep the authoritative COPY of the variables instead:

* ``push(version, tensors)``: the chief copies the flat fp32 buffers (master weights, optimizer state, model
  buffers) to host memory once, then a background thread runs the two-phase push: (1) every buffer's per-task
  shard to every PS task (``vput``, raw fp32, equal 64-element-aligned ranges, task j holds range j of every
  buffer; stored under the NEW version, the previous snapshot's bytes are untouched), (2) ``vcommit`` on every
  task, (3) only then ``vgc`` on every task (drop the versions older than the new one). The training loop only
  waits for the device-to-host copy. A chief that dies anywhere in (1)-(3) leaves the previous snapshot
  committed on every task (`ADVICE` round 2: a single-copy store let a half-finished push destroy it).
* ``latest()`` / ``pull(version)``: the newest version committed on every PS task, and its shards.
  ``trainer/runner.py`` restores from it when it is newer than the latest checkpoint (a job restarted after a
  retryable failure, or with no shared checkpoint volume), then broadcasts to every rank.
"""
from __future__ import annotations

import threading
import uuid
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from k8s_amd.parallel.dist import resolve

ALIGN = 64


def shard_ranges(n: int, parts: int) -> List[Tuple[int, int]]:
    """``parts`` contiguous [lo, hi) ranges covering n elements, boundaries on 64-element multiples."""
    per = -(-n // parts)
    per = -(-per // ALIGN) * ALIGN
    return [(min(n, j * per), min(n, (j + 1) * per)) for j in range(parts)]


class PsVariables:
    def __init__(self, ps_addrs: List[str], timeout: float = 60.0):
        if not ps_addrs:
            raise ValueError("no PS tasks")
        self.addrs = [resolve(a) for a in ps_addrs]
        self.timeout = timeout
        self._thread: Optional[threading.Thread] = None
        self._error: Optional[BaseException] = None
        self.pushed = -1
        self.fault_hook = None  # (testing) called between push phases

    def _call(self, j, hdr, payload=None, want_payload=False):
        from k8s_amd.ps_server.grpc_tensorflow_server import call

        return call(self.addrs[j], hdr, timeout=self.timeout, payload=payload, want_payload=want_payload)

    # ------------------------------------------------------------------ push
    def push(self, version: int, tensors: Dict[str, torch.Tensor], meta: Optional[dict] = None,
             fresh=()) -> None:
        """Snapshot ``tensors`` (flattened to fp32) at ``version`` onto the PS tasks; returns once the host copy
        is taken (the network transfer runs in a background thread; the previous push is awaited first).
        ``fresh``: keys whose tensors are host copies nobody mutates (e.g. ``gather_state`` output): sent as they
        are. Device tensors get exactly one device-to-host copy; other host tensors one host copy."""
        self.wait()

        def snap(k, v):
            v = v.detach().reshape(-1)
            if v.is_cuda:
                return v.to("cpu", torch.float32).numpy()  # a new host tensor already
            v = v.float()
            return v.numpy() if k in fresh else v.numpy().copy()

        host = {k: snap(k, v) for k, v in tensors.items()}
        sizes = {k: int(a.size) for k, a in host.items()}
        meta = dict(meta or {}, sizes=sizes)

        def run():
            try:
                ntask = len(self.addrs)
                push = uuid.uuid4().hex  # a re-push of the same version (after a restart) is a distinct copy
                names = [[] for _ in range(ntask)]
                for j in range(ntask):  # phase 1: every shard lands, under the new version
                    for k, a in host.items():
                        lo, hi = shard_ranges(a.size, ntask)[j]
                        rep = self._call(j, {"op": "vput", "name": k, "lo": lo, "n": hi - lo, "version": version,
                                             "push": push},
                                         payload=memoryview(a[lo:hi]))
                        if not rep or not rep.get("ok"):
                            raise RuntimeError("vput %s@%d on %s failed: %r" % (k, lo, self.addrs[j], rep))
                        names[j].append([k, lo])
                for j in range(ntask):  # phase 2: readable on every task
                    rep = self._call(j, {"op": "vcommit", "version": version, "push": push, "names": names[j],
                                        "meta": meta})
                    if not rep or not rep.get("ok"):
                        raise RuntimeError("vcommit %d on %s failed: %r" % (version, self.addrs[j], rep))
                if self.fault_hook is not None:  # (testing) a chief that dies between commit and GC
                    self.fault_hook("committed")
                for j in range(ntask):  # phase 3: the new version is everywhere, older ones can go
                    self._call(j, {"op": "vgc", "keep": version})
                self.pushed = version
            except BaseException as e:  # surfaced by wait()
                self._error = e

        self._thread = threading.Thread(target=run, name="ps-push", daemon=True)
        self._thread.start()

    def wait(self) -> None:
        """Join the in-flight push; re-raises its error."""
        if self._thread is not None:
            self._thread.join()
            self._thread = None
        if self._error is not None:
            e, self._error = self._error, None
            raise e

    # ------------------------------------------------------------------ pull
    def latest(self) -> Tuple[int, dict]:
        """(newest version committed on EVERY PS task or -1, that snapshot's metadata)."""
        common, meta = None, {}
        for j in range(len(self.addrs)):
            rep = self._call(j, {"op": "vinfo"})
            if not rep or not rep.get("ok"):
                return -1, {}
            vs = set(int(v) for v in rep.get("committed", []))
            common = vs if common is None else common & vs
            for v, m in (rep.get("meta") or {}).items():
                meta.setdefault(int(v), m)
        if not common:
            return -1, {}
        v = max(common)
        return v, meta.get(v, {})

    def pull(self, version: int, names: Optional[List[str]] = None) -> Dict[str, torch.Tensor]:
        """The fp32 buffers of snapshot ``version`` (every shard checked to carry that version)."""
        meta = None
        for j in range(len(self.addrs)):
            rep = self._call(j, {"op": "vinfo"})
            if rep and rep.get("ok") and str(version) in (rep.get("meta") or {}):
                meta = rep["meta"][str(version)]
                break
        if meta is None:
            raise RuntimeError("PS snapshot version %d is not committed" % version)
        sizes = meta.get("sizes", {})
        out = {}
        for k in (names or sorted(sizes)):
            n = int(sizes[k])
            buf = np.empty(n, dtype=np.float32)
            for j, (lo, hi) in enumerate(shard_ranges(n, len(self.addrs))):
                rep, data = self._call(j, {"op": "vget", "name": k, "lo": lo, "version": version},
                                       want_payload=True)
                if not rep or not rep.get("ok") or int(rep.get("version", -1)) != version:
                    raise RuntimeError("PS shard %s@%d: %r (want version %d)" % (k, lo, rep, version))
                if hi > lo:
                    buf[lo:hi] = np.frombuffer(data, dtype=np.float32, count=hi - lo)
            out[k] = torch.from_numpy(buf)
        return out
