"""PS replicas as the variable store of record.

In the reference's TfJobs the variables live on the ``/job:ps`` tasks
(``replica_device_setter``, `/root/reference/examples/tf_sample/tf_sample/tf_smoke.py:116-118`;
the PS runs ``server.join()``, `/root/reference/grpc_tensorflow_server/grpc_tensorflow_server.py:93-115`):
workers are stateless, and a restarted worker reads the current values back from the PS.

Here the per-step gradient exchange stays on RCCL between the GPU ranks (``parallel/ddp.py`` /
``parallel/ps.py``: pushing every step's gradients through a few PS processes' NICs would cap a
MI355X node at TCP speed). The PS tasks keep the authoritative COPY of the variables instead:

* ``push(version, tensors)``: the chief copies the flat fp32 buffers (master weights, optimizer state, model
  buffers) to host memory once, then a background thread streams each buffer's per-PS-task shard
  (``vput``, raw fp32, equal 64-element-aligned ranges, task j holds range j of every buffer) and commits the
  version on every task (``vcommit``): the training loop only waits for the device-to-host copy.
* ``latest()`` / ``pull(version)``: the newest version every PS task has committed, and its shards.
  ``trainer/runner.py`` restores from it when it is newer than the latest checkpoint (a job restarted after a
  retryable failure, or with no shared checkpoint volume), then broadcasts to every rank.
"""
from __future__ import annotations

import threading
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

    def _call(self, j, hdr, payload=None, want_payload=False):
        from k8s_amd.ps_server.grpc_tensorflow_server import call

        return call(self.addrs[j], hdr, timeout=self.timeout, payload=payload, want_payload=want_payload)

    # ------------------------------------------------------------------ push
    def push(self, version: int, tensors: Dict[str, torch.Tensor], meta: Optional[dict] = None) -> None:
        """Snapshot ``tensors`` (flattened to fp32) at ``version`` onto the PS tasks; returns once the host copy
        is taken (the network transfer runs in a background thread; the previous push is awaited first)."""
        self.wait()
        host = {k: v.detach().reshape(-1).to("cpu", torch.float32).numpy().copy() for k, v in tensors.items()}
        sizes = {k: int(a.size) for k, a in host.items()}
        meta = dict(meta or {}, sizes=sizes)

        def run():
            try:
                for j in range(len(self.addrs)):
                    names = []
                    for k, a in host.items():
                        lo, hi = shard_ranges(a.size, len(self.addrs))[j]
                        rep = self._call(j, {"op": "vput", "name": k, "lo": lo, "n": hi - lo, "version": version},
                                         payload=memoryview(a[lo:hi]))
                        if not rep or not rep.get("ok"):
                            raise RuntimeError("vput %s@%d on %s failed: %r" % (k, lo, self.addrs[j], rep))
                        names.append([k, lo])
                    rep = self._call(j, {"op": "vcommit", "version": version, "names": names, "meta": meta})
                    if not rep or not rep.get("ok"):
                        raise RuntimeError("vcommit %d on %s failed: %r" % (version, self.addrs[j], rep))
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
        vs, meta = [], {}
        for j in range(len(self.addrs)):
            rep = self._call(j, {"op": "vinfo"})
            if not rep or not rep.get("ok"):
                return -1, {}
            vs.append(int(rep.get("committed", -1)))
            meta = rep.get("meta") or meta
        v = min(vs)
        return (v, meta) if v >= 0 and all(x == v for x in vs) else (-1, {})

    def pull(self, version: int, names: Optional[List[str]] = None) -> Dict[str, torch.Tensor]:
        """The fp32 buffers of snapshot ``version`` (every shard checked to carry that version)."""
        _, meta = self.latest()
        sizes = meta.get("sizes", {})
        out = {}
        for k in (names or sorted(sizes)):
            n = int(sizes[k])
            buf = np.empty(n, dtype=np.float32)
            for j, (lo, hi) in enumerate(shard_ranges(n, len(self.addrs))):
                rep, data = self._call(j, {"op": "vget", "name": k, "lo": lo}, want_payload=True)
                if not rep or not rep.get("ok") or int(rep.get("version", -1)) != version:
                    raise RuntimeError("PS shard %s@%d: %r (want version %d)" % (k, lo, rep, version))
                if hi > lo:
                    buf[lo:hi] = np.frombuffer(data, dtype=np.float32, count=hi - lo)
            out[k] = torch.from_numpy(buf)
        return out
