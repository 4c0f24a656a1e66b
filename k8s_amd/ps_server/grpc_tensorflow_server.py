#!/usr/bin/env python3
"""Default parameter server for TfJob PS replicas (the IsDefaultPS path).

CLI-compatible with the reference's default PS
(`/root/reference/grpc_tensorflow_server/grpc_tensorflow_server.py:119-157`):

    python grpc_tensorflow_server.py --cluster_spec "master|m-0:2222,ps|p-0:2222;p-1:2222" \\
        --job_name ps --task_id 0 [--gpu_memory_fraction F] [--verbose]

The operator ships this file in the ``cm-ps-<runtime id>`` ConfigMap
(``grpcServerFilePath`` in the controller config) and runs it in every
default-PS pod. Instead of a TF 1.x gRPC server it runs a small TCP task
server that:

* executes ops sent by other tasks on this task's device (what the smoke
  workload's master uses to check every task runs a kernel), and
* is the trainer's VARIABLE STORE OF RECORD (``k8s_amd.parallel.ps_vars``):
  ``vput`` / ``vcommit`` / ``vgc`` / ``vinfo`` / ``vget`` move raw fp32 shards
  of the flat master weights, optimizer state and buffers (binary payload
  after a JSON header, no re-encoding). The chief pushes a versioned snapshot
  every ``--ps-sync-every`` steps; a restarted job pulls the newest snapshot
  committed on EVERY PS task, as TF workers re-read their variables from
  ``/job:ps`` (workers stay stateless). The per-step gradient exchange is not
  here: it rides RCCL between the GPU ranks (``k8s_amd.parallel.ps``).

Snapshots are two-phase and multi-versioned: every shard is stored under its
version (a ``vput`` of version v+1 never overwrites version v's bytes),
``vcommit`` makes a version readable on one task only after all its shards
landed there, and the chief drops older versions (``vgc``) only after the new
one is committed on every task. A chief that dies mid-push therefore leaves
the previous snapshot intact and readable on every task.

The process blocks serving until it receives a ``shutdown`` message or
SIGTERM (exit 0), mirroring ``server.join()``.
The file is self-contained (stdlib + optional torch) because it is executed
from a ConfigMap mount.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import socketserver
import struct
import sys
import threading
from typing import Optional


def parse_cluster_spec(cluster_spec: str, job_name: str = "", task_id: int = 0):
    """'job|h:p;h:p,job2|h:p' -> {job: [hosts]} with the reference's strict errors (:46-88)."""
    cluster = {}
    if not cluster_spec:
        raise ValueError("Empty cluster_spec string")
    for job_string in cluster_spec.split(","):
        if not job_string:
            raise ValueError("Empty job_string in cluster_spec")
        parts = job_string.split("|")
        if len(parts) != 2:
            raise ValueError("Not exactly one instance of '|' in cluster_spec")
        name, hosts = parts
        if not name:
            raise ValueError("Empty job_name in cluster_spec")
        if name in cluster:
            raise ValueError("Duplicate job_name in cluster_spec: %s" % name)
        job_tasks = hosts.split(";")
        if any(not t for t in job_tasks):
            raise ValueError("Empty task string at position in cluster_spec")
        cluster[name] = job_tasks
    if job_name and job_name not in cluster:
        raise ValueError("job_name %r not in cluster_spec" % job_name)
    if job_name and not (0 <= task_id < len(cluster[job_name])):
        raise ValueError("Invalid task_id: %d" % task_id)
    return cluster


def _service_table():
    """The local kubelet's service map: the live file ($K8S_AMD_SERVICE_MAP_FILE, kept current by the kubelet)
    when readable, else the snapshot in $K8S_AMD_SERVICE_MAP taken at container start."""
    f = os.environ.get("K8S_AMD_SERVICE_MAP_FILE")
    if f:
        try:
            with open(f) as fh:
                return json.load(fh)
        except (OSError, ValueError):
            pass
    m = os.environ.get("K8S_AMD_SERVICE_MAP")
    return json.loads(m) if m else None


def resolve(addr: str) -> str:
    t = _service_table()
    if t:
        return t.get(addr) or t.get(addr.rsplit(":", 1)[0]) or addr
    return addr


# ----------------------------------------------------------------------------- wire protocol
def send_msg(sock, obj):
    data = json.dumps(obj).encode()
    sock.sendall(struct.pack("!I", len(data)) + data)


def recv_msg(sock):
    hdr = b""
    while len(hdr) < 4:
        chunk = sock.recv(4 - len(hdr))
        if not chunk:
            return None
        hdr += chunk
    n = struct.unpack("!I", hdr)[0]
    buf = b""
    while len(buf) < n:
        chunk = sock.recv(min(1 << 20, n - len(buf)))
        if not chunk:
            return None
        buf += chunk
    return json.loads(buf)


def recv_exact(sock, n: int) -> Optional[bytearray]:
    """n raw bytes (a variable shard payload) or None if the peer closed first."""
    buf = bytearray(n)
    view, got = memoryview(buf), 0
    while got < n:
        k = sock.recv_into(view[got:], min(8 << 20, n - got))
        if not k:
            return None
        got += k
    return buf


def send_blob(sock, hdr: dict, payload) -> None:
    """JSON header carrying ``nbytes`` followed by the raw payload (bytes / memoryview), no re-encoding."""
    mv = memoryview(payload).cast("B")
    send_msg(sock, dict(hdr, nbytes=mv.nbytes))
    sock.sendall(mv)


def call(addr: str, obj, timeout: float = 30.0, payload=None, want_payload: bool = False):
    """One request/response round trip. ``payload``: raw bytes sent after the header; ``want_payload``: returns
    (reply header, raw bytes) for replies that carry ``nbytes``."""
    host, port = resolve(addr).rsplit(":", 1)
    with socket.create_connection((host, int(port)), timeout=timeout) as s:
        if payload is not None:
            send_blob(s, obj, payload)
        else:
            send_msg(s, obj)
        rep = recv_msg(s)
        if not want_payload:
            return rep
        data = recv_exact(s, int(rep.get("nbytes", 0))) if rep is not None and rep.get("nbytes") else None
        return rep, data


def _device():
    try:
        import torch

        if torch.cuda.is_available() and os.environ.get("K8S_AMD_NO_GPU") != "1":
            return torch, torch.device("cuda", 0)
        return torch, torch.device("cpu")
    except ImportError:
        return None, None


class TaskServer(socketserver.ThreadingTCPServer):
    allow_reuse_address = True
    daemon_threads = True

    def __init__(self, addr, job, task, verbose=False):
        self.job, self.task, self.verbose = job, task, verbose
        # variable store of record (parallel/ps_vars.py): (version, push id, name, lo) -> raw little-endian fp32
        # bytes; `committed`: version -> (push id, metadata) of every version whose shards all landed on this task
        self.shards = {}
        self.committed = {}
        self.lock = threading.Lock()
        super().__init__(addr, _TaskHandler)


class _TaskHandler(socketserver.BaseRequestHandler):
    def handle(self):
        srv: TaskServer = self.server
        while True:
            msg = recv_msg(self.request)
            if msg is None:
                return
            op = msg.get("op")
            if srv.verbose:
                print("[%s:%d] op=%s" % (srv.job, srv.task, op), flush=True)
            if op == "multiply":  # the tf_smoke op: a * b on this task's device
                torch, dev = _device()
                if torch is not None:
                    a = torch.tensor(msg["a"], dtype=torch.int32, device=dev)
                    b = torch.tensor(msg["b"], dtype=torch.int32, device=dev)
                    out = (a * b).cpu().tolist()
                    where = str(dev)
                else:
                    out = [[x * y for x, y in zip(ra, rb)] for ra, rb in zip(msg["a"], msg["b"])]
                    where = "cpu"
                send_msg(self.request, {"ok": True, "result": out, "device": where,
                                        "task": "/job:%s/task:%d" % (srv.job, srv.task)})
            elif op == "vput":  # one variable shard (raw fp32 payload) of push `push` of snapshot `version`
                data = recv_exact(self.request, int(msg["nbytes"]))
                if data is None:
                    return
                v, push = int(msg["version"]), str(msg.get("push", ""))
                with srv.lock:  # keyed by push id: a re-push of a version never touches a committed copy
                    srv.shards[(v, push, msg["name"], int(msg["lo"]))] = data
                send_msg(self.request, {"ok": True})
            elif op == "vcommit":  # every shard of this push has landed on this task: make it readable here
                v, push = int(msg["version"]), str(msg.get("push", ""))
                with srv.lock:
                    names = msg.get("names") or []
                    ok = all((v, push, n, int(lo)) in srv.shards for n, lo in names)
                    if ok:
                        srv.committed[v] = (push, msg.get("meta", {}))
                send_msg(self.request, {"ok": ok, "committed": sorted(srv.committed)})
            elif op == "vgc":  # `keep` is committed on every task: drop older versions and stale partial pushes
                keep = int(msg["keep"])
                with srv.lock:
                    live = srv.committed.get(keep, (None,))[0]
                    for key in [k for k in srv.shards if k[0] < keep or (k[0] == keep and k[1] != live)]:
                        del srv.shards[key]
                    for v in [v for v in srv.committed if v < keep]:
                        del srv.committed[v]
                send_msg(self.request, {"ok": True, "committed": sorted(srv.committed)})
            elif op == "vinfo":
                with srv.lock:
                    send_msg(self.request, {"ok": True, "committed": sorted(srv.committed),
                                            "meta": {str(v): m for v, (_, m) in srv.committed.items()},
                                            "shards": sorted([v, n, lo] for v, _, n, lo in srv.shards)})
            elif op == "vget":
                v = int(msg["version"])
                with srv.lock:
                    ent = srv.committed.get(v)
                    data = srv.shards.get((v, ent[0], msg["name"], int(msg["lo"]))) if ent else None
                if data is None:
                    send_msg(self.request, {"ok": False, "error": "no committed shard %s@%s of version %d"
                                            % (msg["name"], msg["lo"], v)})
                else:
                    send_blob(self.request, {"ok": True, "version": v}, data)
            elif op == "ping":
                send_msg(self.request, {"ok": True, "task": "/job:%s/task:%d" % (srv.job, srv.task)})
            elif op == "shutdown":
                send_msg(self.request, {"ok": True})
                threading.Thread(target=srv.shutdown, daemon=True).start()
                return
            else:
                send_msg(self.request, {"ok": False, "error": "unknown op %r" % op})


def _bool_arg(v: str) -> bool:
    return v.lower() == "true"


def serve(cluster, job_name, task_id, verbose=False) -> int:
    addr = resolve(cluster[job_name][task_id])
    host, port = addr.rsplit(":", 1)
    bind_host = "127.0.0.1" if host in ("127.0.0.1", "localhost") else "0.0.0.0"
    srv = TaskServer((bind_host, int(port)), job_name, task_id, verbose)
    if threading.current_thread() is threading.main_thread():
        signal.signal(signal.SIGTERM, lambda *a: threading.Thread(target=srv.shutdown, daemon=True).start())
    print("Started server /job:%s/task:%d on %s" % (job_name, task_id, addr), flush=True)
    srv.serve_forever()
    srv.server_close()
    return 0


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="Run a default parameter server for a TfJob.")
    p.add_argument("--cluster_spec", type=str, help="Cluster spec: 'job|host:port;host:port,job2|host:port'")
    p.add_argument("--job_name", type=str, help="Job name: e.g., ps")
    p.add_argument("--task_id", type=int, default=0, help="Task index, e.g., 0")
    p.add_argument("--gpu_memory_fraction", type=float, default=1.0,
                   help="Fraction of GPU memory allocated (per-process cap via torch)")
    # the reference registers type "bool" as `v.lower() == "true"` with nargs="?" / const=True
    # (/root/reference/grpc_tensorflow_server/grpc_tensorflow_server.py:150-156): a bare --verbose is True,
    # --verbose=true / --verbose True are True, --verbose False (or anything else) is False
    p.add_argument("--verbose", type=_bool_arg, nargs="?", const=True, default=False, help="Verbose mode")
    return p


def main(argv=None):
    # unknown flags are ignored, as the reference does (parse_known_args,
    # /root/reference/grpc_tensorflow_server/grpc_tensorflow_server.py:159): a PS pod must not crash on an extra flag
    a, unknown = build_parser().parse_known_args(argv)
    if unknown:
        print("ignoring unknown flags: %s" % " ".join(unknown), file=sys.stderr, flush=True)
    cluster = parse_cluster_spec(a.cluster_spec, a.job_name, a.task_id)
    torch, dev = _device()
    if torch is not None and dev is not None and dev.type == "cuda" and a.gpu_memory_fraction < 1.0:
        torch.cuda.set_per_process_memory_fraction(a.gpu_memory_fraction, 0)
    return serve(cluster, a.job_name, a.task_id, a.verbose)


if __name__ == "__main__":
    sys.exit(main())
