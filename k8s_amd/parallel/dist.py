"""Process-group setup: one process per GPU, RCCL over xGMI.

Two ways in:

* ``torchrun``-style env (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR /
  MASTER_PORT) -- what ``bench.py`` is launched with.
* ``TF_CONFIG`` -- what the operator injects into every replica
  (`/root/reference/pkg/trainer/replicas.go:188-203`). ``rank_from_tf_config``
  maps the cluster spec to a deterministic global rank order
  (master -> 0, then worker 0..N-1, then ps 0..M-1; the chief named by the
  TerminationPolicy is rank 0) and uses the MASTER service address as the
  TCP-store rendezvous, so the operator's only contract with the workload
  stays TF_CONFIG.
"""
from __future__ import annotations

import datetime
import json
import os

# dmabuf IPC (see bench.py): must be in the environment before the first HIP call of this process
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

ROLE_ORDER = ("master", "chief", "worker", "ps", "evaluator")


@dataclass
class RankInfo:
    rank: int
    world_size: int
    local_rank: int
    master_addr: str
    master_port: int
    role: str = "worker"
    role_index: int = 0
    compute_world: int = 1  # ranks that run the model (everything but ps)

    @property
    def device_index(self) -> int:
        """The GPU this rank drives: its local rank. ``K8S_AMD_GPU_OVERSUBSCRIBE=1`` wraps it modulo the visible
        devices, so several ranks can share one GPU for a rehearsal of the multi-rank path on a 1-GPU box
        (with ``K8S_AMD_DIST_BACKEND=gloo``: RCCL refuses two ranks on one device)."""
        if os.environ.get("K8S_AMD_GPU_OVERSUBSCRIBE") == "1" and torch.cuda.is_available():
            return self.local_rank % max(1, torch.cuda.device_count())
        return self.local_rank


def resolve(addr: str) -> str:
    """Map a TF_CONFIG "service:port" through $K8S_AMD_SERVICE_MAP (local kubelet's cluster-DNS stand-in)."""
    from k8s_amd.ps_server.grpc_tensorflow_server import _service_table

    table = _service_table()
    if not table:
        return addr
    if addr in table:
        return table[addr]
    host = addr.rsplit(":", 1)[0]
    return table.get(host, addr)


def local_device_count() -> int:
    """GPUs this container was given, WITHOUT initialising the GPU (a process that has touched HIP must not be the
    one that forks the per-GPU trainers): the kubelet's / device plugin's visibility list when set, else the
    runtime's device count (``torch.cuda.device_count`` does not initialise HIP on this image), else 1."""
    for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"):
        v = os.environ.get(k)
        if v is not None and v.strip():
            return len([d for d in v.split(",") if d.strip()])
    if os.environ.get("K8S_AMD_NO_GPU") == "1":
        return 1
    try:
        return max(1, torch.cuda.device_count())
    except Exception:  # noqa: BLE001
        return 1


def task_gpus_table() -> Optional[Dict[str, int]]:
    """``TFJOB_TASK_GPUS`` (set by the operator next to TF_CONFIG): GPUs per task of every replica type."""
    v = os.environ.get("TFJOB_TASK_GPUS")
    if not v:
        return None
    try:
        return {str(k).lower(): int(n) for k, n in json.loads(v).items()}
    except (ValueError, TypeError, AttributeError):
        return None


def own_task_processes(role: str) -> int:
    """Processes THIS task runs (one per GPU): its role's entry in ``TFJOB_TASK_GPUS`` when the operator set one,
    else this container's device count. The world size every rank computes (``rank_from_tf_config``) uses the same
    table, so a task whose container sees fewer GPUs than the table says would leave the rendezvous one rank short
    until its timeout: that is refused here, up front, with the two numbers."""
    mine = local_device_count()
    table = task_gpus_table()
    if table is None or role not in table:
        return mine
    want = max(1, int(table[role]))
    if want > mine:
        raise ValueError("TFJOB_TASK_GPUS gives a %s task %d GPUs but this container sees %d" % (role, want, mine))
    return want


def rank_from_tf_config(tf_config: str, port_offset: int = 0, local_rank: Optional[int] = None,
                        task_gpus: Optional[Dict[str, int]] = None) -> RankInfo:
    """Deterministic rank assignment from a TF_CONFIG JSON string.

    Compute ranks (the collective group) are master/chief first, then workers;
    PS tasks do not join the RCCL group (rank -1): in this framework the
    parameter service is sharded over the compute ranks (parallel/ps.py) and
    the PS replicas run the parameter/rendezvous server (ps_server/).

    A task given n > 1 GPUs runs n processes, one per GPU (``trainer/runner.py`` forks them, ``LOCAL_RANK`` i):
    the reference's single MASTER pod with ``--num-gpus=N`` (`/root/reference/examples/gke/TF on GKE.ipynb`
    lines 976, 988; in-graph replication, `/root/reference/tf_job_design_doc.md:101-103`) becomes N ranks.
    Task t's processes take global ranks ``sum(n of the tasks before t) + i``; the world is the sum over tasks.
    ``task_gpus`` (role -> GPUs per task, from the operator's ``TFJOB_TASK_GPUS``) gives every task's n; without
    it every compute task is assumed to have this container's device count.

    The TCP-store rendezvous listens on the first compute task's own ``tfPort``
    (``port_offset`` 0): that is the one port the operator's per-replica
    ClusterIP Service forwards (`/root/reference/pkg/trainer/replicas.go:156-186`,
    port ``tf-port``), and the trainer itself binds nothing else there. RCCL's
    own bootstrap/data connections go pod-to-pod and need no Service.
    """
    cfg = json.loads(tf_config)
    cluster: Dict[str, List[str]] = cfg.get("cluster", {})
    task = cfg.get("task", {})
    ttype, tidx = task.get("type", "master").lower(), int(task.get("index", 0))
    order = []
    for role in ROLE_ORDER:
        if role == "ps":
            continue
        for i, addr in enumerate(cluster.get(role, [])):
            order.append((role, i, addr))
    for role in sorted(cluster):  # unknown roles last, deterministic
        if role not in ROLE_ORDER:
            for i, addr in enumerate(cluster[role]):
                order.append((role, i, addr))
    if not order and not cluster.get("ps"):
        raise ValueError("TF_CONFIG has an empty cluster")
    keys = [(r, i) for r, i, _ in order]
    if local_rank is None:
        local_rank = int(os.environ.get("LOCAL_RANK", 0))
    table = task_gpus if task_gpus is not None else task_gpus_table()
    mine = local_device_count()

    def procs(role):  # processes a task of this role runs (a CPU-only task: one)
        if table is None:
            return mine
        return max(1, int(table.get(role, mine)))

    counts = [procs(r) for r, _, _ in order]
    if table is not None and ttype in table and ttype != "ps" and procs(ttype) > mine:
        raise ValueError("TFJOB_TASK_GPUS gives a %s task %d GPUs but this container sees %d"
                         % (ttype, procs(ttype), mine))
    if ttype == "ps":
        rank = -1
    elif (ttype, tidx) in keys:
        k = keys.index((ttype, tidx))
        if local_rank >= counts[k]:
            raise ValueError("local rank %d but task %s:%d runs %d processes" % (local_rank, ttype, tidx, counts[k]))
        rank = sum(counts[:k]) + local_rank
    else:
        raise ValueError("task %s:%d not in cluster %s" % (ttype, tidx, sorted(cluster)))
    first = order[0][2] if order else cluster["ps"][0]
    host, _, port = resolve(first).rpartition(":")
    world = sum(counts)
    return RankInfo(rank=rank, world_size=world, local_rank=local_rank,
                    master_addr=host or first, master_port=int(port or 2222) + port_offset, role=ttype,
                    role_index=tidx, compute_world=world)


def rank_from_env() -> Optional[RankInfo]:
    if "WORLD_SIZE" in os.environ and "RANK" in os.environ:
        ws = int(os.environ["WORLD_SIZE"])
        return RankInfo(rank=int(os.environ["RANK"]), world_size=ws,
                        local_rank=int(os.environ.get("LOCAL_RANK", 0)),
                        master_addr=os.environ.get("MASTER_ADDR", "127.0.0.1"),
                        master_port=int(os.environ.get("MASTER_PORT", 29500)), compute_world=ws)
    if "TF_CONFIG" in os.environ:
        return rank_from_tf_config(os.environ["TF_CONFIG"])
    return None


def init_process_group(info: Optional[RankInfo] = None, backend: Optional[str] = None,
                       timeout_s: float = 600.0, force: bool = False) -> RankInfo:
    """Initialise torch.distributed (nccl == RCCL on ROCm, gloo on CPU; ``K8S_AMD_DIST_BACKEND`` overrides the
    default). Idempotent. A world of one creates no group unless ``force`` (a one-rank RCCL communicator: the
    transports then run their real collectives on one GPU -- ``bench.py --force-dist``, ``tests/test_rccl_gpu.py``);
    a forced world-1 group without a torchrun env rendezvouses on a free local port."""
    env_info = rank_from_env()
    if info is None and env_info is None and force:
        from k8s_amd.fakeapi.server import free_port

        info = RankInfo(0, 1, 0, "127.0.0.1", free_port())
    info = info or env_info or RankInfo(0, 1, 0, "127.0.0.1", 29500)
    if (info.world_size > 1 or force) and not dist.is_initialized():
        if backend is None:
            backend = os.environ.get("K8S_AMD_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if torch.cuda.is_available():
            torch.cuda.set_device(info.device_index)
        dist.init_process_group(backend=backend, init_method="tcp://%s:%d" % (info.master_addr, info.master_port),
                                rank=info.rank, world_size=info.world_size,
                                timeout=datetime.timedelta(seconds=timeout_s))
    elif torch.cuda.is_available():
        torch.cuda.set_device(info.device_index)
    return info


def barrier():
    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def all_reduce_max(x: float, device) -> float:
    if not (dist.is_available() and dist.is_initialized()):
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def destroy():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
