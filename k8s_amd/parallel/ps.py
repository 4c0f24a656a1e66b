"""Parameter-server data parallelism the MI355X way.

The reference's TfJobs place variables on ``/job:ps`` tasks and every worker
pushes gradients to / pulls parameters from them over gRPC
(`/root/reference/examples/tf_job.yaml:1-24`; ``replica_device_setter`` in
`/root/reference/examples/tf_sample/tf_sample/tf_smoke.py:116-118`).
Translating that literally -- a process per PS shard receiving every worker's
gradient over TCP -- would put the whole update on a few links. Here the
*parameter service is sharded over the compute ranks* and push / pull are
RCCL collectives over xGMI:

    push   = reduce-scatter of each gradient bucket: rank r ends with the summed
             gradient of its 1/world slice ("the PS shard it owns")
    update = the fused SGD/Adam kernel on the owned slices only; the optimizer
             keeps fp32 state for those slices only (ZeRO-1: 1/world of the
             moments per rank -- the PS role really holds the state)
    pull   = all-gather of the updated fp32 master slices; the bf16 working
             copy is refreshed locally

Two push transports:

* ``comm_dtype=float32``: ``reduce_scatter_tensor`` in place (the output IS
  this rank's slice of the bucket).
* ``comm_dtype=bfloat16`` (Llama-scale models): each bucket is cast to bf16
  and exchanged with ONE ``all_to_all_single`` -- on a fully connected 8-GPU
  xGMI mesh that is a direct one-hop exchange over all 7 links -- and the
  world received slices are summed in fp32 on the owner. Half the bytes of
  the fp32 push, with fp32 accumulation (the only rounding is each rank's
  contribution to bf16 once).

Buckets are fixed ranges of the flat buffer taken from the END (backward
produces the last layers' gradients first), each a multiple of world*64
elements, so a bucket's push starts as soon as every parameter overlapping it
has deposited -- overlapped with the rest of backward like ``GradReducer``.

PS replicas of a TfJob (``--job_name ps``) run the default PS server
(rendezvous / liveness / shutdown; ``ps_server/``) and are the variable store
of record: the chief pushes versioned snapshots of the weights, optimizer
state and buffers to them, sharded over the PS tasks, and a restarted job
resumes from the newest committed snapshot (``parallel/ps_vars.py``).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from k8s_amd.parallel.flat import ALIGN, ParamStore, _round_up


class _Range:
    __slots__ = ("index", "lo", "hi", "pending", "params")

    def __init__(self, index, lo, hi):
        self.index, self.lo, self.hi = index, lo, hi
        self.pending = 0
        self.params = []


class ShardedParameterService:
    def __init__(self, store: ParamStore, optimizer, group=None, bucket_mb: float = 64.0,
                 comm_dtype: torch.dtype = torch.float32, zero1: bool = True):
        self.store, self.opt, self.group = store, optimizer, group
        init = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if init else 1
        self.rank = dist.get_rank(group) if init else 0
        if comm_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError("comm_dtype must be float32 or bfloat16")
        self.comm_dtype = comm_dtype
        unit = self.world * ALIGN
        if store.total % unit:
            raise ValueError("ParamStore.total (%d) must be a multiple of world*%d: finalize(pad_to=%d)"
                             % (store.total, ALIGN, unit))
        cap = max(unit, _round_up(int(bucket_mb * 1024 * 1024 / store.grad.element_size()), unit))
        self.buckets: List[_Range] = []
        hi = store.total
        while hi > 0:
            lo = max(0, hi - cap)
            self.buckets.append(_Range(len(self.buckets), lo, hi))
            hi = lo
        self.buckets_of: Dict[int, List[_Range]] = {}
        for p in store.params:
            a, b = p.offset, p.offset + _round_up(p.numel)
            for bk in self.buckets:
                if a < bk.hi and b > bk.lo:
                    bk.params.append(p)
                    self.buckets_of.setdefault(p.index, []).append(bk)
        self.works = []
        self.a2a = []  # (bucket, send, recv, work) of in-flight bf16 pushes
        self.next_launch = 0
        self.sharded = zero1 and self.world > 1
        if self.sharded:
            optimizer.shard(self.owned_ranges)
        store.hooks.append(self._on_deposit)

    # ---------------------------------------------------------------- shards
    def shard(self, bk: _Range) -> Tuple[int, int]:
        n = (bk.hi - bk.lo) // self.world
        return bk.lo + self.rank * n, bk.lo + (self.rank + 1) * n

    @property
    def owned_ranges(self) -> List[Tuple[int, int]]:
        return [self.shard(b) for b in self.buckets]

    # ---------------------------------------------------------------- step protocol
    def begin_step(self):
        self.store.begin_step()
        for b in self.buckets:
            b.pending = sum(p.uses for p in b.params)
        self.works = []
        self.a2a = []
        self.next_launch = 0

    def _on_deposit(self, p):
        for b in self.buckets_of.get(p.index, ()):
            b.pending -= 1
        self._launch_ready()

    def _launch_ready(self):
        while self.next_launch < len(self.buckets) and self.buckets[self.next_launch].pending <= 0:
            self._push(self.buckets[self.next_launch])
            self.next_launch += 1

    def _push(self, b: _Range):
        if self.world == 1:
            return
        g = self.store.grad[b.lo:b.hi]
        if self.comm_dtype == torch.bfloat16:
            send = g.to(torch.bfloat16)
            recv = torch.empty_like(send)
            self.a2a.append((b, send, recv, dist.all_to_all_single(recv, send, group=self.group, async_op=True)))
        else:
            lo, hi = self.shard(b)  # in place: the output is this rank's slice of the input
            self.works.append(dist.reduce_scatter_tensor(self.store.grad[lo:hi], g, group=self.group,
                                                         async_op=True))

    def _finish_pushes(self):
        for w in self.works:
            w.wait()
        self.works = []
        for b, _send, recv, w in self.a2a:
            w.wait()
            lo, hi = self.shard(b)
            # fp32 accumulation of the world bf16 contributions, in rank order (deterministic)
            torch.sum(recv.view(self.world, hi - lo).float(), dim=0, out=self.store.grad[lo:hi])
        self.a2a = []

    def step(self, lr: Optional[float] = None):
        """Finish the pushes, update the owned shards, pull the new weights."""
        s = self.store
        for b in self.buckets:  # parameters never used this step contribute zero gradient
            if b.pending > 0:
                for p in b.params:
                    if not p.written:
                        p.grad.zero_()
                        p.written = True
                b.pending = 0
        self._launch_ready()
        self._finish_pushes()
        reduce = None
        if self.world > 1:
            def reduce(stats):
                dist.all_reduce(stats, group=self.group)
        self.opt.step(grad_scale=1.0 / self.world, lr=lr, ranges=self.owned_ranges, stats_reduce=reduce)
        if self.world > 1:
            # fp32 master (biases / norm parameters are read from it) then the bf16 copy locally
            self._pull(s.master)
            s.refresh_lowp()

    def _pull(self, buf: torch.Tensor):
        works = []
        for b in self.buckets:
            lo, hi = self.shard(b)
            works.append(dist.all_gather_into_tensor(buf[b.lo:b.hi], buf[lo:hi], group=self.group, async_op=True))
        for w in works:
            w.wait()

    # ---------------------------------------------------------------- checkpoint support
    def full_optimizer_state(self) -> Dict[str, torch.Tensor]:
        """Whole-model optimizer state (attribute -> full-size flat tensor) gathered from the owners; every
        rank must call it (collective). Unsharded: the optimizer's own tensors."""
        if not self.sharded:
            return {a: getattr(self.opt, a) for a in self.opt.STATE}
        out = {}
        for attr in self.opt.STATE:
            compact = getattr(self.opt, attr)
            full = torch.zeros(self.store.total, dtype=compact.dtype, device=compact.device)
            works = []
            for b, (lo, hi, off) in zip(self.buckets, self.opt.layout):
                works.append(dist.all_gather_into_tensor(full[b.lo:b.hi], compact[off:off + hi - lo],
                                                         group=self.group, async_op=True))
            for w in works:
                w.wait()
            out[attr] = full
        return out

    def sync_state(self):
        """Kept for callers of the unsharded service: gather the owners' state onto every rank."""
        if self.world == 1 or self.sharded:
            return
        for t in self.opt.state_tensors():
            self._pull(t)
