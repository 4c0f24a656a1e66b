"""Parameter-server data parallelism the MI355X way.

The reference's TfJobs place variables on ``/job:ps`` tasks and every worker
pushes gradients to / pulls parameters from them over gRPC
(`/root/reference/examples/tf_job.yaml:1-24`, ``replica_device_setter`` in
the TF programs it runs). Translating that literally -- a CPU/GPU process per
PS shard receiving every worker's gradient over TCP -- would put the whole
update on a few links. Here the *parameter service is sharded over the
compute ranks* and the push/pull are RCCL collectives over xGMI:

    push  = reduce-scatter of each gradient bucket: rank r receives the summed
            gradient of its 1/world slice of the bucket
    update= the fused SGD/Adam kernel runs on the owned slices only
            (fp32 master + optimizer state are "owned" -- the PS role)
    pull  = all-gather of the updated fp32 master slices (biases and norm
            parameters are read from it), bf16 working copy refreshed locally

Per step that moves the same bytes as one all-reduce (reduce-scatter +
all-gather), but the optimizer touches 1/world of the state, and fp32
master/optimizer state could be dropped on non-owner ranks (ZeRO-1). Buckets
are fixed ranges of the flat buffer taken from the END (backward produces
the last layers' gradients first), each a multiple of world*64 elements, so
a bucket's push starts as soon as every parameter overlapping it has
deposited -- overlapped with the rest of backward like ``GradReducer``.

PS replicas of a TfJob (``--job_name ps``) still run the default PS server
(rendezvous / liveness / shutdown); ``num_shards`` = compute world.
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
    def __init__(self, store: ParamStore, optimizer, group=None, bucket_mb: float = 64.0):
        self.store, self.opt, self.group = store, optimizer, group
        init = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if init else 1
        self.rank = dist.get_rank(group) if init else 0
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
        self.backend = dist.get_backend(group) if init else None
        self.works = []
        self.next_launch = 0
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
        lo, hi = self.shard(b)
        if self.backend == "nccl":
            # in place: the output is this rank's slice of the input (RCCL allows recv = send + rank*count)
            self.works.append(dist.reduce_scatter_tensor(self.store.grad[lo:hi], g, group=self.group,
                                                         async_op=True))
        else:  # gloo has no reduce-scatter: same result through an all-reduce
            self.works.append(dist.all_reduce(g, group=self.group, async_op=True))

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
        for w in self.works:
            w.wait()
        self.works = []
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
            src = buf[lo:hi] if self.backend == "nccl" else buf[lo:hi].clone()  # RCCL: in-place all-gather
            works.append(dist.all_gather_into_tensor(buf[b.lo:b.hi], src, group=self.group, async_op=True))
        for w in works:
            w.wait()

    def sync_state(self):
        """Gather the owners' optimizer state onto every rank (e.g. before a checkpoint); between calls
        only the owned slices of it are current."""
        if self.world == 1:
            return
        for t in self.opt.state_tensors():
            self._pull(t)
