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
    pull   = bf16 all-gather of the updated working-copy slices (the owner's
             optimizer kernel writes its slice of the bf16 copy in the same
             pass as the update), bucket by bucket and overlapped with the next
             forward: each bucket is waited for by the first layer that reads
             one of its weights (``Param.weight``). The fp32 master stays
             sharded -- each rank keeps only its owned slices current -- except
             for the parameters the kernels read in fp32 (norm / BN affines,
             biases: a few hundred K values), which come back in one small fp32
             all-gather. Checkpoints and PS snapshots gather the master on
             demand (``sync_master``). On the CPU (fp32 compute reads the
             master) the pull is the full fp32 all-gather.

Two push transports:

* ``comm_dtype=float32``: ``reduce_scatter_tensor`` in place (the output IS
  this rank's slice of the bucket).
* ``comm_dtype=bfloat16`` (Llama-scale models): each bucket is cast to bf16
  (``cast_bf16`` HIP kernel) and exchanged with ONE ``all_to_all_single`` --
  on a fully connected 8-GPU xGMI mesh that is a direct one-hop exchange over
  all 7 links -- and the world received slices are summed in fp32 on the
  owner (``slice_sum`` HIP kernel, rank order, one pass). Half the bytes of
  the fp32 push, with fp32 accumulation (the only rounding is each rank's
  contribution to bf16 once). On the GPU the sum is enqueued on a side stream
  behind the bucket's exchange the moment the exchange is issued (the stream
  waits on the collective device-side), so it overlaps the rest of backward
  instead of running after it.

This service is also the all-reduce strategy's ZeRO-1 mode (``--zero``,
``trainer/runner.py``): reduce-scatter + owner update + all-gather moves the
same bytes over xGMI as an all-reduce, and each rank runs the optimizer and
holds its fp32 state for 1/world of the model (Llama-3-8B: 96 GB of Adam
state and the 42 ms update pass, per rank, divided by 8).

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

import os
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from k8s_amd.ops._ext import load as _load_ext
from k8s_amd.parallel.flat import ALIGN, ParamStore, _round_up


class _Range:
    __slots__ = ("index", "lo", "hi", "pending", "params")

    def __init__(self, index, lo, hi):
        self.index, self.lo, self.hi = index, lo, hi
        self.pending = 0
        self.params = []


class ShardedParameterService:
    def __init__(self, store: ParamStore, optimizer, group=None, bucket_mb: float = 64.0,
                 comm_dtype: torch.dtype = torch.float32, zero1: bool = True, pull: str = "auto",
                 enabled: Optional[bool] = None):
        self.store, self.opt, self.group = store, optimizer, group
        init = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if init else 1
        self.rank = dist.get_rank(group) if init else 0
        # enabled: run the push / pull collectives (default: world > 1). ``enabled=True`` at world 1 drives the whole
        # transport through a one-rank process group -- how the GPU tests pin RCCL's stream semantics on one GPU
        self.active = (self.world > 1) if enabled is None else bool(enabled)
        if self.active and not init:
            raise ValueError("enabled=True needs an initialised process group")
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
        self.sharded = zero1 and self.active
        if self.sharded:
            optimizer.shard(self.owned_ranges)
        # bf16 pushes on the GPU: the owner's fp32 sum runs on this stream, device-ordered behind each exchange
        self.side = (torch.cuda.Stream(store.grad.device) if store.grad.is_cuda and self.active else None)
        self.side_busy = False
        self.fault_injection = os.environ.get("K8S_AMD_FAULT_TRANSPORT") == "1"  # see GradReducer.fault_injection
        self.fault = False
        self.pool = CommBufferPool()
        store.hooks.append(self._on_deposit)
        # pull: "lowp" = bf16 working copy + fp32 non-lowp parameters (GPU default), "fp32" = the full fp32 master
        if pull not in ("auto", "lowp", "fp32"):
            raise ValueError("pull must be auto, lowp or fp32")
        if pull == "auto":
            pull = "lowp" if (store.master.is_cuda and store.half is not None) else "fp32"
        if pull == "lowp" and store.half is None:
            raise ValueError("the bf16 pull needs a low-precision working copy")
        self.pull = pull if self.sharded else "fp32"
        self.master_stale = False  # non-owned master slices are not current (bf16 pull)
        if self.pull == "lowp":
            self._build_f32_pack()

    # ---------------------------------------------------------------- shards
    def shard(self, bk: _Range) -> Tuple[int, int]:
        n = (bk.hi - bk.lo) // self.world
        return bk.lo + self.rank * n, bk.lo + (self.rank + 1) * n

    @property
    def owned_ranges(self) -> List[Tuple[int, int]]:
        return [self.shard(b) for b in self.buckets]

    # ---------------------------------------------------------------- step protocol
    def begin_step(self):
        # (no wait for the last pull here: each bucket is waited by the first forward layer that reads it,
        # ``Param.weight``, and the rest by ``step`` before the optimizer rewrites the working copy)
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
        if not self.active:
            return
        g = self.store.grad[b.lo:b.hi]
        if self.comm_dtype == torch.bfloat16:
            send, recv = self.pool.acquire(b.index, b.hi - b.lo, g.device)
            cast_bf16(g, send)
            w = dist.all_to_all_single(recv, send, group=self.group, async_op=True)
            if self.side is not None:
                lo, hi = self.shard(b)
                with torch.cuda.stream(self.side):
                    w.wait()  # device-side: the side stream waits for this bucket's exchange, the host does not
                    nw = self.world - 1 if self.fault else self.world
                    _load_ext().slice_sum(recv[:nw * (hi - lo)], nw, self.store.grad[lo:hi], None)
                self.pool.release(b.index, self.side)  # no record_stream: see CommBufferPool
                self.side_busy = True
            else:
                self.a2a.append((b, send, recv, w))
        else:
            lo, hi = self.shard(b)  # in place: the output is this rank's slice of the input
            op = dist.ReduceOp.MAX if self.fault else dist.ReduceOp.SUM
            self.works.append(dist.reduce_scatter_tensor(self.store.grad[lo:hi], g, op=op, group=self.group,
                                                         async_op=True))

    def _finish_pushes(self):
        for w in self.works:
            w.wait()
        self.works = []
        for b, _send, recv, w in self.a2a:
            w.wait()
            lo, hi = self.shard(b)
            # fp32 accumulation of the world bf16 contributions, in rank order (deterministic)
            nw = self.world - 1 if self.fault else self.world
            slice_sum(recv[:nw * (hi - lo)], nw, self.store.grad[lo:hi])
        self.a2a = []
        if self.side_busy:
            torch.cuda.current_stream(self.store.grad.device).wait_stream(self.side)
            self.side_busy = False

    def self_check(self) -> Dict[str, object]:
        """Step-0 transport check of the push (outside any timed region): push bucket 0 with the configured
        transport and compare this rank's owned slice with a plain fp32 ``all_reduce`` of the same data
        (``ddp.transport_check``). Collective; the bucket's gradient range is restored afterwards."""
        from k8s_amd.parallel.ddp import transport_check

        if not self.active or not self.buckets:
            return {"ok": True, "transport": "none (world 1)"}
        b = self.buckets[0]

        def run():
            self.works, self.a2a = [], []
            self.fault = self.fault_injection  # armed for the check only, never for a training step
            try:
                self._push(b)
                self._finish_pushes()
            finally:
                self.fault = False

        name = "zero1-" + ("bf16" if self.comm_dtype == torch.bfloat16 else "fp32")
        res = transport_check(self.store.grad, b.lo, b.hi, self.shard(b), run, self.comm_dtype, self.group, name)
        if self.pull == "lowp":
            pull = self._check_pull(b)
            res["pull"] = pull
            res["ok"] = bool(res["ok"] and pull["ok"])
        return res

    def _check_pull(self, b: _Range) -> Dict[str, object]:
        """Step-0 check of the lazily-waited bf16 pull: every rank writes a rank-keyed pattern (exact in bf16) into
        its owned slice of bucket ``b``'s working copy, the bucket is all-gathered asynchronously and registered as
        pending exactly like ``_pull_lowp`` does, and the comparison kernel runs after the wait ``Param.weight``
        performs (the device-side ``Work.wait`` on the current stream). A missing or host-only wait, a wrong shard
        order or a wrong gather would leave other ranks' slices stale. The working copy is restored afterwards."""
        s = self.store
        half = s.half[b.lo:b.hi]
        save = half.clone()
        n = (b.hi - b.lo) // self.world
        idx = torch.arange(n, device=half.device)
        expect = torch.stack([(((idx * 7 + r * 131) % 509) - 254).float() / 64.0 for r in range(self.world)])
        expect = expect.reshape(-1).to(half.dtype)
        lo, hi = self.shard(b)
        half[lo - b.lo:hi - b.lo].copy_(expect[lo - b.lo:hi - b.lo])
        keep_pending, keep_of = s.pending, s.pending_of
        s.pending, s.pending_of = {}, {}
        work = dist.all_gather_into_tensor(half, half[lo - b.lo:hi - b.lo], group=self.group, async_op=True)
        s.pending, s.pending_of = {b.index: work}, self.buckets_of
        reader = next((p for p in b.params if p.lowp), None)
        if reader is not None:
            reader.weight  # noqa: B018 -- the lazy wait under test
        else:  # a bucket of fp32-read parameters only: the step's catch-all wait
            s.wait_pending()
        bad = torch.zeros(1, dtype=torch.float64, device=half.device)
        bad[0] = (half != expect).sum()
        dist.all_reduce(bad, group=self.group)
        s.wait_pending()
        s.pending, s.pending_of = keep_pending, keep_of
        half.copy_(save)
        wrong = int(bad.item())
        return {"ok": wrong == 0, "transport": "zero1-pull-bf16", "elements": int(b.hi - b.lo), "wrong": wrong}

    # ---------------------------------------------------------------- bf16 pull
    def _build_f32_pack(self):
        """Index plan of the small fp32 pull: the elements of the parameters the kernels read in fp32 (``lowp=False``),
        per bucket and owning rank, padded to the largest rank's count so one ``all_gather_into_tensor`` moves all of
        them: rank r sends ``master[send_idx]`` (its owned elements, padded with a repeat), everyone receives
        [world][total] and scatters the valid entries back (``recv_pos`` -> ``dst_idx``)."""
        s = self.store
        flag = torch.zeros(s.total, dtype=torch.bool)
        for p in s.params:
            if not p.lowp:
                flag[p.offset:p.offset + p.numel] = True
        per_rank = [[] for _ in range(self.world)]
        width = 0
        for b in self.buckets:
            n = (b.hi - b.lo) // self.world
            parts = [torch.nonzero(flag[b.lo + r * n:b.lo + (r + 1) * n]).flatten() + b.lo + r * n
                     for r in range(self.world)]
            m = max(len(t) for t in parts)
            for r in range(self.world):
                t = parts[r]
                pad = t[:1].repeat(m - len(t)) if len(t) else torch.full((m,), b.lo + r * n, dtype=torch.long)
                per_rank[r].append((torch.cat([t, pad]) if m else t, len(t)))
            width += m
        self.f32_width = width
        dev = s.master.device
        self.f32_send_idx = torch.cat([t for t, _ in per_rank[self.rank]]).to(dev) if width else None
        pos, dst = [], []
        for r in range(self.world):
            off = r * width
            for t, valid in per_rank[r]:
                pos.append(torch.arange(off, off + valid))
                dst.append(t[:valid])
                off += len(t)
        self.f32_recv_pos = torch.cat(pos).to(dev) if width else None
        self.f32_dst_idx = torch.cat(dst).to(dev) if width else None

    def _pull_lowp(self):
        """The fp32 all-gather of the non-lowp parameters (a few hundred K values, waited here), then the bf16
        all-gather of every bucket's working copy (async; waited lazily by ``Param.weight``, the rest in ``step``).

        Order matters on RCCL: one communicator runs its collectives in issue order, so the small fp32 gather goes
        FIRST (waiting on it after the bf16 buckets would wait for all of them), and the bf16 buckets go in
        ascending offset order -- ``self.buckets`` is built from the END of the flat buffer, so that is
        ``reversed(self.buckets)``: the first layers' weights arrive first and the next forward starts behind the
        first bucket instead of the whole pull."""
        s = self.store
        if self.f32_width:
            send = s.master.index_select(0, self.f32_send_idx)
            recv = torch.empty(self.world * self.f32_width, dtype=send.dtype, device=send.device)
            dist.all_gather_into_tensor(recv, send, group=self.group)
            s.master.index_copy_(0, self.f32_dst_idx, recv.index_select(0, self.f32_recv_pos))
        pending = {}
        for b in reversed(self.buckets):  # ascending offsets: the first layers' weights are requested first
            lo, hi = self.shard(b)
            pending[b.index] = dist.all_gather_into_tensor(s.half[b.lo:b.hi], s.half[lo:hi], group=self.group,
                                                           async_op=True)
        s.set_pending(pending, self.buckets_of)
        self.master_stale = True
        self.pull_order = [b.index for b in reversed(self.buckets)]

    def sync_master(self):
        """Make the whole fp32 master current on every rank (checkpoints, PS snapshots, end-of-run checks):
        the full fp32 all-gather the bf16 pull skips every step. Collective."""
        if self.active and self.master_stale:
            self.store.wait_pending()
            self._pull(self.store.master)
            self.master_stale = False

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
        # buckets of the last pull that no forward layer read: the optimizer below rewrites their owned slices
        self.store.wait_pending()
        reduce = None
        if self.active:
            def reduce(stats):
                dist.all_reduce(stats, group=self.group)
        self.opt.step(grad_scale=1.0 / self.world, lr=lr, ranges=self.owned_ranges, stats_reduce=reduce)
        if self.active:
            if self.pull == "lowp":
                self._pull_lowp()
            else:
                # fp32 master (the CPU's fp32 compute reads it) then the bf16 copy locally
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
    def gather_state(self, dst: int = 0) -> Optional[Dict[str, torch.Tensor]]:
        """Whole-model optimizer state (attribute -> fp32 [total] tensor in host memory) on rank ``dst``, None on
        the others; every rank must call it (collective). Bucket by bucket: the owners' slices are gathered into
        one bucket-sized device buffer on ``dst`` and copied into (pinned) host memory, so no rank ever holds a
        full-size device copy of a state tensor (an all-gather of every state onto every rank was
        ~64 GB per GPU for Llama-3-8B). Unsharded: the optimizer's own tensors, copied to host on ``dst``."""
        if not self.sharded:
            if self.rank != dst:
                return None
            return {a: getattr(self.opt, a).detach().to("cpu") for a in self.opt.STATE}
        dev = self.store.master.device
        out = {} if self.rank == dst else None
        stage = None
        for attr in self.opt.STATE:
            compact = getattr(self.opt, attr)
            if out is not None:
                # pageable host memory: a page-locked allocation of the whole state per call (Llama-3-8B with Adam:
                # ~64 GB) cost more than the faster copies it buys, and ps_vars keeps the result until its push ends
                out[attr] = torch.empty(self.store.total, dtype=torch.float32)
            for b, (lo, hi, off) in zip(self.buckets, self.opt.layout):
                n = hi - lo
                glist = None
                if out is not None:
                    if stage is None or stage.numel() < b.hi - b.lo:
                        stage = torch.empty(b.hi - b.lo, dtype=torch.float32, device=dev)
                    glist = [stage[r * n:(r + 1) * n] for r in range(self.world)]
                dist.gather(compact[off:off + n], glist, dst=dst, group=self.group)
                if out is not None:
                    out[attr][b.lo:b.hi].copy_(stage[:b.hi - b.lo])
        return out

    def scatter_state(self, full: Optional[Dict[str, torch.Tensor]], src: int = 0):
        """Inverse of ``gather_state``: rank ``src`` holds whole-model state tensors (host or device, attribute
        -> [>= total]); every rank receives only the slices it owns, bucket by bucket (collective)."""
        if not self.sharded:
            raise RuntimeError("scatter_state is for the sharded (ZeRO-1) optimizer")
        dev = self.store.master.device
        stage = None
        for attr in self.opt.STATE:
            compact = getattr(self.opt, attr)
            for b, (lo, hi, off) in zip(self.buckets, self.opt.layout):
                n = hi - lo
                slist = None
                if self.rank == src:
                    if stage is None or stage.numel() < b.hi - b.lo:
                        stage = torch.empty(b.hi - b.lo, dtype=torch.float32, device=dev)
                    stage[:b.hi - b.lo].copy_(full[attr].reshape(-1)[b.lo:b.hi])
                    slist = [stage[r * n:(r + 1) * n] for r in range(self.world)]
                dist.scatter(compact[off:off + n], slist, src=src, group=self.group)

    def sync_state(self):
        """Kept for callers of the unsharded service: gather the owners' state onto every rank."""
        if not self.active or self.sharded:
            return
        for t in self.opt.state_tensors():
            self._pull(t)


class CommBufferPool:
    """Per-bucket bf16 send / receive buffers of the bf16 transports, allocated once and reused every step.

    The transient form (a fresh ``torch.empty`` per bucket per step, kept alive for the side stream with
    ``Tensor.record_stream``) makes the caching allocator hold every freed block until the HOST has seen an event
    recorded on the side stream at free time: with the host a whole step ahead of the GPU, each step's buckets are
    allocated anew, and under memory pressure through the out-of-memory release path (15x slower in the round-5
    side-stream weight-gradient experiment, ``profiles/r05_notes.md``). Here a bucket's buffers live as long as the
    reducer, and reuse is ordered on the device: ``release`` records an event on the stream of the buffers' last use
    (the side stream, after the all-gather / owner sum that read them); ``acquire`` makes the acquiring stream wait
    for it. Memory: one bf16 copy of the gradient per buffer kind -- the transient form held the same amount at the
    end of backward, when every bucket is in flight. ``reserved_bytes`` is what the memory test pins."""

    def __init__(self):
        self.bufs: Dict[Tuple[int, str], torch.Tensor] = {}
        self.free_ev: Dict[int, torch.cuda.Event] = {}

    def acquire(self, key: int, n: int, device, kinds=("send", "recv")) -> List[torch.Tensor]:
        out = []
        for k in kinds:
            t = self.bufs.get((key, k))
            if t is None or t.numel() != n:
                t = torch.empty(n, dtype=torch.bfloat16, device=device)
                self.bufs[(key, k)] = t
            out.append(t)
        ev = self.free_ev.pop(key, None)
        if ev is not None:
            torch.cuda.current_stream(device).wait_event(ev)
        return out

    def release(self, key: int, stream) -> None:
        ev = torch.cuda.Event()
        ev.record(stream)
        self.free_ev[key] = ev

    @property
    def reserved_bytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in self.bufs.values())


def cast_bf16(g: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fp32 -> bf16 copy of a gradient bucket (HIP kernel on the GPU), into ``out`` when given."""
    if g.is_cuda:
        return _load_ext().cast_bf16(g.contiguous(), out)
    if out is not None:
        out.copy_(g)
        return out
    return g.to(torch.bfloat16)


def slice_sum(recv: torch.Tensor, world: int, out: Optional[torch.Tensor] = None,
              out_bf: Optional[torch.Tensor] = None):
    """Rank-order fp32 sum of the ``world`` bf16 chunks of ``recv`` into ``out`` (fp32) and/or ``out_bf``."""
    if recv.is_cuda:
        _load_ext().slice_sum(recv, world, out, out_bf)
        return
    s = recv.view(world, -1).float().sum(0)
    if out is not None:
        out.copy_(s)
    if out_bf is not None:
        out_bf.copy_(s.to(torch.bfloat16))
