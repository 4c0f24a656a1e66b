"""Flat parameter store: the memory layout every other layer builds on.

MI355X-first design (288 GB HBM, 16-B vector kernels, RCCL buckets):

* ONE contiguous fp32 master buffer holds every parameter of a model, each in
  a 64-element-aligned slot (256 B), so any slot is a valid 16-B vector
  operand and the fused optimizer updates the whole model in one launch.
* ONE bf16 "low-precision" buffer mirrors the master for the weights that
  feed MFMA GEMM/conv kernels; the optimizer kernel writes it in the same
  pass that updates the master (no separate cast kernel).
* ONE gradient buffer (fp32 or bf16) with the same slot layout. Backward
  kernels deposit gradients straight into their slots (write on first use,
  accumulate on later uses), and the data-parallel reducer all-reduces
  contiguous ranges of this buffer in place: gradient buckets ARE slices of
  the flat buffer, there is no pack/unpack.
* A per-64-element decay mask selects weight decay inside the optimizer.

Custom autograd functions take ``store.anchor`` (a scalar leaf that requires
grad) as an extra input so their backward always runs -- even for the first
layer, whose input needs no gradient -- and return ``None`` for parameters,
whose gradients they deposit directly.
"""
from __future__ import annotations

import math
import os
from typing import Callable, Dict, List, Optional

import torch

ALIGN = 64
_DEBUG_PULL = os.environ.get("K8S_AMD_DEBUG_PULL") == "1"


def _round_up(n: int, a: int = ALIGN) -> int:
    return (n + a - 1) // a * a


class Param:
    """One parameter slot in a :class:`ParamStore`."""

    __slots__ = ("name", "shape", "numel", "offset", "decay", "lowp", "init", "index", "store",
                 "master", "half", "grad", "written", "uses")

    def __init__(self, store, index, name, shape, init, decay, lowp):
        self.store = store
        self.index = index
        self.name = name
        self.shape = tuple(int(s) for s in shape)
        self.numel = int(math.prod(self.shape)) if self.shape else 1
        self.init = init
        self.decay = decay
        self.lowp = lowp
        self.offset = -1
        self.master: Optional[torch.Tensor] = None
        self.half: Optional[torch.Tensor] = None
        self.grad: Optional[torch.Tensor] = None
        self.written = False
        self.uses = 1  # deposits expected per step (tied weights: >1); the reducer waits for all of them

    @property
    def weight(self) -> torch.Tensor:
        """The tensor compute kernels consume: bf16 copy for MFMA weights, fp32 master otherwise. With a bf16 pull in
        flight (ZeRO-1, parallel/ps.py) the first read of a weight waits for its bucket(s) only."""
        if self.store.pending:
            if _DEBUG_PULL and torch.cuda.current_stream() != torch.cuda.default_stream():
                raise RuntimeError("Param.weight read on a side stream while a bf16 pull is pending (%s)" % self.name)
            self.store.wait_param(self)
        return self.half if self.half is not None else self.master

    def __repr__(self):
        return "Param(%s, %s, off=%d)" % (self.name, self.shape, self.offset)


# --------------------------------------------------------------------------- initialisers
def init_kaiming_normal(fan_in: int, gain: float = math.sqrt(2.0)) -> Callable:
    std = gain / math.sqrt(max(1, fan_in))

    def f(t: torch.Tensor, g: torch.Generator):
        t.normal_(0.0, std, generator=g)

    return f


def init_normal(std: float) -> Callable:
    def f(t, g):
        t.normal_(0.0, std, generator=g)

    return f


def init_uniform(bound: float) -> Callable:
    def f(t, g):
        t.uniform_(-bound, bound, generator=g)

    return f


def init_const(v: float) -> Callable:
    def f(t, g):
        t.fill_(v)

    return f


class ZeroArena:
    """Per-step bump allocator of ZEROED fp32 scratch (e.g. the conv epilogue's BatchNorm statistics
    accumulators): one fill kernel per step at ``reset()`` instead of a tiny ``torch.zeros`` launch per layer.
    Slices handed out in a step stay valid until the next ``reset()`` (stream-ordered)."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.buf: Optional[torch.Tensor] = None
        self.off = 0
        self.dirty = 0

    def take(self, n: int) -> torch.Tensor:
        n = _round_up(n)
        if self.buf is None or self.off + n > self.buf.numel():
            cap = max(1 << 16, 2 * (self.off + n))
            self.buf = torch.zeros(cap, dtype=torch.float32, device=self.device)  # old slices keep the old buffer
            self.off = self.dirty = 0
        t = self.buf[self.off:self.off + n]
        self.off += n
        self.dirty = max(self.dirty, self.off)
        return t

    def reset(self):
        if self.buf is not None and self.dirty:
            self.buf[:self.dirty].zero_()
        self.off = self.dirty = 0


class ParamStore:
    """Owns the flat master / low-precision / gradient buffers of one model."""

    def __init__(self):
        self.params: List[Param] = []
        self.by_name: Dict[str, Param] = {}
        self.master: Optional[torch.Tensor] = None
        self.half: Optional[torch.Tensor] = None
        self.grad: Optional[torch.Tensor] = None
        self.decay_mask: Optional[torch.Tensor] = None
        self.anchor: Optional[torch.Tensor] = None
        self.total = 0
        self.hooks: List[Callable[[Param], None]] = []
        self.finalized = False
        # in-flight pull collectives (bucket index -> async work) and param index -> its buckets (parallel/ps.py)
        self.pending: Dict[int, object] = {}
        self.pending_of: Dict[int, list] = {}

    # ---- construction
    def new(self, name: str, shape, init: Callable, decay: bool = True, lowp: bool = True) -> Param:
        if self.finalized:
            raise RuntimeError("ParamStore already finalized")
        if name in self.by_name:
            raise ValueError("duplicate parameter name %r" % name)
        p = Param(self, len(self.params), name, shape, init, decay, lowp)
        self.params.append(p)
        self.by_name[name] = p
        return p

    def finalize(self, device, grad_dtype=torch.float32, seed: int = 0, lowp_dtype=torch.bfloat16,
                 pad_to: int = ALIGN):
        """Lay the parameters out in the flat buffers. ``pad_to`` rounds the total up (the sharded
        parameter service needs a multiple of world_size * ALIGN)."""
        device = torch.device(device)
        off = 0
        for p in self.params:
            p.offset = off
            off += _round_up(p.numel)
        self.total = _round_up(max(off, ALIGN), max(pad_to, ALIGN))
        self.master = torch.zeros(self.total, dtype=torch.float32, device=device)
        any_lowp = any(p.lowp for p in self.params)
        self.half = torch.zeros(self.total, dtype=lowp_dtype, device=device) if any_lowp else None
        self.grad = torch.zeros(self.total, dtype=grad_dtype, device=device)
        mask = torch.zeros(self.total // ALIGN, dtype=torch.uint8)
        gen = torch.Generator(device="cpu")
        gen.manual_seed(seed)
        for p in self.params:
            sl = slice(p.offset, p.offset + p.numel)
            t = torch.empty(p.shape, dtype=torch.float32)
            p.init(t, gen)
            self.master[sl].copy_(t.reshape(-1))
            p.master = self.master[sl].view(p.shape)
            p.grad = self.grad[sl].view(p.shape)
            if p.lowp:
                p.half = self.half[sl].view(p.shape)
            if p.decay:
                mask[p.offset // ALIGN: _round_up(p.offset + p.numel) // ALIGN] = 1
        self.decay_mask = mask.to(device)
        self.anchor = torch.zeros((), device=device, requires_grad=True)
        self.refresh_lowp()
        self.finalized = True
        return self

    # ---- pull bookkeeping (ZeRO-1 bf16 pull)
    def set_pending(self, works: Dict[int, object], buckets_of: Dict[int, list]):
        self.wait_pending()
        self.pending = dict(works)
        self.pending_of = buckets_of

    def wait_param(self, p: Param):
        """Order the current stream after the pull of ``p``'s bucket(s) (device-side wait for RCCL; blocking for
        gloo), once per bucket.

        Contract (the pull is lazily waited, ``parallel/ps.py``): every reader of the working copy goes through
        ``Param.weight``, and the first read of a bucket happens on the stream that later reads it -- the work is
        popped after ONE device-side wait, so a direct ``store.half`` / ``p.half`` read, or a first read on a side
        stream, would race the in-flight all-gather. ``ShardedParameterService._check_pull`` pins the wait itself;
        ``K8S_AMD_DEBUG_PULL=1`` makes ``Param.weight`` refuse a read from a non-default stream while a pull is
        pending."""
        for b in self.pending_of.get(p.index, ()):
            w = self.pending.pop(b.index, None)
            if w is not None:
                w.wait()

    def wait_pending(self):
        works, self.pending = self.pending, {}
        for w in works.values():
            w.wait()

    def refresh_lowp(self):
        if self.half is not None:
            self.half.copy_(self.master)

    # ---- gradient plumbing
    def begin_step(self):
        for p in self.params:
            p.written = False
        arena = self.__dict__.get("zero_arena")
        if arena is not None:
            arena.reset()

    def deposit(self, p: Param, g: torch.Tensor):
        """Write (first use in this step) or accumulate a parameter gradient into its slot."""
        g = g.reshape(p.shape)
        if p.written:
            p.grad.add_(g.to(p.grad.dtype))
            self._notify(p)
        else:
            p.grad.copy_(g)
            self.mark_written(p)

    def slot_for_write(self, p: Param) -> Optional[torch.Tensor]:
        """Slot a kernel may overwrite directly, or None if it must accumulate (already written)."""
        if p.written or p.grad.dtype != torch.float32:
            return None
        return p.grad

    def mark_written(self, p: Param):
        p.written = True
        self._notify(p)

    def _notify(self, p: Param):
        for h in self.hooks:
            h(p)

    def zero_unwritten(self):
        for p in self.params:
            if not p.written:
                p.grad.zero_()

    # ---- introspection / checkpoint
    def num_parameters(self) -> int:
        return sum(p.numel for p in self.params)

    def state_dict(self) -> Dict[str, torch.Tensor]:
        return {p.name: p.master.detach().clone() for p in self.params}

    def load_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True):
        missing = [p.name for p in self.params if p.name not in sd]
        if strict and missing:
            raise KeyError("missing parameters: %s" % missing[:8])
        with torch.no_grad():
            for p in self.params:
                if p.name in sd:
                    p.master.copy_(sd[p.name].reshape(p.shape))
        self.refresh_lowp()
