"""Fused flat-buffer optimizers (K7 SGD+momentum, K8 Adam/AdamW).

One kernel launch updates every parameter of the model: fp32 master, fp32
state, gradient (fp32 or bf16) and the bf16 working copy in a single pass
over HBM (see ``csrc/kernels/optim.hip``). Gradient averaging for data
parallelism and gradient clipping are folded into the kernel's scale
(device-side clip factor: no host sync, hipGraph-capturable).
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch

from k8s_amd.ops import reference as ref
from k8s_amd.ops._ext import load as _load_ext
from k8s_amd.parallel.flat import ParamStore


class _FlatOptimizer:
    # attribute -> state_dict key of every flat fp32 state buffer
    STATE: Dict[str, str] = {}

    def __init__(self, store: ParamStore, lr: float, weight_decay: float, max_grad_norm: Optional[float] = None):
        self.store = store
        self.lr = lr
        self.weight_decay = weight_decay
        self.max_grad_norm = max_grad_norm
        self.step_count = 0
        self.hyper: Optional[torch.Tensor] = None  # device [lr, step] (hipGraph replay), see use_device_hyper
        self.layout: Optional[List[Tuple[int, int, int]]] = None  # ZeRO-1 shard layout [(lo, hi, offset)]
        for attr in self.STATE:
            setattr(self, attr, torch.zeros_like(store.master))

    # ---- ZeRO-1: optimizer state only for the shards this rank owns
    def shard(self, ranges: Sequence[Tuple[int, int]]):
        """Keep state only for ``ranges`` of the flat buffers (the parameter service's owned shards), packed
        back to back: a rank then holds 1/world of the fp32 moments. ``step`` must be called with exactly
        these ranges afterwards."""
        layout, off = [], 0
        for lo, hi in ranges:
            layout.append((lo, hi, off))
            off += hi - lo
        self.layout = layout
        for attr in self.STATE:
            setattr(self, attr, torch.zeros(off, dtype=torch.float32, device=self.store.master.device))

    def _st(self, t: torch.Tensor, lo: int, hi: int) -> torch.Tensor:
        """State slice for flat range [lo, hi) (a sub-range of one owned shard when sharded)."""
        if self.layout is None:
            return t[lo:hi]
        for a, b, off in self.layout:
            if a <= lo and hi <= b:
                return t[off + lo - a: off + hi - a]
        raise ValueError("range [%d, %d) is not owned by this rank's optimizer shard" % (lo, hi))

    def state_numel(self) -> int:
        return sum(getattr(self, a).numel() for a in self.STATE)

    def use_device_hyper(self):
        """Kernels read lr (and Adam's step) from a device tensor instead of launch arguments, so a step
        captured in a hipGraph replays with the current schedule (``utils/graph.StepGraph``)."""
        if self.hyper is None:
            self.hyper = torch.zeros(2, dtype=torch.float32, device=self.store.master.device)
        return self.hyper

    def set_hyper(self, lr: float, step: int):
        self.hyper[0].fill_(float(lr))
        self.hyper[1].fill_(float(step))

    def prepare_replay(self, lr: float):
        """Host bookkeeping + device hyperparameters for one replay of a captured step (mirrors ``step``)."""
        raise NotImplementedError

    def _ranges(self, ranges: Optional[Sequence[Tuple[int, int]]]) -> List[Tuple[int, int]]:
        return [(0, self.store.total)] if ranges is None else list(ranges)

    def _views(self, lo: int, hi: int):
        s = self.store
        return (s.master[lo:hi], s.grad[lo:hi], None if s.half is None else s.half[lo:hi],
                s.decay_mask[lo // 64: hi // 64])

    def _clip(self, scale: float, ranges, stats_reduce: Optional[Callable] = None) -> Optional[torch.Tensor]:
        """Device-side clip factor from the gradient norm over ``ranges``; ``stats_reduce`` (e.g. an
        all-reduce) combines the [sum of squares, non-finite count] partials of a sharded update. (Also the step's
        first read of the gradients.)"""
        if not self.max_grad_norm:
            return None
        g = self.store.grad
        if g.is_cuda:
            C = _load_ext()
            stats = None
            for lo, hi in ranges:
                st = C.grad_sumsq(g[lo:hi])
                stats = st if stats is None else stats + st
            if stats_reduce is not None:
                stats_reduce(stats)
            # the clip test sees the *scaled* (averaged) gradient norm
            stats[0:1].mul_(scale * scale)
            return C.clip_factor(stats, float(self.max_grad_norm))
        stats = sum(ref.grad_sumsq(g[lo:hi]) for lo, hi in ranges)
        if stats_reduce is not None:
            stats_reduce(stats)
        norm = float(stats[0].sqrt()) * scale
        f = min(1.0, self.max_grad_norm / (norm + 1e-6)) if bool(stats[1] == 0) else 0.0
        return torch.tensor([f])

    def state_tensors(self):
        return [getattr(self, a) for a in self.STATE]

    def state_dict(self, full: Optional[Dict[str, torch.Tensor]] = None):
        """Flat state by key; when sharded pass ``full`` (attribute -> full-size tensor, gathered by the
        parameter service) to get checkpointable whole-model tensors."""
        d = {key: (full[attr] if full is not None else getattr(self, attr)) for attr, key in self.STATE.items()}
        d["step"] = self.step_count
        return d

    def load_state_dict(self, sd):
        """Accepts whole-model flat tensors (a checkpoint); a sharded optimizer keeps its owned slices."""
        for attr, key in self.STATE.items():
            src, dst = sd[key], getattr(self, attr)
            if self.layout is None:
                dst.copy_(src.reshape(-1)[:dst.numel()])
            else:
                src = src.reshape(-1)
                for lo, hi, off in self.layout:
                    dst[off:off + hi - lo].copy_(src[lo:hi])
        self.step_count = int(sd["step"])


class FusedSGD(_FlatOptimizer):
    STATE = {"mom": "momentum_buffer"}

    def __init__(self, store: ParamStore, lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=False,
                 max_grad_norm=None):
        super().__init__(store, lr, weight_decay, max_grad_norm)
        self.momentum = momentum
        self.nesterov = nesterov

    def step(self, grad_scale: float = 1.0, lr: Optional[float] = None, ranges=None, stats_reduce=None):
        """Update the flat buffers (or only ``ranges`` of them: the shards this rank owns)."""
        lr = self.lr if lr is None else lr
        ranges = self._ranges(ranges)
        clip = self._clip(grad_scale, ranges, stats_reduce)
        first = self.step_count == 0
        for lo, hi in ranges:
            p, g, h, mask = self._views(lo, hi)
            m = self._st(self.mom, lo, hi)
            if p.is_cuda:
                _load_ext().fused_sgd(p, m, g, h, mask, lr, self.momentum, self.weight_decay, grad_scale, clip,
                                      self.nesterov, first, self.hyper)
            else:
                ref.sgd(p, m, g, h, mask, lr, self.momentum, self.weight_decay, grad_scale, clip, self.nesterov,
                        first)
        self.step_count += 1

    def prepare_replay(self, lr: float):
        if self.step_count == 0:
            raise RuntimeError("capture after at least one eager step (momentum initialisation)")
        self.set_hyper(lr, self.step_count)
        self.step_count += 1



class FusedAdam(_FlatOptimizer):
    STATE = {"m1": "exp_avg", "m2": "exp_avg_sq"}

    def __init__(self, store: ParamStore, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01,
                 adamw=True, max_grad_norm=None):
        super().__init__(store, lr, weight_decay, max_grad_norm)
        self.b1, self.b2 = betas
        self.eps = eps
        self.adamw = adamw

    def step(self, grad_scale: float = 1.0, lr: Optional[float] = None, ranges=None, stats_reduce=None):
        lr = self.lr if lr is None else lr
        ranges = self._ranges(ranges)
        clip = self._clip(grad_scale, ranges, stats_reduce)
        self.step_count += 1
        for lo, hi in ranges:
            p, g, h, mask = self._views(lo, hi)
            a, b = self._st(self.m1, lo, hi), self._st(self.m2, lo, hi)
            if p.is_cuda:
                _load_ext().fused_adam(p, a, b, g, h, mask, lr, self.b1, self.b2, self.eps, self.weight_decay,
                                       grad_scale, clip, self.step_count, self.adamw, self.hyper)
            else:
                ref.adam(p, a, b, g, h, mask, lr, self.b1, self.b2, self.eps, self.weight_decay, grad_scale, clip,
                         self.step_count, self.adamw)

    def prepare_replay(self, lr: float):
        self.step_count += 1
        self.set_hyper(lr, self.step_count)

