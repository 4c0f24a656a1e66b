"""Fused flat-buffer optimizers (K7 SGD+momentum, K8 Adam/AdamW).

One kernel launch updates every parameter of the model: fp32 master, fp32
state, gradient (fp32 or bf16) and the bf16 working copy in a single pass
over HBM (see ``csrc/kernels/optim.hip``). Gradient averaging for data
parallelism and gradient clipping are folded into the kernel's scale
(device-side clip factor: no host sync, hipGraph-capturable).
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import torch

from k8s_amd.ops import reference as ref
from k8s_amd.ops._ext import load as _load_ext
from k8s_amd.parallel.flat import ParamStore


class _FlatOptimizer:
    def __init__(self, store: ParamStore, lr: float, weight_decay: float, max_grad_norm: Optional[float] = None):
        self.store = store
        self.lr = lr
        self.weight_decay = weight_decay
        self.max_grad_norm = max_grad_norm
        self.step_count = 0
        self.hyper: Optional[torch.Tensor] = None  # device [lr, step] (hipGraph replay), see use_device_hyper

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
        all-reduce) combines the [sum of squares, non-finite count] partials of a sharded update."""
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

    def state_dict(self):
        raise NotImplementedError

    def load_state_dict(self, sd):
        raise NotImplementedError


class FusedSGD(_FlatOptimizer):
    def __init__(self, store: ParamStore, lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=False,
                 max_grad_norm=None):
        super().__init__(store, lr, weight_decay, max_grad_norm)
        self.momentum = momentum
        self.nesterov = nesterov
        self.mom = torch.zeros_like(store.master)

    def step(self, grad_scale: float = 1.0, lr: Optional[float] = None, ranges=None, stats_reduce=None):
        """Update the flat buffers (or only ``ranges`` of them: the shards this rank owns)."""
        lr = self.lr if lr is None else lr
        ranges = self._ranges(ranges)
        clip = self._clip(grad_scale, ranges, stats_reduce)
        first = self.step_count == 0
        for lo, hi in ranges:
            p, g, h, mask = self._views(lo, hi)
            m = self.mom[lo:hi]
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

    def state_tensors(self):
        return [self.mom]

    def state_dict(self):
        return {"momentum_buffer": self.mom, "step": self.step_count}

    def load_state_dict(self, sd):
        self.mom.copy_(sd["momentum_buffer"])
        self.step_count = int(sd["step"])


class FusedAdam(_FlatOptimizer):
    def __init__(self, store: ParamStore, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01,
                 adamw=True, max_grad_norm=None):
        super().__init__(store, lr, weight_decay, max_grad_norm)
        self.b1, self.b2 = betas
        self.eps = eps
        self.adamw = adamw
        self.m1 = torch.zeros_like(store.master)
        self.m2 = torch.zeros_like(store.master)

    def step(self, grad_scale: float = 1.0, lr: Optional[float] = None, ranges=None, stats_reduce=None):
        lr = self.lr if lr is None else lr
        ranges = self._ranges(ranges)
        clip = self._clip(grad_scale, ranges, stats_reduce)
        self.step_count += 1
        for lo, hi in ranges:
            p, g, h, mask = self._views(lo, hi)
            a, b = self.m1[lo:hi], self.m2[lo:hi]
            if p.is_cuda:
                _load_ext().fused_adam(p, a, b, g, h, mask, lr, self.b1, self.b2, self.eps, self.weight_decay,
                                       grad_scale, clip, self.step_count, self.adamw, self.hyper)
            else:
                ref.adam(p, a, b, g, h, mask, lr, self.b1, self.b2, self.eps, self.weight_decay, grad_scale, clip,
                         self.step_count, self.adamw)

    def prepare_replay(self, lr: float):
        self.step_count += 1
        self.set_hyper(lr, self.step_count)

    def state_tensors(self):
        return [self.m1, self.m2]

    def state_dict(self):
        return {"exp_avg": self.m1, "exp_avg_sq": self.m2, "step": self.step_count}

    def load_state_dict(self, sd):
        self.m1.copy_(sd["exp_avg"])
        self.m2.copy_(sd["exp_avg_sq"])
        self.step_count = int(sd["step"])
