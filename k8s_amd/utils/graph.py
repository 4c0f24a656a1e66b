"""Whole-step hipGraph capture: forward + backward + gradient reduction + fused optimizer as ONE graph launch.

The MI355X answer to a tracing compiler: after a few eager steps (kernel autotuning, workspace growth, lazy
library init), the step's kernel sequence is fixed -- same shapes, same buffers (flat parameter/gradient
store, zero arena, static batch) -- so it is captured once with ``torch.cuda.graph`` (hipStreamBeginCapture)
and replayed. Replay removes the per-kernel launch cost and the Python / autograd dispatch between
kernels; what still changes per step (learning rate, Adam's step for bias correction) is read by the
optimizer kernels from a device tensor (``_FlatOptimizer.use_device_hyper``) that is refreshed before each
replay.

Constraints (checked or documented):
* the body must not synchronise with the host (``.item()``, host-built device tensors) -- the framework's
  step does not: gradient clipping and loss scaling are device-side;
* inputs are static: a new batch is copied into the captured input tensors before replay;
* single process, or collectives explicitly allowed (``allow_collectives``): RCCL can be captured, but a
  captured all-reduce ties every rank to replaying in lock step, which the trainer guarantees only with
  the all-reduce strategy.
"""
from __future__ import annotations

from typing import Callable, Optional, Sequence

import torch


class StepGraph:
    def __init__(self, body: Callable[[Sequence[torch.Tensor], float], torch.Tensor], optimizer,
                 warmup: int = 2, allow_collectives: bool = False):
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1 and not allow_collectives:
            raise RuntimeError("StepGraph with world > 1 needs allow_collectives=True")
        self.body, self.opt, self.warmup = body, optimizer, warmup
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.static_inputs = None
        self.static_loss = None
        self.eager_steps = 0
        self.replays = 0

    def _hyper_for_next_step(self, lr):
        """Device [lr, step] for the step the next eager ``body`` call (which bumps step_count) performs."""
        saved = self.opt.step_count
        self.opt.prepare_replay(lr)
        self.opt.step_count = saved

    def _capture(self, inputs, lr):
        self.opt.use_device_hyper()
        self.static_inputs = tuple(inputs)
        # one more eager step on a side stream (the capture recipe: lazy per-stream state is created here)
        self._hyper_for_next_step(lr)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            loss = self.body(self.static_inputs, lr)  # this call's real step
            self.eager_steps += 1
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self._hyper_for_next_step(lr)
        saved = self.opt.step_count
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.static_loss = self.body(self.static_inputs, lr)
        self.opt.step_count = saved  # capture executed nothing
        self.graph = g
        return loss

    def __call__(self, inputs: Sequence[torch.Tensor], lr: float) -> torch.Tensor:
        if self.graph is None:
            if self.eager_steps < max(1, self.warmup):
                self.eager_steps += 1
                return self.body(inputs, lr)
            return self._capture(inputs, lr)
        for dst, src in zip(self.static_inputs, inputs):
            if dst.data_ptr() != src.data_ptr():
                dst.copy_(src, non_blocking=True)
        self.opt.prepare_replay(lr)
        self.graph.replay()
        self.replays += 1
        return self.static_loss
