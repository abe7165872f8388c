"""A train step captured once into a hipGraph and replayed (torch.cuda.CUDAGraph is hipGraph on ROCm).

The production container step (march -> union -> routing / dispatch -> 4 Instant-NGP experts
-> blend -> packed compositing -> MSE -> backward -> FlatAdam) is ~150 short launches per 4096-ray step; launched one
by one from Python the GPU idles between them.  With every size kept on the device (the
"device-sized" render of container.py) the step has no host read, so it can be captured: a replay submits the whole
step at once.  Measured on this ROCm (profiles/r06/a5, a6): a replay costs the host about what the
eager launches do and the early steps are GPU-bound, so the container bench keeps eager launches by default
(``--graph`` opts in).

What a replay cannot take from the host, the step reads from device memory:
  * the ray batch seed and the marching jitter seed: ``seed = base + step * mul`` with ``step`` an int64 counter in HBM
    (nerf_pick_pixels_dseed / nerf_occ_march_multi_staged_dseed), advanced by a node of the graph.  The batch draws
    are the eager step's (base = rank, mul = world: shard_seed); the marching jitter is a different counter stream
    than the eager path's host draws (same distribution);
  * the Adam step count (nerf_adam_dstep; FlatAdam.device_step);
  * the visibility thresholds (container.vis_thresholds: one persistent tensor updated in place).
What stays on the host, between replays: the occupancy-grid updates (every 16 steps, meta_container.py:368-372) —
``pre_fn`` runs them eagerly before a replay, in stream order, and refreshes the thresholds in place.  The packed
sample buffers have a fixed capacity while captured (container._DevSizes.freeze): a march past it keeps the first
samples of each (expert, ray) pair and is reported by ``frozen_report()``.

Single rank only (collectives are not captured here).
"""
from __future__ import annotations

from typing import Callable, Optional

import torch


class GraphedStep:
    """``step_fn()`` -> loss, run eagerly ``warmup`` times (allocator and cache warm-up), then captured; every later call
    replays.  ``pre_fn(step)`` runs eagerly before each call.

    Everything runs on the caller's current stream, which must not be the default stream, and the capture is taken on
    that same stream: the autograd graph's AccumulateGrad nodes (one per leaf, created by the eager steps before the
    capture and kept alive across steps) then sit on the capturing stream.  (With torch's side-stream recipe they sat on
    the default stream, so the backward forked the default stream into the capture; the graph instantiation at the
    end of that capture segfaulted in the HIP runtime on the full-size container step.)"""

    def __init__(self, step_fn: Callable[[], torch.Tensor], pre_fn: Optional[Callable[[int], None]] = None,
                 warmup: int = 2, before_capture: Optional[Callable[[], None]] = None):
        self.step_fn, self.pre_fn, self.warmup = step_fn, pre_fn, int(warmup)
        self.before_capture = before_capture
        self.graph = None
        self.out = None
        self.calls = 0

    def __call__(self, step: int) -> torch.Tensor:
        st = torch.cuda.current_stream()
        if st == torch.cuda.default_stream():
            raise RuntimeError("GraphedStep: run the train step on a non-default stream (torch.cuda.stream(...))")
        if self.pre_fn is not None:
            self.pre_fn(step)
        if self.graph is None and self.calls < self.warmup:
            out = self.step_fn()
            self.calls += 1
            return out
        if self.graph is None:
            if self.before_capture is not None:
                self.before_capture()
            torch.cuda.synchronize()
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph, stream=st):
                self.out = self.step_fn()
        self.graph.replay()
        self.calls += 1
        return self.out
