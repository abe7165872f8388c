"""Adam over flat parameter / gradient buffers on the HIP kernels — the optimiser of the reference's train
steps (``torch.optim.Adam`` over the named groups of common/utils.py:16-76, ``clip_grad_norm_`` of
pipelines/online_stage/runtime_adapt.py:305-307) for autograd-driven models (containers, occupancy rendering).

Every parameter of the given groups is re-pointed to a view of ONE flat fp32 buffer and its ``.grad`` to a view
of ONE flat gradient buffer (autograd accumulates into those views in place), so a step is two launches:
``nerf_grad_sqnorm`` (clip) and ``nerf_adam`` (per-group learning rates as segments), no host sync.  The
parameters are tagged ``_nerf_flat_grad``: the Instant-NGP hash-table backward then scatter-adds straight into
the table's ``.grad`` view (gradients of FlatAdam-owned parameters come from ``loss.backward()``).
"""
from __future__ import annotations

from typing import Dict, List

import torch

from . import kernels as K
from .dp import allreduce_flat


class FlatAdam:
    def __init__(self, groups: List[Dict], betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 grad_clip=1.0, world_size: int = 1):
        if len(groups) > 8:
            raise ValueError("at most 8 parameter groups (nerf_adam segments)")
        params = [p for g in groups for p in g["params"]]
        if len({id(p) for p in params}) != len(params):
            raise ValueError("a parameter appears in two groups")
        dev = params[0].device
        n = sum(p.numel() for p in params)
        self.flat = torch.empty(n, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(n, dtype=torch.float32, device=dev)
        self.m = torch.zeros(n, dtype=torch.float32, device=dev)
        self.v = torch.zeros(n, dtype=torch.float32, device=dev)
        self.partials = torch.empty(256, dtype=torch.float32, device=dev)
        self.seg_off, self.seg_lr = [0], []
        o = 0
        with torch.no_grad():
            for g in groups:
                for p in g["params"]:
                    k = p.numel()
                    self.flat[o:o + k].copy_(p.detach().reshape(-1).float())
                    p.data = self.flat[o:o + k].view_as(p)
                    p.grad = self.grad[o:o + k].view_as(p)
                    # HIP ops may accumulate this parameter's gradient in place (e.g. the hash-table scatter);
                    # use loss.backward(), not torch.autograd.grad, for parameters owned by FlatAdam
                    p._nerf_flat_grad = True
                    o += k
                self.seg_off.append(o)
                self.seg_lr.append(float(g["lr"]))
        self.params = params
        self.betas, self.eps, self.wd, self.grad_clip = betas, eps, weight_decay, grad_clip
        self.world_size = int(world_size)
        self.step_count = 0

    def zero_grad(self):
        self.grad.zero_()
        lo, hi = self.grad.data_ptr(), self.grad.data_ptr() + self.grad.numel() * 4
        for p in self.params:  # autograd must keep accumulating into the flat views
            if p.grad is None or not lo <= p.grad.data_ptr() < hi:
                raise RuntimeError("a parameter's .grad left the flat buffer (do not set grads to None)")

    def allreduce_grads(self):
        """Data parallel (as for the vanilla step): ONE all-reduce of the flat gradient buffer, then
        the mean over ranks (each rank's loss is its local-batch mean) — the gradient DDP would produce."""
        if self.world_size > 1:
            allreduce_flat(self.grad, self.world_size)
            self.grad.mul_(1.0 / self.world_size)

    def step(self):
        self.allreduce_grads()
        self.step_count += 1
        if self.grad_clip is not None and self.grad_clip > 0:
            K.grad_sqnorm(self.grad, self.partials)
            parts, mx = self.partials, float(self.grad_clip)
        else:
            parts, mx = None, 0.0
        K.adam(self.flat, self.grad, self.m, self.v, self.seg_off, self.seg_lr, self.step_count, self.betas, self.eps,
               self.wd, parts, mx)
