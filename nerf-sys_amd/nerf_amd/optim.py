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

_SHARD_ALIGN = 64  # floats: every rank's shard starts 256-B aligned (float4 Adam path)


class FlatAdam:
    """``shard=True`` (opt-in, world_size > 1) shards the optimiser: the flat gradient is
    reduce-scattered (each rank receives the rank-mean of ONE 1/N slice), each rank runs the clip and Adam on its
    slice only (m / v are slice-sized), and the updated parameter slices are all-gathered into every rank's flat
    buffer.  The bytes on the wire equal one all-reduce of the gradient; the optimiser's HBM traffic and m / v memory
    drop N-fold (at N = 8 the production container's 134 M-element Adam, 0.75 ms per step on one GPU, becomes ~0.1
    ms).  A touched-rows exchange of the hash tables does not pay at these batch sizes: one 4096-ray step touches
    ~61 % of an expert's 2^20-entry levels (tools/hash_requests.py), and an (index, value) pair costs
    more bytes than the dense value at that density.  shard=False (the default) keeps the replicated update (one
    all-reduce): the sharded collectives have only run emulated (gloo, two ranks on one GPU), never over RCCL, so
    they stay opt-in until an 8-GPU run covers them."""

    def __init__(self, groups: List[Dict], betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 grad_clip=1.0, world_size: int = 1, shard: bool = False, bucket_tables: bool = True,
                 bucket_min_numel: int = 1 << 20):
        if len(groups) > 8:
            raise ValueError("at most 8 parameter groups (nerf_adam segments)")
        params = [p for g in groups for p in g["params"]]
        if len({id(p) for p in params}) != len(params):
            raise ValueError("a parameter appears in two groups")
        dev = params[0].device
        n = sum(p.numel() for p in params)
        self.world_size = int(world_size)
        self.shard = bool(shard) and self.world_size > 1
        if self.shard:
            import torch.distributed as dist
            self.rank = dist.get_rank()
            S = -(-n // (self.world_size * _SHARD_ALIGN)) * _SHARD_ALIGN
            self.shard_size, self.shard_off = S, self.rank * S
            npad = S * self.world_size
            # gloo moves CUDA tensors for all_reduce only: the 1-GPU multi-process tests emulate the two collectives
            self._emulate = dist.get_backend() == "gloo" and dev.type == "cuda"
        else:
            npad = n
        self.n = n
        self.flat = torch.zeros(npad, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(npad, dtype=torch.float32, device=dev)
        ns = self.shard_size if self.shard else n
        self.m = torch.zeros(ns, dtype=torch.float32, device=dev)
        self.v = torch.zeros(ns, dtype=torch.float32, device=dev)
        if self.shard:
            self.gshard = torch.empty(ns, dtype=torch.float32, device=dev)
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
        self.step_count = 0
        # device_step(): the step count also lives in HBM and the step reads it there (nerf_adam_dstep), so a captured
        # hipGraph of the train step advances it per replay (graph_step.py)
        self.step_dev = None
        # Bucketed exchange (replicated update, world_size > 1): a parameter whose gradient a HIP backward writes in
        # place (the Instant-NGP hash tables, 0.54 GB for four experts) is its own bucket.  The backward calls
        # _bucket_ready when it has enqueued its write; the all-reduces are ISSUED in one fixed bucket order on every
        # rank (RCCL / gloo match collectives by issue order), so a bucket starts as soon as it and every bucket
        # before it in that order are ready, overlapping the rest of the backward.  Whether an expert's backward runs
        # at all depends on the rank's data (an expert with no samples skips it), so step() issues every bucket not
        # yet started, in the same order, then all-reduces the ranges outside the buckets — the same collective
        # sequence on every rank whatever its data.  The order is the reverse of the flat layout: autograd runs the
        # experts' backward in reverse of their forward, and the groups list the experts' tables in forward order.
        self.bucket_tables = bool(bucket_tables) and self.world_size > 1 and not self.shard
        self._slices = {}
        o = 0
        for p in params:
            self._slices[id(p)] = (o, p.numel())
            o += p.numel()
        self._inflight = []     # (handle, offset, numel) of buckets started in this step
        self.exchange_events = None
        self._ready = set()
        self._next = 0          # buckets [0, _next) of _buckets have been issued this step
        self._buckets = []
        if self.bucket_tables:
            self._buckets = [p for p in params if p.numel() >= int(bucket_min_numel)][::-1]
            for p in self._buckets:
                p._nerf_grad_ready = self._bucket_ready
        # the ranges no bucket covers, fixed at construction (identical on every rank)
        cov = sorted(self._slices[id(p)] for p in self._buckets)
        self._rest, lo = [], 0
        for o, k in cov + [(self.grad.numel(), 0)]:
            if o > lo:
                self._rest.append((lo, o))
            lo = max(lo, o + k)

    def _bucket_ready(self, p):
        if id(p) in self._ready:
            raise RuntimeError("bucketed exchange: a bucketed gradient was written twice in one step")
        self._ready.add(id(p))
        self._issue(all_buckets=False)

    def _issue(self, all_buckets):
        import torch.distributed as dist
        while self._next < len(self._buckets):
            q = self._buckets[self._next]
            if not all_buckets and id(q) not in self._ready:
                break
            o, k = self._slices[id(q)]
            self._inflight.append((dist.all_reduce(self.grad[o:o + k], async_op=True), o, k))
            self._next += 1

    def zero_grad(self):
        if self._inflight:
            raise RuntimeError("zero_grad with bucketed all-reduces in flight (call step() first)")
        self._ready.clear()
        self._next = 0
        self.grad.zero_()
        lo, hi = self.grad.data_ptr(), self.grad.data_ptr() + self.grad.numel() * 4
        for p in self.params:  # autograd must keep accumulating into the flat views
            if p.grad is None or not lo <= p.grad.data_ptr() < hi:
                raise RuntimeError("a parameter's .grad left the flat buffer (do not set grads to None)")

    def allreduce_grads(self):
        """Data parallel (as for the vanilla step): ONE all-reduce of the flat gradient buffer, then
        the mean over ranks (each rank's loss is its local-batch mean) — the gradient DDP would produce.  With
        buckets: the buckets not started during the backward, in the fixed order, then the uncovered ranges."""
        if self.world_size > 1:
            ev = self.exchange_events  # optional (start, end) torch.cuda.Events: the exchange's exposed tail
            if ev is not None:
                ev[0].record()
            if self._buckets:
                import torch.distributed as dist
                self._issue(all_buckets=True)
                for h, _, _ in self._inflight:
                    h.wait()  # orders the current stream after the collective (no host sync on RCCL)
                self._inflight = []
                self._ready.clear()
                self._next = 0
                for lo, hi in self._rest:
                    dist.all_reduce(self.grad[lo:hi])
            else:
                allreduce_flat(self.grad, self.world_size)
            if ev is not None:
                ev[1].record()
            self.grad.mul_(1.0 / self.world_size)

    def _step_sharded(self):
        import torch.distributed as dist
        S, off, W = self.shard_size, self.shard_off, self.world_size
        if self._emulate:
            full = self.grad.clone()
            dist.all_reduce(full)
            self.gshard.copy_(full[off:off + S])
        else:
            dist.reduce_scatter_tensor(self.gshard, self.grad)
        self.gshard.mul_(1.0 / W)
        if self.grad_clip is not None and self.grad_clip > 0:
            # the global norm: per-block partial sums of this slice, summed over ranks block by block
            K.grad_sqnorm(self.gshard, self.partials)
            dist.all_reduce(self.partials)
            parts, mx = self.partials, float(self.grad_clip)
        else:
            parts, mx = None, 0.0
        pshard = self.flat[off:off + S]
        seg = [min(max(o - off, 0), S) for o in self.seg_off]
        K.adam(pshard, self.gshard, self.m, self.v, seg, self.seg_lr, self.step_count, self.betas, self.eps,
               self.wd, parts, mx)
        if self._emulate:
            full = torch.zeros_like(self.flat)
            full[off:off + S].copy_(pshard)
            dist.all_reduce(full)  # every other rank's slice is 0 here: the sum is exact
            self.flat.copy_(full)
        else:
            dist.all_gather_into_tensor(self.flat, pshard)  # in place: pshard is this rank's slice of flat

    def device_step(self):
        """Keep the step count in device memory from now on (graph capture of the train step; world_size 1)."""
        if self.world_size > 1:
            raise ValueError("device-counted steps are for single-rank graph capture")
        if self.step_dev is None:
            self.step_dev = torch.full((1,), self.step_count, dtype=torch.int64, device=self.flat.device)
        return self.step_dev

    def step(self):
        self.step_count += 1
        if self.step_dev is not None:
            self.step_dev.add_(1)
        if self.shard:
            self._step_sharded()
            return
        self.allreduce_grads()
        if self.grad_clip is not None and self.grad_clip > 0:
            K.grad_sqnorm(self.grad, self.partials)
            parts, mx = self.partials, float(self.grad_clip)
        else:
            parts, mx = None, 0.0
        K.adam(self.flat, self.grad, self.m, self.v, self.seg_off, self.seg_lr,
               self.step_count if self.step_dev is None else self.step_dev, self.betas, self.eps, self.wd, parts, mx)
