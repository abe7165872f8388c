"""Fused train step of the Instant-NGP expert on flat buffers.

The reference's plain train loop (pipelines/online_stage/runtime_adapt.py:278-313) with the production
expert (MetaNGP, models/inr/meta_ngp.py; nerf_runner.py:103-121 hash config) on the stratified renderer
(ray_rendering.py:290-345, ``--ray_samples 96``, common/args.py:96):

  rays -> sample_stratified -> build_xd -> hash_encode -> ngp_fwd (fused MLP) -> composite_fwd(+loss)
  -> composite_bwd -> ngp_bwd (recompute + backward, d_enc) -> hash_encode_bwd (scatter into d_table)
  -> [RCCL all_reduce of the flat gradient] -> grad_sqnorm -> Adam (groups encoding / sigma / color with
     encoding_lr / sigma_lr / color_lr, common/args.py:115-119)

Parameters live in ONE flat fp32 buffer [hash table | packed MLP]; no host synchronisation in the step.
"""
from __future__ import annotations

import torch

from . import kernels as K
from . import ngp as G
from .dp import allreduce_flat, inv_count as _inv_count

_CS = ("linear", "srgb", "identity")


class NGPTrainer:
    def __init__(self, model: "G.InstantNGP", *, n_samples: int = 96, lr_encoding: float = 1e-2,
                 lr_sigma: float = 2e-3, lr_color: float = 2e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, grad_clip=1.0, color_space: str = "linear", bg: str = "white",
                 world_size: int = 1, device="cuda"):
        self.model = model
        self.device = torch.device(device)
        tab = model.xyz_encoder.hash_table
        self.F = model.xyz_encoder.features_per_level
        self.T = tab.numel()
        self.P = model.layout.total
        with torch.no_grad():
            self.params = torch.cat([tab.detach().reshape(-1).to(self.device),
                                     model.packed().detach().to(self.device)]).contiguous()
        self.gbuf = torch.zeros(self.T + self.P + 4, dtype=torch.float32, device=self.device)
        self.grads = self.gbuf[: self.T + self.P]
        self.loss_buf = self.gbuf[self.T + self.P: self.T + self.P + 1]
        self.m = torch.zeros_like(self.params)
        self.v = torch.zeros_like(self.params)
        self.partials = torch.empty(256, dtype=torch.float32, device=self.device)
        cs = self.T + model.layout.color_start
        self.seg_off = [0, self.T, cs, self.T + self.P]
        self.seg_lr = [lr_encoding, lr_sigma, lr_color]
        self.S = n_samples
        self.betas, self.eps, self.wd, self.grad_clip = betas, eps, weight_decay, grad_clip
        if color_space not in _CS:
            raise ValueError(f"Invalid color_space={color_space!r}")
        self.color_space = color_space
        if bg not in ("white", "black", "none"):
            raise ValueError("trainer background must be 'white', 'black' or 'none'")
        self.bg_policy = bg
        self.world_size = world_size
        self.step_count = 0
        self._bg = {}
        self.events = None  # optional list of (name, start, end) torch events for the next step

    def table(self):
        return self.params[: self.T].view(-1, self.F)

    def w(self):
        return self.params[self.T:]

    def _background(self, n):
        if self.bg_policy == "none":
            return None
        b = self._bg.get(n)
        if b is None:
            b = torch.full((n, 3), 1.0 if self.bg_policy == "white" else 0.0, device=self.device)
            self._bg[n] = b
        return b

    def _ev(self, name):
        if self.events is None:
            return None
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        self.events.append((name, e0, e1))
        e0.record()
        return e1

    @staticmethod
    def _end(e):
        if e is not None:
            e.record()

    def step(self, rays: torch.Tensor, gt: torch.Tensor, seed: int, u_strat=None) -> torch.Tensor:
        m = self.model
        N = rays.shape[0]
        bg = self._background(N)
        inv_count = _inv_count(N, self.world_size)
        self.gbuf.zero_()
        t = K.sample_stratified(rays, self.S, True, u_strat, seed)
        xd = K.build_xd(rays, t)
        e = self._ev("fwd_enc")  # hash encoding + MLP forward in one launch (production shape)
        fused = G.ngp_fwd_enc(m.net_struct, m.xyz_encoder.grid, self.table(), self.w(), xd, m._aabb_host, m._eps)
        self._end(e)
        if fused is not None:
            rs, enc = fused
        else:
            e = self._ev("hash_fwd")
            enc = G.hash_encode(m.xyz_encoder.grid, self.table(), xd, m._aabb_host, m._eps)
            self._end(e)
            e = self._ev("mlp_fwd")
            rs = G.ngp_fwd(m.net_struct, self.w(), enc, xd)
            self._end(e)
        _, _, _, _, _, drgb = K.composite_fwd(rs, t, bg, 1.0, gt=gt, color_space=self.color_space,
                                              inv_count=inv_count, loss_sum=self.loss_buf)
        d_rs = K.composite_bwd(rs, t, bg, drgb)
        e = self._ev("bwd_hash")  # MLP backward + table scatter in one launch (production shape)
        fused = G.ngp_bwd_hash(m.net_struct, m.xyz_encoder.grid, self.w(), enc, xd, d_rs,
                               self.grads[: self.T].view(-1, self.F), m._aabb_host, m._eps,
                               d_w=self.grads[self.T:])
        self._end(e)
        if fused is None:
            e = self._ev("mlp_bwd")
            d_enc, _ = G.ngp_bwd(m.net_struct, self.w(), enc, xd, d_rs, d_w=self.grads[self.T:])
            self._end(e)
            e = self._ev("hash_bwd")
            G.hash_encode_bwd(m.xyz_encoder.grid, xd, d_enc, 0, m._aabb_host, m._eps,
                              d_table=self.grads[: self.T].view(-1, self.F))
            self._end(e)
        allreduce_flat(self.gbuf, self.world_size)
        self.step_count += 1
        if self.grad_clip is not None and self.grad_clip > 0:
            K.grad_sqnorm(self.grads, self.partials)
            parts, mx = self.partials, float(self.grad_clip)
        else:
            parts, mx = None, 0.0
        e = self._ev("adam")
        K.adam(self.params, self.grads, self.m, self.v, self.seg_off, self.seg_lr, self.step_count, self.betas,
               self.eps, self.wd, parts, mx)
        self._end(e)
        return self.loss_buf

    @torch.no_grad()
    def sync_to_modules(self):
        m = self.model
        m.xyz_encoder.hash_table.copy_(self.table())
        w = self.w()
        for n, idx in zip(m.layout.names, torch.split(m.layout.index.to(w.device),
                                                      [p.numel() for p in m.tensors()])):
            dict(m.named_parameters())[n].copy_(w[idx].view_as(dict(m.named_parameters())[n]))
