"""Occupancy-grid rendering on the HIP kernels: a drop-in for the nerfacc 0.5.3 API
the reference uses — ``OccGridEstimator`` (``sampling``, ``update_every_n_steps``,
``mark_invisible_cells``), ``render_weight_from_density``, ``pack_info`` — and the integration of
``render_expert_occ`` (nerfs/ray_rendering.py:484-558) as ONE fused kernel (``render_packed``: weights,
``accumulate_along_rays`` of rgb / depth / acc and the background term together).

nerfacc's source is not in the image: the algorithms follow its published description, restated in
``oracle/occ_oracle.py`` (PARITY UNPINNED; checked by known-answer and property tests and against that
restatement).  Kernels: ``csrc/occ.hip``.
"""
from __future__ import annotations

import ctypes
from typing import Callable, Optional

import torch
import torch.nn as nn
from torch.autograd.function import once_differentiable

from ._lib import check, lib, need, ptr, stream


class NerfOccGrid(ctypes.Structure):
    _fields_ = [("levels", ctypes.c_int32), ("resolution", ctypes.c_int32), ("roi", ctypes.c_float * 6)]


def _addr(s):
    return ctypes.c_void_p(ctypes.addressof(s))


def exclusive_scan(x):
    """int32 (n,) -> int32 (n+1,) exclusive prefix sums (device)."""
    n = x.numel()
    out = torch.empty(n + 1, dtype=torch.int32, device=x.device)
    wsb = int(lib().nerf_scan_workspace_bytes(n))
    ws = torch.empty(wsb, dtype=torch.uint8, device=x.device)
    check(lib().nerf_exclusive_scan_i32(ptr(x), n, ptr(out), ptr(ws), wsb, stream()), "nerf_exclusive_scan_i32")
    return out


def pack_info(ray_indices, n_rays):
    """nerfacc.pack_info: (n_rays, 2) [start, count] — and the offsets (n_rays+1) used by the kernels."""
    ri = ray_indices.to(torch.int32).contiguous()
    counts = torch.empty(max(n_rays, 1), dtype=torch.int32, device=ri.device)
    check(lib().nerf_ray_counts(ptr(ri) if ri.numel() else None, ri.numel(), n_rays, ptr(counts), stream()),
          "nerf_ray_counts")
    counts = counts[:n_rays]
    offs = exclusive_scan(counts)
    return torch.stack([offs[:-1], counts], -1), offs


class _PackedRenderFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, rgb_sigma, t0, t1, offsets, bg):
        rs = rgb_sigma.contiguous().float()
        N = offsets.numel() - 1
        M = rs.shape[0]
        rgb = torch.empty((N, 3), dtype=torch.float32, device=rs.device)
        depth = torch.empty(N, dtype=torch.float32, device=rs.device)
        acc = torch.empty(N, dtype=torch.float32, device=rs.device)
        w = torch.empty(M, dtype=torch.float32, device=rs.device)
        bgc = None if bg is None else bg.contiguous().float()
        check(lib().nerf_packed_composite_fwd(ptr(rs), ptr(t0), ptr(t1), ptr(offsets), N, ptr(bgc), ptr(rgb),
                                              ptr(depth), ptr(acc), ptr(w), stream()), "nerf_packed_composite_fwd")
        ctx.save_for_backward(rs, t0, t1, offsets, bgc if bgc is not None else torch.empty(0), acc)
        ctx.has_bg = bgc is not None
        return rgb, depth, w, acc

    @staticmethod
    @once_differentiable
    def backward(ctx, g_rgb, g_depth, g_w, g_acc):
        rs, t0, t1, offs, bg, acc = ctx.saved_tensors
        bg = bg if ctx.has_bg else None
        N = offs.numel() - 1
        if g_rgb is None:
            g_rgb = torch.zeros(N, 3, device=rs.device)
        d = torch.empty_like(rs)
        f = lambda t: None if t is None else t.contiguous().float()
        check(lib().nerf_packed_composite_bwd(ptr(rs), ptr(t0), ptr(t1), ptr(offs), N, ptr(bg), ptr(f(g_rgb)),
                                              ptr(f(g_depth)), ptr(f(g_acc)), ptr(f(g_w)), ptr(d), stream()),
              "nerf_packed_composite_bwd")
        d_bg = None
        if ctx.has_bg and ctx.needs_input_grad[4]:
            d_bg = (1.0 - acc).unsqueeze(-1) * g_rgb
        return d, None, None, None, d_bg


def render_packed(rgb_sigma, t_starts, t_ends, offsets, bg=None):
    """render_weight_from_density + accumulate_along_rays for rgb / depth (t_mid) / acc, + (1-acc) bg."""
    return _PackedRenderFn.apply(rgb_sigma, t_starts.contiguous().float(), t_ends.contiguous().float(),
                                 offsets.to(torch.int32).contiguous(), bg)


def render_weight_from_density(t_starts, t_ends, sigmas, packed_info=None, ray_indices=None, n_rays=None):
    """nerfacc.render_weight_from_density -> (weights, trans, alphas) (no gradient: use render_packed)."""
    if packed_info is not None:
        offs = torch.cat([packed_info[:, 0], packed_info[-1:, 0] + packed_info[-1:, 1]]).to(torch.int32)
    else:
        _, offs = pack_info(ray_indices, n_rays)
    rs = torch.zeros(sigmas.shape[0], 4, device=sigmas.device)
    rs[:, 3] = sigmas.reshape(-1)
    with torch.no_grad():
        _, _, w, _ = render_packed(rs, t_starts, t_ends, offs)
    sdt = sigmas.reshape(-1) * (t_ends - t_starts)
    alphas = 1.0 - torch.exp(-sdt)
    trans = torch.where(alphas < 1.0, w / (alphas + (alphas == 0)), torch.zeros_like(w))
    return w, trans, alphas


class OccGridEstimator(nn.Module):
    """nerfacc.OccGridEstimator(roi_aabb, resolution, levels) on HIP kernels."""

    def __init__(self, roi_aabb, resolution: int = 128, levels: int = 1, **kwargs):
        super().__init__()
        roi = torch.as_tensor(roi_aabb, dtype=torch.float32).reshape(6)
        if isinstance(resolution, (list, tuple)):
            if len(set(resolution)) != 1:
                raise ValueError("anisotropic grid resolutions are not supported")
            resolution = resolution[0]
        self.levels = int(levels)
        self.resolution = int(resolution)
        self.cells_per_lvl = self.resolution ** 3
        c, h = (roi[:3] + roi[3:]) * 0.5, (roi[3:] - roi[:3]) * 0.5
        aabbs = torch.stack([torch.cat([c - h * 2 ** l, c + h * 2 ** l]) for l in range(self.levels)])
        self.register_buffer("aabbs", aabbs)
        self.register_buffer("occs", torch.zeros(self.levels * self.cells_per_lvl))
        self.register_buffer("binaries", torch.zeros(self.levels, self.resolution, self.resolution, self.resolution,
                                                     dtype=torch.uint8))
        self.register_buffer("_thre", torch.zeros(int(lib().nerf_occ_threshold_floats())), persistent=False)
        g = NerfOccGrid()
        g.levels, g.resolution = self.levels, self.resolution
        for i, v in enumerate(roi.tolist()):
            g.roi[i] = float(v)
        self.grid = g
        self.gen = 0  # bumped whenever a HIP kernel rewrites occs (torch's version counter does not see those)

    def _seed(self):
        return int(torch.randint(0, 2 ** 62, (1,)).item())

    def _march(self, rays, near_plane, far_plane, step, cone_angle, stratified, max_steps=8192):
        N = rays.shape[0]
        dev = rays.device
        counts = torch.empty(max(N, 1), dtype=torch.int32, device=dev)
        seed = self._seed()
        L = lib()
        args = (_addr(self.grid), ptr(self.binaries), ptr(rays), N, float(near_plane), float(far_plane), float(step),
                float(cone_angle), int(stratified), None, ctypes.c_uint64(seed), int(max_steps))
        check(L.nerf_occ_march(*args, ptr(counts), None, None, None, None, stream()), "nerf_occ_march(count)")
        offs = exclusive_scan(counts[:N])
        M = int(offs[-1].item())  # the packed size: one host read, as nerfacc's traversal
        ri = torch.empty(max(M, 1), dtype=torch.int32, device=dev)
        t0 = torch.empty(max(M, 1), dtype=torch.float32, device=dev)
        t1 = torch.empty(max(M, 1), dtype=torch.float32, device=dev)
        check(L.nerf_occ_march(*args, None, ptr(offs), ptr(ri), ptr(t0), ptr(t1), stream()), "nerf_occ_march(write)")
        return ri[:M], t0[:M], t1[:M], offs

    @torch.no_grad()
    def sampling_packed(self, rays_o, rays_d, sigma_fn: Optional[Callable] = None, near_plane: float = 0.0,
                        far_plane: float = 1e10, t_min=None, t_max=None, render_step_size: float = 1e-3,
                        early_stop_eps: float = 1e-4, alpha_thre: float = 0.0, stratified: bool = False,
                        cone_angle: float = 0.0):
        """sampling() that also returns the int32 ray offsets (N+1) the packed kernels use."""
        N = rays_o.shape[0]
        dev = rays_o.device
        tmin = t_min if t_min is not None else torch.zeros(N, device=dev)
        tmax = t_max if t_max is not None else torch.full((N,), 1e10, device=dev)
        rays = torch.cat([rays_o.float(), rays_d.float(), tmin.float().reshape(N, 1), tmax.float().reshape(N, 1)],
                         -1).contiguous()
        need(rays, "rays")
        ri, t0, t1, offs = self._march(rays, near_plane, far_plane, render_step_size, cone_angle, stratified)
        if (alpha_thre > 0.0 or early_stop_eps > 0.0) and sigma_fn is not None and ri.numel() > 0:
            alpha_thre = min(alpha_thre, float(self.occs.mean().item()))
            sig = sigma_fn(t0, t1, ri.long()).reshape(-1).contiguous().float()
            keep = torch.empty(ri.numel(), dtype=torch.int32, device=dev)
            check(lib().nerf_packed_visibility(ptr(t0), ptr(t1), ptr(sig), ptr(offs), N, float(early_stop_eps),
                                               float(alpha_thre), ptr(keep), stream()), "nerf_packed_visibility")
            pos = exclusive_scan(keep)
            Mk = int(pos[-1].item())
            ri2 = torch.empty(max(Mk, 1), dtype=torch.int32, device=dev)
            t02 = torch.empty(max(Mk, 1), dtype=torch.float32, device=dev)
            t12 = torch.empty(max(Mk, 1), dtype=torch.float32, device=dev)
            cnt = torch.zeros(max(N, 1), dtype=torch.int32, device=dev)
            check(lib().nerf_packed_compact(ptr(keep), ptr(pos), ri.numel(), ptr(ri), ptr(t0), ptr(t1), ptr(ri2),
                                            ptr(t02), ptr(t12), ptr(cnt), stream()), "nerf_packed_compact")
            ri, t0, t1, offs = ri2[:Mk], t02[:Mk], t12[:Mk], exclusive_scan(cnt[:N])
        return ri, t0, t1, offs

    @torch.no_grad()
    def sampling(self, rays_o, rays_d, sigma_fn=None, alpha_fn=None, near_plane=0.0, far_plane=1e10, t_min=None,
                 t_max=None, render_step_size=1e-3, early_stop_eps=1e-4, alpha_thre=0.0, stratified=False,
                 cone_angle=0.0):
        """nerfacc OccGridEstimator.sampling -> (ray_indices int64, t_starts, t_ends)."""
        if alpha_fn is not None:
            raise NotImplementedError("alpha_fn is not used by the reference (sigma_fn only)")
        ri, t0, t1, _ = self.sampling_packed(rays_o, rays_d, sigma_fn, near_plane, far_plane, t_min, t_max,
                                             render_step_size, early_stop_eps, alpha_thre, stratified, cone_angle)
        return ri.long(), t0, t1

    @torch.no_grad()
    def _update(self, step, occ_eval_fn, occ_thre=0.01, ema_decay=0.95, warmup_steps=256):
        dev = self.occs.device
        cpl = self.cells_per_lvl
        L = lib()
        if step < warmup_steps:
            cells = torch.arange(self.levels * cpl, dtype=torch.int32, device=dev)
        else:
            # uniform + occupied cells per level, drawn on the device (no nonzero / host read)
            n = cpl // 4
            flags = self.binaries.reshape(-1).to(torch.int32)
            pos = exclusive_scan(flags)
            occ_list = torch.empty(flags.numel(), dtype=torch.int32, device=dev)
            check(L.nerf_flag_compact(ptr(flags), ptr(pos), flags.numel(), ptr(occ_list), stream()),
                  "nerf_flag_compact")
            cells = torch.empty(self.levels * 2 * n, dtype=torch.int32, device=dev)
            check(L.nerf_occ_sample_cells(ptr(occ_list), ptr(pos), self.levels, cpl, n, ctypes.c_uint64(self._seed()),
                                          ptr(cells), stream()), "nerf_occ_sample_cells")
            # evaluate the drawn cells in cell order: neighbouring points then share hash-grid vertices at the
            # coarse levels, so the density's gathers hit the caches (the draws are a set; a duplicated cell's
            # update stays the last-writer-wins of the reference's index assignment)
            cells = torch.sort(cells).values
        n = cells.numel()
        x = torch.empty((n, 3), dtype=torch.float32, device=dev)
        check(lib().nerf_occ_cell_points(_addr(self.grid), ptr(cells), n, ctypes.c_uint64(self._seed()), ptr(x),
                                         stream()), "nerf_occ_cell_points")
        val = occ_eval_fn(x).reshape(-1).contiguous().float()
        self.gen += 1
        check(lib().nerf_occ_update(ptr(self.occs), ptr(cells), ptr(val), n, float(ema_decay), stream()),
              "nerf_occ_update")
        check(lib().nerf_occ_threshold(ptr(self.occs), self.occs.numel(), float(occ_thre), ptr(self._thre), stream()),
              "nerf_occ_threshold")
        check(lib().nerf_occ_binarize(ptr(self.occs), self.occs.numel(), ptr(self._thre), ptr(self.binaries),
                                      stream()), "nerf_occ_binarize")

    @torch.no_grad()
    def update_every_n_steps(self, step, occ_eval_fn, occ_thre=1e-2, ema_decay=0.95, warmup_steps=256, n=16):
        if not self.training:
            raise RuntimeError("update_every_n_steps should be called only during training")
        if step % n == 0:
            self._update(step, occ_eval_fn, occ_thre, ema_decay, warmup_steps)

    @torch.no_grad()
    def mark_invisible_cells(self, K, c2w, width, height, near_plane=0.0, chunk=32 ** 3):
        K = torch.as_tensor(K, dtype=torch.float32, device=self.occs.device).reshape(-1, 3, 3).contiguous()
        c2w = torch.as_tensor(c2w, dtype=torch.float32, device=self.occs.device)[:, :3, :4].contiguous()
        check(lib().nerf_occ_mark_invisible(_addr(self.grid), ptr(K), ptr(c2w), c2w.shape[0], int(width), int(height),
                                            float(near_plane), ptr(self.occs), stream()), "nerf_occ_mark_invisible")
        self.gen += 1
