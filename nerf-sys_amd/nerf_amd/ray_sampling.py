"""Ray generation on the GPU — mirrors nerfs/ray_sampling.py (+ nerfs/scene_box.py) of the reference.

Same names, argument meaning and error behaviour:
  get_ray_directions (ray_sampling.py:111-136), get_rays (:50-108), clamp_rays_near_far (:139-176),
  pack_rays / unpack_rays (:28-46), SceneBox.ray_aabb_intersect (scene_box.py:45-107);
plus ndc_rays (canonical forward-facing NDC, absent in the reference) for the LLFF/Fern config.

Directions are generated inside the ray kernel from (H, W, intrinsics); ``get_ray_directions``
returns the unit camera-frame directions by running that kernel with the identity pose.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import torch
from torch import Tensor

from . import kernels as K


@dataclass
class SceneBox:
    """AABB (2,3) = [min, max] (nerfs/scene_box.py:10-31)."""

    aabb: Tensor

    @property
    def min(self):
        return self.aabb[0]

    @property
    def max(self):
        return self.aabb[1]

    def to(self, dev):
        return SceneBox(aabb=self.aabb.to(dev))

    def ray_aabb_intersect(self, origins, directions, eps=1e-8, max_bound=1e10, invalid_value=1e10):
        """nerfs/scene_box.py:45-107 (eps fixed at 1e-8 in the kernel, as get_rays passes it)."""
        if eps != 1e-8:
            raise ValueError("the HIP slab test uses eps=1e-8 (the value get_rays passes)")
        n = origins.shape[0]
        rays = torch.cat([origins, directions, torch.zeros(n, 2, device=origins.device)], -1).float().contiguous()
        out = _aabb_from_rays(rays, self.aabb, max_bound, invalid_value)
        return out[:, 6], out[:, 7]


def _aabb_from_rays(rays, aabb, max_bound, invalid_value):
    # slab test for rays built from caller-supplied directions (torch device ops; the training/render
    # hot path uses the fused HIP kernel through rays_for_camera, which runs the same test in-kernel).
    o, d = rays[:, :3], rays[:, 3:6]
    eps = 1e-8
    rd = torch.where(d.abs() < eps, torch.where(d >= 0, torch.full_like(d, eps), torch.full_like(d, -eps)), d)
    inv = 1.0 / rd
    a = aabb.to(rays.device, torch.float32)
    t0 = (a[0] - o) * inv
    t1 = (a[1] - o) * inv
    tmin = torch.minimum(t0, t1).amax(-1).clamp(0.0, max_bound)
    tmax = torch.maximum(t0, t1).amin(-1).clamp(0.0, max_bound)
    bad = tmax <= tmin
    out = rays.clone()
    out[:, 6] = torch.where(bad, torch.full_like(tmin, invalid_value), tmin)
    out[:, 7] = torch.where(bad, torch.full_like(tmax, invalid_value), tmax)
    return out


def get_ray_directions(H: int, W: int, fx: float, fy: float, cx: float, cy: float, center_pixels: bool,
                       device) -> Tensor:
    """Unit camera-frame directions (H, W, 3), OpenGL/RUB (ray_sampling.py:111-136)."""
    eye = torch.eye(4, dtype=torch.float32, device=device)[:3]
    rays = K.rays_gen(eye.contiguous(), H, W, fx, fy, cx, cy, near=0.0, far=0.0, center_pixels=center_pixels)
    return rays[:, 3:6].reshape(H, W, 3)


def get_rays(directions: Tensor, c2w: Tensor, scene_box: Optional[SceneBox] = None, near: Optional[float] = None,
             far: Optional[float] = None, *, aabb_max_bound: float = 1e10, aabb_invalid_value: float = 1e10) -> Tensor:
    """(H,W,3)->(H,W,8) or (N,3)->(N,8) packed rays [o, d, near, far] (ray_sampling.py:50-108).

    Rotation of arbitrary given directions runs as a (N,3)x(3,3) product; the fused HIP path that
    never materialises directions is ``rays_for_camera``."""
    if directions.ndim == 2 and directions.shape[1] == 3:
        flat, shp = True, None
    elif directions.ndim == 3 and directions.shape[-1] == 3:
        flat, shp = False, directions.shape[:2]
    else:
        raise ValueError(f"directions must be (H, W, 3) or (N, 3), got {tuple(directions.shape)}")
    if scene_box is None and (near is None or far is None):
        raise ValueError("Provide near/far when scene_box is None")
    d = directions.reshape(-1, 3)
    R, t = c2w[:3, :3].to(d), c2w[:3, 3].to(d)
    dw = d @ R.T
    ow = t.expand_as(dw)
    n = dw.shape[0]
    rays = torch.cat([ow, dw, torch.zeros(n, 2, device=d.device, dtype=d.dtype)], -1).contiguous()
    if scene_box is not None:
        rays = _aabb_from_rays(rays, scene_box.aabb, aabb_max_bound, aabb_invalid_value)
    else:
        rays[:, 6] = float(near)
        rays[:, 7] = float(far)
    return rays if flat else rays.view(*shp, 8)


def rays_for_camera(H, W, fx, fy, cx, cy, c2w, *, near=None, far=None, scene_box=None, center_pixels=True,
                    pix=None, images_u8=None):
    """Fused HIP ray generation: directions + cam->world + near/far (+ pixel gather) in one kernel."""
    aabb = None if scene_box is None else scene_box.aabb.to(c2w.device, torch.float32)
    return K.rays_gen(c2w.float().contiguous(), H, W, fx, fy, cx, cy, pix=pix, near=near, far=far, aabb=aabb,
                      center_pixels=center_pixels, images_u8=images_u8)


def pack_rays(rays_o, rays_d, near, far):
    return torch.cat([rays_o, rays_d, near, far], dim=-1)


def unpack_rays(rays):
    assert rays.shape[-1] == 8, "packed rays must be (..., 8)"
    flat = rays.view(-1, 8).contiguous()
    return flat[:, :3], flat[:, 3:6], flat[:, 6:7], flat[:, 7:8]


@torch.no_grad()
def clamp_rays_near_far(rays: Tensor, near_far_override: Optional[Tuple[Optional[float], Optional[float]]], *,
                        eps: float = 1e-6, invalid_value: float = float("inf")):
    """ray_sampling.py:139-176 — returns (rays_clamped, valid_mask)."""
    if near_far_override is None:
        n, f = rays[:, 6], rays[:, 7]
        return rays, torch.isfinite(n) & torch.isfinite(f) & (f > n + eps)
    no, fo = near_far_override
    return K.clamp_near_far(rays.float().contiguous(), no, fo, eps, invalid_value)


def ndc_rays(H: int, W: int, focal: float, near_plane: float, rays: Tensor) -> Tensor:
    """Forward-facing NDC (canonical NeRF; parity unpinned — absent in the reference)."""
    return K.rays_ndc(rays.float().contiguous(), H, W, focal, near_plane)
