"""Synthetic scenes for the benchmark configs (Lego / Fern are not in the container — BASELINE.json).

* Blender-style (C1/C2/C3/C5): 800x800, camera_angle_x = 0.6911112 (focal 1111.111), poses on the upper
  hemisphere at radius 4.0311 looking at the origin, near 2 / far 6, white background.
* LLFF-style forward-facing (C4, "Fern"): 1008x756, focal 815, poses on a small spiral facing -z,
  rendered through NDC (near plane 1).
The content is an analytic set of seeded coloured opaque spheres (ray-sphere first hit, Lambert shading),
so ground truth is exact without sampling.  Images are uint8 (like 8-bit PNG data) and live in HBM;
the training batch (pixel pick + ray generation + colour gather) is one HIP kernel (trainer.RayBatcher).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

BLENDER_FOCAL = 0.5 * 800 / math.tan(0.5 * 0.6911112)


def look_at(cam_pos: torch.Tensor, target=(0.0, 0.0, 0.0), up=(0.0, 0.0, 1.0)) -> torch.Tensor:
    """c2w (3,4), OpenGL/RUB: camera looks along -z."""
    c = cam_pos.double()
    z = c - torch.tensor(target, dtype=torch.float64)
    z = z / z.norm()
    upv = torch.tensor(up, dtype=torch.float64)
    x = torch.linalg.cross(upv, z)
    if x.norm() < 1e-8:
        x = torch.tensor([1.0, 0.0, 0.0], dtype=torch.float64)
    x = x / x.norm()
    y = torch.linalg.cross(z, x)
    return torch.stack([x, y, z, c], 1).float()


def hemisphere_poses(n: int, radius: float = 4.0311, seed: int = 0) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    az = torch.rand(n, generator=g, dtype=torch.float64) * 2 * math.pi
    el = torch.rand(n, generator=g, dtype=torch.float64) * (math.pi / 2 - 0.15) + 0.1
    pos = torch.stack([torch.cos(az) * torch.cos(el), torch.sin(az) * torch.cos(el), torch.sin(el)], 1) * radius
    return torch.stack([look_at(p) for p in pos])


def spiral_poses(n: int, seed: int = 0) -> torch.Tensor:
    """Forward-facing cameras near z=+4 looking at -z (LLFF-like)."""
    poses = []
    for k in range(n):
        a = 2 * math.pi * k / max(n, 1)
        pos = torch.tensor([0.3 * math.cos(a), 0.2 * math.sin(a), 4.0 + 0.1 * math.sin(2 * a)])
        poses.append(look_at(pos, target=(0.0, 0.0, -6.0), up=(0.0, 1.0, 0.0)))
    return torch.stack(poses)


@dataclass
class Scene:
    H: int
    W: int
    focal: float
    near: float
    far: float
    poses: torch.Tensor      # (n,3,4) train
    images: torch.Tensor     # (n,H,W,3) uint8
    test_poses: torch.Tensor
    test_images: torch.Tensor
    ndc: bool = False

    @property
    def intrinsics(self):
        return (self.focal, self.focal, self.W / 2.0, self.H / 2.0)


def _spheres(seed: int, forward: bool):
    g = torch.Generator().manual_seed(1000 + seed)
    k = 10
    if forward:
        cen = torch.stack([torch.rand(k, generator=g) * 4 - 2, torch.rand(k, generator=g) * 3 - 1.5,
                           -(torch.rand(k, generator=g) * 6 + 2)], 1)
        rad = torch.rand(k, generator=g) * 0.5 + 0.3
    else:
        cen = (torch.rand(k, 3, generator=g) * 2 - 1) * 0.9
        rad = torch.rand(k, generator=g) * 0.3 + 0.15
    col = torch.rand(k, 3, generator=g) * 0.8 + 0.1
    return cen, rad, col


@torch.no_grad()
def render_analytic(poses, H, W, focal, seed=0, forward=False, device="cpu", rows_per_chunk=None):
    """Exact images of the sphere scene (torch device ops; data generation, not the hot path)."""
    cen, rad, col = [t.to(device) for t in _spheres(seed, forward)]
    light = torch.tensor([0.4, 0.5, 0.75], device=device)
    light = light / light.norm()
    out = torch.empty(poses.shape[0], H, W, 3, dtype=torch.uint8, device=device)
    j, i = torch.meshgrid(torch.arange(H, device=device, dtype=torch.float32),
                          torch.arange(W, device=device, dtype=torch.float32), indexing="ij")
    dirs = torch.stack([(i + 0.5 - W / 2) / focal, -(j + 0.5 - H / 2) / focal, -torch.ones_like(i)], -1)
    dirs = dirs / dirs.norm(dim=-1, keepdim=True)
    if rows_per_chunk is None:  # whole image per pass on the GPU, bounded chunks on the CPU
        rows_per_chunk = H if str(device).startswith("cuda") else 64
    for p in range(poses.shape[0]):
        c2w = poses[p].to(device)
        for r0 in range(0, H, rows_per_chunk):
            d = dirs[r0:r0 + rows_per_chunk].reshape(-1, 3) @ c2w[:3, :3].T
            o = c2w[:3, 3].expand_as(d)
            oc = o[:, None, :] - cen[None]                       # (R,K,3)
            b = (oc * d[:, None, :]).sum(-1)
            cc = (oc * oc).sum(-1) - rad[None] ** 2
            disc = b * b - cc
            tt = -b - torch.sqrt(disc.clamp_min(0))
            tt = torch.where((disc > 0) & (tt > 0), tt, torch.full_like(tt, float("inf")))
            tmin, kk = tt.min(-1)
            hit = torch.isfinite(tmin)
            x = o + d * tmin.clamp_max(1e3)[:, None]
            nrm = x - cen[kk]
            nrm = nrm / nrm.norm(dim=-1, keepdim=True).clamp_min(1e-9)
            shade = 0.35 + 0.65 * (nrm @ light).clamp_min(0)
            rgb = col[kk] * shade[:, None]
            rgb = torch.where(hit[:, None], rgb, torch.ones_like(rgb))
            out[p, r0:r0 + rows_per_chunk] = (rgb.clamp(0, 1) * 255 + 0.5).to(torch.uint8).view(-1, W, 3)
    return out


def make_blender_scene(n_train=100, n_test=25, H=800, W=800, seed=0, device="cpu") -> Scene:
    focal = 0.5 * W / math.tan(0.5 * 0.6911112)
    poses = hemisphere_poses(n_train + n_test, seed=seed)
    imgs = render_analytic(poses, H, W, focal, seed=seed, device=device)
    return Scene(H, W, focal, 2.0, 6.0, poses[:n_train].to(device), imgs[:n_train], poses[n_train:].to(device),
                 imgs[n_train:])


def make_llff_scene(n_train=20, n_test=4, H=756, W=1008, focal=815.0, seed=0, device="cpu") -> Scene:
    poses = spiral_poses(n_train + n_test, seed=seed)
    imgs = render_analytic(poses, H, W, focal, seed=seed, forward=True, device=device)
    return Scene(H, W, focal, 0.0, 1.0, poses[:n_train].to(device), imgs[:n_train], poses[n_train:].to(device),
                 imgs[n_train:], ndc=True)
