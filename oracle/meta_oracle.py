"""CPU restatement of the reference's data path and meta-learning updates — TEST
INFRASTRUCTURE ONLY (imported by tests/ as the checker; never by the product package).

* ``process_single_image``  — data/ram_rays_dataset.py:46-121 (_process_single_image): rays of one image,
  keep mask, near/far clamp with override, valid filter, rgb / 255, image index.
* ``val_balancing``         — ram_rays_dataset.py:236-260 (_apply_meganerf_val_balancing_static), RNG = torch's.
* ``task_adapt``            — pipelines/offline_stage/meta_core.py:14-68, first-order (fomaml / reptile): fast
  weights, ``torch.autograd.grad`` of the MSE loss, ``w - inner_lr * g`` per tensor.
* ``reptile_update``        — meta_core.py:145-176: mean delta over fast lists, per-tensor finite / non-zero guard.

Parity is PINNED: tests/golden/data.npz and tests/golden/meta.npz were produced by importing the reference
(tools/gen_golden.py gen_data / gen_meta).
"""
from __future__ import annotations

from collections import OrderedDict

import torch

from . import nerf_oracle as O


def process_single_image(img_u8, mask, H, W, intrinsics, c2w, aabb, center_pixels=True, near_far_override=None,
                         image_index=0):
    """ram_rays_dataset.py:46-121 for one in-memory image (H, W, 3) uint8 and an optional (H, W) bool mask.
    Returns (rgbs (n,3) fp32, rays (n,8), indices (n,) int32) or None (empty after masking / clamping)."""
    if mask is not None and int(mask.sum()) == 0:                                     # :83-85
        return None
    fx, fy, cx, cy = [float(v) for v in intrinsics]
    dirs = O.get_ray_directions(H, W, fx, fy, cx, cy, center_pixels)                 # :88-90
    rays = O.get_rays(dirs, c2w[:3, :4].float(), aabb=aabb).reshape(-1, 8)           # :91-92
    img = img_u8.reshape(-1, 3)
    if mask is not None:                                                              # :95-101
        keep = mask.reshape(-1).bool()
        rays, img = rays[keep], img[keep]
    rays, valid = O.clamp_rays_near_far(rays, near_far_override)                     # :104-106
    if not bool(valid.any()):
        return None
    rays = rays[valid]
    rgbs = img[valid].to(torch.float32).div_(255.0)                                   # :111-112
    return rgbs, rays, torch.full((rgbs.shape[0],), int(image_index), dtype=torch.int32)


def val_balancing(keep_mask, H, W):
    """ram_rays_dataset.py:236-260: move the right half's kept count onto random unkept left-half pixels
    (torch.randperm draw), then drop the right half."""
    keep_mask = keep_mask.reshape(H, W).clone()
    left = keep_mask[:, : W // 2]
    right = keep_mask[:, W // 2:]
    n_right = int(right.sum())
    if n_right > 0:
        cand = torch.arange(H * W).view(H, W)[:, : W // 2][~left]
        if cand.numel() > 0:
            add = cand[torch.randperm(cand.numel())[:n_right]]
            flat = keep_mask.view(-1)
            flat[add] = True
    keep_mask[:, W // 2:] = False
    return keep_mask.reshape(-1)


def task_adapt(expert, params, rays, gt, S, inner_lr, iterations, color_space="linear", bg="white"):
    """meta_core.py:14-68 first-order: expert(p, x_d) -> (M,4); eval-mode (deterministic) t; MSE loss of
    nerfs/losses.py:10-32. Returns (fast OrderedDict, [loss per iteration])."""
    fast = OrderedDict((n, v.detach().clone().requires_grad_(True)) for n, v in params.items())
    losses = []
    for _ in range(int(iterations)):
        rgb = O.render_rays(lambda x_d: expert(fast, x_d), rays, S, training=False, bg=bg)[0]
        loss = O.mse_loss(rgb, gt, color_space)
        grads = torch.autograd.grad(loss, tuple(fast.values()), allow_unused=True)
        fast = OrderedDict((n, w if g is None else (w - inner_lr * g)) for (n, w), g in zip(fast.items(), grads))
        losses.append(loss.detach())
    return fast, losses


@torch.no_grad()
def reptile_update(theta, fast_list, lr):
    """meta_core.py:145-176 on a {name: tensor} theta (updated in place); returns the updated names."""
    snap = {k: v.clone() for k, v in theta.items()}
    sums = {k: torch.zeros_like(v) for k, v in snap.items()}
    for fast in fast_list:
        for k, v in fast.items():
            if k in sums:
                sums[k].add_(v.detach() - snap[k])
    n = float(len(fast_list))
    done = []
    for k, p in theta.items():
        if k in sums:
            delta = sums[k] / n
            if torch.isfinite(delta).all() and delta.abs().sum() > 0:
                p.add_(lr * delta)
                done.append(k)
    return done
