"""Loss head — nerfs/losses.py:10-32 + nerfs/color_space.py:4-66 of the reference.

``compute_mse_loss(P, model, data, ...)`` keeps the reference signature (P.ray_samples,
P.chunk_points, P.color_space) and adds the canonical coarse+fine term when P.n_importance > 0.
The fused training engine (trainer.py) computes the same loss inside the compositing kernel.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .ray_rendering import render_rays


def linear_to_srgb(x):
    x = x.clamp(0, 1)
    return torch.where(x <= 0.0031308, 12.92 * x, 1.055 * x.pow(1 / 2.4) - 0.055)


def srgb_to_linear(x):
    return torch.where(x <= 0.04045, x / 12.92, ((x + 0.055) / 1.055).pow(2.4))


def color_space_transformer(pred_linear, gt_tensor, color_space: str):
    cs = str(color_space).lower()
    pred32 = pred_linear.to(torch.float32)
    gt32 = gt_tensor.to(torch.float32).clamp(0, 1)
    if cs == "linear":
        pred, gt = pred32.clamp(0, 1), srgb_to_linear(gt32).clamp(0, 1)
    elif cs == "srgb":
        pred, gt = linear_to_srgb(pred32).clamp(0, 1), gt32.clamp(0, 1)
    elif cs == "identity":
        if (gt32.max() > 1) or (gt32.min() < 0):
            raise ValueError("GT out of [0,1]; identity mode assumes normalized linear GT.")
        pred, gt = pred32, gt32
    else:
        raise ValueError(f"Invalid color_space={color_space!r}; use 'linear'|'srgb'|'identity'")
    return pred.to(pred_linear.dtype), gt.to(pred_linear.dtype)


def compute_mse_loss(P, model, data, params=None, active_module=None, reduction="mean"):
    gt_rgb, rays = data["rgbs"], data["rays"]
    n_imp = int(getattr(P, "n_importance", 0) or 0)
    out = render_rays(model, rays, ray_samples=P.ray_samples, params=params, active_module=active_module,
                      chunk=P.chunk_points, n_importance=n_imp, return_extras=True)
    pred_rgb, extras = out[0], out[-1]
    cs = getattr(P, "color_space", "linear")
    a, b = color_space_transformer(pred_rgb, gt_rgb, cs)
    loss = F.mse_loss(a, b, reduction=reduction)
    if n_imp > 0:
        a, b = color_space_transformer(extras["rgb_coarse"], gt_rgb, cs)
        loss = loss + F.mse_loss(a, b, reduction=reduction)
    return loss


def psnr(mse: float) -> float:
    import math
    return -10.0 * math.log10(max(float(mse), 1e-8))


def image_psnr(pred_linear, gt_u8_or_srgb, color_space: str = "linear") -> float:
    """Full-image PSNR as the reference evaluates it (pipelines/online_stage/runtime_adapt.py:150-157):
    the rendered image is linear, the ground truth is 8-bit sRGB, and both are brought into
    ``color_space`` (the training colour space, args.py:98-102) by color_space_transformer."""
    gt = gt_u8_or_srgb.float() / 255.0 if gt_u8_or_srgb.dtype == torch.uint8 else gt_u8_or_srgb.float()
    a, b = color_space_transformer(pred_linear.float(), gt.to(pred_linear.device), color_space)
    return psnr(F.mse_loss(a, b).item())


def compute_fim_loss(P, model, data, params=None, active_module=None, *, grad_buffer=None, update_fisher=False,
                     clamp_factor=5):
    """Fisher-weighted loss (nerfs/losses.py:35-151): one render through the HIP path, per-ray MSE.

    Without a Fisher store on the container and the active expert (``model.fisher_store`` / ``model.fim_loss``
    and ``expert.fisher_store.tracked``, the reference's own guard at :81-87) it is the plain mean of the per-ray
    MSE.  With them, the gradients of that loss w.r.t. the tracked tensors give the Fisher weight
    (``expert.fim_loss.fim_weight``; per ray with ``P.fim_per_sample``), the weighted loss is returned and, on
    the support path (``grad_buffer`` given or ``update_fisher``), the weighted gradients are written into
    ``grad_buffer`` and the store is updated from the squared unweighted gradients."""
    pred = render_rays(model, data["rays"], ray_samples=P.ray_samples, params=params, active_module=active_module,
                       chunk=P.chunk_points)[0]
    pred, gt = color_space_transformer(pred, data["rgbs"], getattr(P, "color_space", "linear"))
    per_ray = F.mse_loss(pred, gt, reduction="none").mean(dim=-1)
    base = per_ray.mean()
    if active_module is None or not (hasattr(model, "fisher_store") and hasattr(model, "fim_loss")):
        return base
    expert = model.submodules[active_module]
    store = expert.fisher_store
    if not store.tracked:
        return base
    names = [n for n, _ in store.tracked]
    tensors = [t for _, t in store.tracked]
    if str(getattr(P, "algo", "")).lower() not in ("fomaml", "reptile"):
        raise NotImplementedError("Fisher-weighted loss with second-order gradients is not on the HIP path")
    support = bool(grad_buffer) or bool(update_fisher)  # need_grads of the reference (:56)
    per_sample = bool(getattr(P, "fim_per_sample", False))
    g0 = torch.autograd.grad(base, tensors, allow_unused=True, retain_graph=(not support) or per_sample)
    gd = {n: g.detach() for n, g in zip(names, g0) if g is not None}
    lim = (1.0 / clamp_factor, float(clamp_factor))
    if per_sample:
        w = expert.fim_loss.fim_weight(gd, mse_i=per_ray, per_sample=True, clamp=lim)
        loss = (w.detach() * per_ray).mean()
        if not support:
            return loss
        gw = torch.autograd.grad(loss, tensors, allow_unused=True)
    else:
        w = expert.fim_loss.fim_weight(gd, per_sample=False, clamp=lim).detach()
        loss = w * base
        if not support:
            return loss
        gw = [None if g is None else w * g for g in g0]
    if update_fisher and gd:
        with torch.no_grad():
            store.update_from_grads({n: g.pow(2) for n, g in gd.items()})
    if grad_buffer is not None:
        for n, g in zip(names, gw):
            if g is not None:
                grad_buffer[n] = g
    return loss
