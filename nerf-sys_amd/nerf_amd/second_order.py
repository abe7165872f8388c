"""Second-order MAML (``create_graph=True``) for the vanilla expert: the PyTorch composite SURVEY.md §8(b) names
("second-order is unsupported: raise -> PyTorch fallback").

The HIP MLP and compositing kernels are autograd Functions with first-order backwards only (``once_differentiable``):
their backward kernels have no derivative of their own.  The reference's inner loop with ``algo="maml"``
(pipelines/offline_stage/meta_core.py:23,54-64) takes ``torch.autograd.grad(loss, fast, create_graph=True)``, so the
inner gradient must itself be differentiable.  Inside ``second_order()`` the two differentiable pieces of the stratified
render run as torch GPU ops instead, written from the reference's definitions:

  * the vanilla expert (models/inr/meta_vanilla.py:109-154; MetaLinear ``inputs.matmul(W.t()) + b``,
    models/metamodule/metamodule.py:150-156; ``trunc_exp`` as models/trunc_exp.py:43-57, whose backward saves the
    clamped input, so its second derivative through ``exp`` is not propagated there either);
  * ``volume_render`` (nerfs/ray_rendering.py:114-165).

Everything that carries no fast-weight gradient stays on the HIP kernels: ray sampling, the frequency encodings (their
inputs need no gradient), ``sample_pdf`` (detached), the background MLP (its output enters the inner gradient's graph as
a value; its own backward is first order).  The query loss and the outer ``backward`` run on the HIP path as usual
(a plain backward through the inner gradient's torch graph needs no double backward of a HIP kernel).

Not covered (raises under ``second_order()``): the Instant-NGP expert, the occupancy renderer and a full container's
expert mix — their backward kernels sit on the path from the loss to the fast weights.  This is a GPU composite of
torch ops for an off-hot-path feature, not a CPU fallback: every tensor stays on the device.
"""
from __future__ import annotations

import contextlib
import threading

import torch

_state = threading.local()


def active() -> bool:
    """True inside ``second_order()`` with grad mode on."""
    return bool(getattr(_state, "depth", 0)) and torch.is_grad_enabled()


@contextlib.contextmanager
def second_order():
    _state.depth = getattr(_state, "depth", 0) + 1
    try:
        yield
    finally:
        _state.depth -= 1


def refuse(what: str):
    if active():
        raise NotImplementedError(f"second-order MAML (create_graph=True) through {what} is not supported; "
                                  "use algo='fomaml' / 'reptile', or a vanilla expert on the stratified renderer")


def _linear(h, W, b):
    return h.matmul(W.t()) + b          # metamodule.py:153-156


def vanilla_forward(net, x_d, params=None):
    """meta_vanilla.py:123-154 in torch ops: x_d (M,6) -> (M,4) [rgb, sigma]."""
    from .encodings import FrequencyEncoder
    from .vanilla import PARAM_SHAPES, trunc_exp_torch
    T = dict(zip(PARAM_SHAPES, net.tensors(params)))
    x, d = x_d[:, :3].detach(), x_d[:, 3:6].detach()
    enc = FrequencyEncoder(3, 10)(x)        # HIP kernel: no gradient is needed w.r.t. positions
    denc = FrequencyEncoder(3, 4)(d)
    h = enc
    for i in range(8):
        if i == 4:
            h = torch.cat([h, enc], dim=-1)
        h = torch.relu(_linear(h, T[f"trunk.{i}.linear.weight"], T[f"trunk.{i}.linear.bias"]))
    sigma = trunc_exp_torch(_linear(h, T["sigma_head.weight"], T["sigma_head.bias"]))
    geo = _linear(h, T["geo_head.weight"], T["geo_head.bias"])
    c = torch.relu(_linear(torch.cat([geo, denc], dim=-1), T["color_mlp.layer0.linear.weight"],
                           T["color_mlp.layer0.linear.bias"]))
    rgb = torch.sigmoid(_linear(c, T["color_mlp.color_out.weight"], T["color_mlp.color_out.bias"]))
    return torch.cat([rgb, sigma], dim=-1)


def volume_render(rgb_sigma, t_vals, bg_rgb=None, sigma_scale=1.0):
    """ray_rendering.py:114-165 (raw_rgb = raw_sigma = False) in torch ops."""
    rgb = rgb_sigma[..., :3].clamp(0.0, 1.0)
    sigma = rgb_sigma[..., 3].clamp_min(0.0)
    if sigma_scale != 1.0:
        sigma = sigma * float(sigma_scale)
    dists = (t_vals[:, 1:] - t_vals[:, :-1]).clamp_min(1e-4)
    dists = torch.cat([dists, dists[:, -1:]], dim=1)
    alpha = (1.0 - torch.exp(-sigma * dists)).clamp(0.0, 1.0 - 1e-7)
    T = torch.cumprod(torch.cat([torch.ones_like(alpha[:, :1]), 1.0 - alpha + 1e-10], dim=1), dim=1)[:, :-1]
    w = alpha * T
    rgb_map = (w.unsqueeze(-1) * rgb).sum(dim=1)
    depth = (w * t_vals).sum(dim=1)
    acc = w.sum(dim=1)
    if bg_rgb is not None:
        rgb_map = rgb_map + (1.0 - acc.unsqueeze(-1)) * bg_rgb
    return rgb_map, depth, w, acc
