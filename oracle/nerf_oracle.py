"""CPU restatement of the reference's NeRF hot path — TEST INFRASTRUCTURE ONLY.

This module is the parity oracle (and the timed CPU baseline, ``cpu_baseline.kind
= "port"``).  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it, and only as the checker.  The product path
(``nerf-sys_amd/nerf_amd``) never imports it and has no CPU fallback.

Every function restates one reference function (cited ``file:line`` relative to
``/root/reference/adaptive_nerf``).  It is written from the reference's observed
behaviour, in plain PyTorch on the CPU, so that autograd supplies the reference
gradients.  Parity of this restatement is PINNED against golden vectors produced
by importing the reference itself (``tools/gen_golden.py`` → ``tests/golden``),
except for two components the reference does not have:

* ``sample_pdf``  (hierarchical inverse-CDF resampling) — **parity unpinned**;
  canonical NeRF formulation (Mildenhall et al. 2020, ``run_nerf_helpers.sample_pdf``),
  pinned only by known-answer / property tests.
* ``ndc_rays`` (forward-facing NDC) — **parity unpinned**; canonical formulation.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import torch
import torch.nn.functional as F

# --------------------------------------------------------------------------
# rays  (nerfs/ray_sampling.py, nerfs/scene_box.py)
# --------------------------------------------------------------------------


def get_ray_directions(H, W, fx, fy, cx, cy, center_pixels=True, dtype=torch.float32):
    """nerfs/ray_sampling.py:111-136 — unit camera-frame directions (H,W,3), OpenGL/RUB."""
    j, i = torch.meshgrid(torch.arange(H, dtype=dtype), torch.arange(W, dtype=dtype), indexing="ij")
    if center_pixels:
        i = i + 0.5
        j = j + 0.5
    dirs = torch.stack([(i - cx) / fx, -(j - cy) / fy, -torch.ones_like(i)], dim=-1)
    return dirs / dirs.norm(dim=-1, keepdim=True).clamp_min(1e-12)


def ray_aabb_intersect(o, d, aabb, eps=1e-8, max_bound=1e10, invalid_value=1e10):
    """nerfs/scene_box.py:45-107 — slab test, clamp to [0,max_bound], invalid -> invalid_value."""
    rd = torch.where(d.abs() < eps, torch.where(d >= 0, torch.full_like(d, eps), torch.full_like(d, -eps)), d)
    inv = 1.0 / rd
    t0 = (aabb[0].unsqueeze(0) - o) * inv
    t1 = (aabb[1].unsqueeze(0) - o) * inv
    tmin = torch.minimum(t0, t1).amax(dim=-1).clamp(0.0, max_bound)
    tmax = torch.maximum(t0, t1).amin(dim=-1).clamp(0.0, max_bound)
    bad = tmax <= tmin
    iv = torch.as_tensor(invalid_value, dtype=o.dtype)
    return torch.where(bad, iv, tmin), torch.where(bad, iv, tmax)


def get_rays(dirs, c2w, aabb=None, near=None, far=None, max_bound=1e10, invalid_value=1e10):
    """nerfs/ray_sampling.py:50-108 (+ _rays_cam_to_world :10-24) — packed (…,8) rays."""
    shp = dirs.shape[:-1]
    df = dirs.reshape(-1, 3)
    R, t = c2w[:3, :3], c2w[:3, 3]
    dw = df @ R.T
    ow = t.expand_as(dw)
    if aabb is not None:
        n, f = ray_aabb_intersect(ow, dw, aabb, 1e-8, max_bound, invalid_value)
    else:
        n = torch.full((df.shape[0],), float(near), dtype=df.dtype)
        f = torch.full((df.shape[0],), float(far), dtype=df.dtype)
    return torch.cat([ow, dw, n[:, None], f[:, None]], -1).reshape(*shp, 8)


def clamp_rays_near_far(rays, override, eps=1e-6, invalid_value=float("inf")):
    """nerfs/ray_sampling.py:139-176."""
    if override is None:
        n, f = rays[:, 6], rays[:, 7]
        return rays, torch.isfinite(n) & torch.isfinite(f) & (f > n + eps)
    no, fo = override
    rays = rays.clone()
    n, f = rays[:, 6], rays[:, 7]
    if no is not None:
        n = torch.maximum(n, torch.as_tensor(float(no), dtype=rays.dtype))
    if fo is not None:
        f = torch.minimum(f, torch.as_tensor(float(fo), dtype=rays.dtype))
    valid = torch.isfinite(n) & torch.isfinite(f) & (f > n + eps)
    iv = torch.full_like(n, float(invalid_value))
    rays[:, 6] = torch.where(valid, n, iv)
    rays[:, 7] = torch.where(valid, f, iv)
    return rays, valid


def ndc_rays(H, W, focal, near_plane, rays):
    """Forward-facing NDC rays (canonical NeRF ``ndc_rays``) — PARITY UNPINNED (absent in reference).

    Input rays (N,8) world space; output (N,8) with o,d in NDC and [near,far]=[0,1].
    Directions are NOT renormalised (t in [0,1] spans near-plane to infinity)."""
    o, d = rays[:, :3], rays[:, 3:6]
    t = -(near_plane + o[:, 2]) / d[:, 2]
    o = o + t[:, None] * d
    o0 = -1.0 / (W / (2.0 * focal)) * o[:, 0] / o[:, 2]
    o1 = -1.0 / (H / (2.0 * focal)) * o[:, 1] / o[:, 2]
    o2 = 1.0 + 2.0 * near_plane / o[:, 2]
    d0 = -1.0 / (W / (2.0 * focal)) * (d[:, 0] / d[:, 2] - o[:, 0] / o[:, 2])
    d1 = -1.0 / (H / (2.0 * focal)) * (d[:, 1] / d[:, 2] - o[:, 1] / o[:, 2])
    d2 = -2.0 * near_plane / o[:, 2]
    z = torch.zeros_like(o0)
    return torch.stack([o0, o1, o2, d0, d1, d2, z, z + 1.0], -1)


# --------------------------------------------------------------------------
# sampling  (nerfs/ray_rendering.py)
# --------------------------------------------------------------------------


def stratified_t_vals(near, far, S, randomized, u=None):
    """nerfs/ray_rendering.py:262-287.  ``u`` replaces ``torch.rand_like(low)`` (:286)."""
    t_lin = torch.linspace(0.0, 1.0, S, dtype=near.dtype, device=near.device).unsqueeze(0)
    t = near.unsqueeze(1) * (1.0 - t_lin) + far.unsqueeze(1) * t_lin
    if randomized:
        mids = 0.5 * (t[:, :-1] + t[:, 1:])
        low = torch.cat([t[:, :1], mids], 1)
        high = torch.cat([mids, t[:, -1:]], 1)
        if u is None:
            u = torch.rand_like(low)
        t = low + (high - low) * u
    return t


def sample_pdf(bins, weights, n_samples, u=None, det=False):
    """Inverse-CDF resampling — PARITY UNPINNED (absent in reference; canonical NeRF).

    bins (N,B+1) interval edges, weights (N,B).  Returns (N,n_samples).  ``u`` (N,n) in [0,1)
    is consumed as given (the GPU kernel sorts it first; the merged output is identical)."""
    weights = weights + 1e-5
    # normaliser accumulated in fp64 and rounded once (ISA-independent; torch's own fp32 sum order
    # depends on the host's vector width).  cumsum already accumulates fp32 in fp64 on the CPU.
    pdf = weights / weights.double().sum(-1, keepdim=True).to(weights.dtype)
    cdf = torch.cumsum(pdf, -1)
    cdf = torch.cat([torch.zeros_like(cdf[:, :1]), cdf], -1)  # (N,B+1)
    if u is None:
        if det:
            u = torch.linspace(0.0, 1.0, n_samples, dtype=bins.dtype).expand(cdf.shape[0], n_samples)
        else:
            u = torch.rand(cdf.shape[0], n_samples, dtype=bins.dtype)
    u = u.contiguous()
    inds = torch.searchsorted(cdf, u, right=True)
    below = (inds - 1).clamp_min(0)
    above = inds.clamp_max(cdf.shape[-1] - 1)
    cdf0, cdf1 = torch.gather(cdf, 1, below), torch.gather(cdf, 1, above)
    b0, b1 = torch.gather(bins, 1, below), torch.gather(bins, 1, above)
    denom = cdf1 - cdf0
    denom = torch.where(denom < 1e-5, torch.ones_like(denom), denom)
    tt = (u - cdf0) / denom
    return b0 + tt * (b1 - b0)


def hierarchical_t_vals(t_coarse, weights_coarse, n_importance, u=None, det=False):
    """t_coarse (N,S) sorted, weights (N,S) → merged sorted (N,S+n_importance), detached.

    Canonical NeRF: bins = midpoints of t (N,S-1), pdf over interior weights[:,1:-1]."""
    with torch.no_grad():
        mids = 0.5 * (t_coarse[:, 1:] + t_coarse[:, :-1])
        fine = sample_pdf(mids, weights_coarse[:, 1:-1], n_importance, u=u, det=det)
        merged, _ = torch.sort(torch.cat([t_coarse, fine], -1), -1)
    return merged


# --------------------------------------------------------------------------
# model  (models/encodings.py, models/inr/meta_vanilla.py, models/trunc_exp.py)
# --------------------------------------------------------------------------


def freq_encode(x, n_freq, include_input=True):
    """models/encodings.py:437-444 — per input dim [cos f0..f_{L-1}, sin f0..f_{L-1}], dim-major."""
    bands = 2.0 ** torch.arange(n_freq, dtype=torch.float32).to(device=x.device, dtype=x.dtype)
    xe = x[..., None] * bands
    pe = torch.cat([torch.cos(xe), torch.sin(xe)], -1).reshape(*x.shape[:-1], -1)
    return torch.cat([x, pe], -1) if include_input else pe


_EXP_MAX = {torch.float16: 11.089866488, torch.bfloat16: 88.722839111,
            torch.float32: 88.722839111, torch.float64: 709.782712893}


class _TruncExp(torch.autograd.Function):
    """models/trunc_exp.py:43-57 — bwd g·exp(clamp(x)), does NOT vanish outside the clamp."""

    @staticmethod
    def forward(ctx, x):
        m = _EXP_MAX.get(x.dtype, _EXP_MAX[torch.float32])
        xc = x.clamp(-m, m)
        ctx.save_for_backward(xc)
        return torch.exp(xc)

    @staticmethod
    def backward(ctx, g):
        (xc,) = ctx.saved_tensors
        return g * torch.exp(xc)


def trunc_exp(x):
    return _TruncExp.apply(x)


# parameter names follow MetaModule.meta_named_parameters() of MetaNeRF(encoding_dir="frequency")
_shapes = OrderedDict()
for _i in range(8):
    _shapes[f"trunk.{_i}.linear.weight"] = (256, 63 if _i == 0 else (319 if _i == 4 else 256))
    _shapes[f"trunk.{_i}.linear.bias"] = (256,)
_shapes["sigma_head.weight"] = (1, 256)
_shapes["sigma_head.bias"] = (1,)
_shapes["geo_head.weight"] = (15, 256)
_shapes["geo_head.bias"] = (15,)
_shapes["color_mlp.layer0.linear.weight"] = (128, 42)
_shapes["color_mlp.layer0.linear.bias"] = (128,)
_shapes["color_mlp.color_out.weight"] = (3, 128)
_shapes["color_mlp.color_out.bias"] = (3,)
VANILLA_SHAPES = _shapes
del _shapes, _i


def init_vanilla_params(seed=0, dtype=torch.float32):
    """nn.Linear default init (kaiming-uniform a=√5 ⇒ U(±1/√fan_in) for W and b), own generator."""
    g = torch.Generator().manual_seed(seed)
    p = OrderedDict()
    for name, shp in VANILLA_SHAPES.items():
        fan_in = VANILLA_SHAPES[name.replace(".bias", ".weight")][1]
        bound = 1.0 / math.sqrt(fan_in)
        p[name] = ((torch.rand(shp, generator=g, dtype=torch.float64) * 2 - 1) * bound).to(dtype)
    return p


def _f16(x):
    return x.to(torch.float16).to(x.dtype)


class _MatmulF16(torch.autograd.Function):
    """``x.matmul(W.t())`` inside ``torch.autocast(float16)``: both operands cast to fp16 (matmul is on autocast's
    lower-precision list), fp32 accumulation, fp16 output; the backward's two GEMMs take the fp16 gradient and return
    fp16 results, which the autocast cast nodes hand back as fp32 (x, W are fp32 tensors)."""

    @staticmethod
    def forward(ctx, x, W):
        x16, W16 = _f16(x), _f16(W)
        ctx.save_for_backward(x16, W16)
        return _f16(x16.matmul(W16.t()))

    @staticmethod
    def backward(ctx, g):
        x16, W16 = ctx.saved_tensors
        g16 = _f16(g)
        return _f16(g16.matmul(W16)), _f16(g16.t().matmul(x16))


def _lin(x, p, name, amp=None):
    """models/metamodule/metamodule.py:140-156 — out = x @ W^T + b.  amp="fp16" restates the reference's
    autocast(float16) numerics (configs/train.json "use_amp"): the matmul in fp16 (_MatmulF16), then the fp32 bias
    added — an fp16 (M,N) tensor plus an fp32 (N,) tensor promotes to fp32, so every layer output, the ReLU and the
    sigma head's trunc_exp input stay fp32 (trunc_exp clamps at 88.72, not fp16's 11.09; pinned by the imported
    reference in tests/golden/amp.npz)."""
    if amp == "fp16":
        return _MatmulF16.apply(x, p[name + ".weight"]) + p[name + ".bias"]
    return x.matmul(p[name + ".weight"].t()) + p[name + ".bias"]


def vanilla_density(p, x, amp=None):
    """models/inr/meta_vanilla.py:123-141 — skip at layer 4 is cat([h, enc]) (hidden first)."""
    enc = freq_encode(x, 10, True)
    h = enc
    for i in range(8):
        if i == 4:
            h = torch.cat([h, enc], -1)
        h = torch.relu(_lin(h, p, f"trunk.{i}.linear", amp))
    sigma = trunc_exp(_lin(h, p, "sigma_head", amp))
    geo = _lin(h, p, "geo_head", amp)
    return sigma, geo


def vanilla_forward(p, x_d, amp=None):
    """Expert contract (M,6)->(M,4) [rgb∈[0,1], σ≥0] (cf. models/inr/meta_ngp.py:226-241)
    around MetaNeRF.forward (meta_vanilla.py:143-154, color :109-121).  amp: see _lin."""
    x, d = x_d[:, :3], x_d[:, 3:6]
    sigma, geo = vanilla_density(p, x, amp)
    h = torch.cat([geo, freq_encode(d, 4, True)], -1)
    h = torch.relu(_lin(h, p, "color_mlp.layer0.linear", amp))
    rgb = torch.sigmoid(_lin(h, p, "color_mlp.color_out", amp))
    return torch.cat([rgb, sigma], -1)


# --------------------------------------------------------------------------
# compositing  (nerfs/ray_rendering.py:114-165)
# --------------------------------------------------------------------------


def volume_render(rgb_sigma, t, bg=None, sigma_scale=1.0):
    """nerfs/ray_rendering.py:114-165 (raw_rgb=raw_sigma=False as called at :336-343)."""
    rgb = rgb_sigma[..., :3].clamp(0.0, 1.0)
    sigma = rgb_sigma[..., 3].clamp_min(0.0)
    if sigma_scale != 1.0:
        sigma = sigma * float(sigma_scale)
    dists = (t[:, 1:] - t[:, :-1]).clamp_min(1e-4)
    dists = torch.cat([dists, dists[:, -1:]], 1)
    alpha = (1.0 - torch.exp(-sigma * dists)).clamp(0.0, 1.0 - 1e-7)
    T = torch.cumprod(torch.cat([torch.ones_like(alpha[:, :1]), 1.0 - alpha + 1e-10], 1), 1)[:, :-1]
    w = alpha * T
    rgb_map = (w.unsqueeze(-1) * rgb).sum(1)
    depth = (w * t).sum(1)
    acc = w.sum(1)
    if bg is not None:
        rgb_map = rgb_map + (1.0 - acc.unsqueeze(-1)) * bg
    return rgb_map, depth, w, acc


def bg_default(N, policy, dtype=torch.float32, device=None):
    """nerfs/ray_rendering.py:48-79 (deterministic policies only)."""
    if policy == "none":
        return None
    if policy == "white":
        return torch.ones(N, 3, dtype=dtype, device=device)
    if policy == "black":
        return torch.zeros(N, 3, dtype=dtype, device=device)
    raise ValueError(policy)


def render_rays(p_coarse, rays, S, training=False, u_strat=None, bg="white",
                p_fine=None, n_importance=0, u_pdf=None, amp=None):
    """nerfs/ray_rendering.py:290-345 (stratified) + canonical hierarchical extension.

    Returns (rgb, depth, weights, acc, extras) where extras holds the coarse outputs when
    n_importance > 0.  Fine network = p_fine (or p_coarse when None).  A network is a vanilla
    parameter dict, or any callable expert x_d (M,6) -> (M,4) (e.g. the Instant-NGP oracle)."""
    o, d = rays[:, :3], rays[:, 3:6]
    N = rays.shape[0]
    t = stratified_t_vals(rays[:, 6], rays[:, 7], S, training, u_strat)
    bgc = bg if isinstance(bg, torch.Tensor) or bg is None else bg_default(N, bg, rays.dtype, rays.device)

    def one_pass(p, tv):
        pts = o.unsqueeze(1) + d.unsqueeze(1) * tv.unsqueeze(-1)
        dirs = d.unsqueeze(1).expand_as(pts)
        x_d = torch.cat([pts, dirs], -1).reshape(-1, 6)
        rs = (p(x_d) if callable(p) else vanilla_forward(p, x_d, amp)).view(N, tv.shape[1], 4)
        return volume_render(rs, tv, bgc)

    out = one_pass(p_coarse, t)
    if n_importance <= 0:
        return (*out, {})
    tm = hierarchical_t_vals(t, out[2].detach(), n_importance, u=u_pdf, det=not training)
    fine = one_pass(p_fine if p_fine is not None else p_coarse, tm)
    return (*fine, {"rgb_coarse": out[0], "depth_coarse": out[1], "weights_coarse": out[2],
                    "acc_coarse": out[3], "t_coarse": t, "t_fine": tm})


# --------------------------------------------------------------------------
# loss / optimiser  (nerfs/color_space.py, nerfs/losses.py, pipelines/online_stage/runtime_adapt.py)
# --------------------------------------------------------------------------


def srgb_to_linear(x):
    """nerfs/color_space.py:13-19."""
    return torch.where(x <= 0.04045, x / 12.92, ((x + 0.055) / 1.055).pow(2.4))


def linear_to_srgb(x):
    """nerfs/color_space.py:4-10."""
    x = x.clamp(0, 1)
    return torch.where(x <= 0.0031308, 12.92 * x, 1.055 * x.pow(1 / 2.4) - 0.055)


def color_space_transformer(pred, gt, color_space="linear"):
    """nerfs/color_space.py:22-66."""
    gt = gt.clamp(0, 1)
    if color_space == "linear":
        return pred.clamp(0, 1), srgb_to_linear(gt).clamp(0, 1)
    if color_space == "srgb":
        return linear_to_srgb(pred).clamp(0, 1), gt
    if color_space == "identity":
        return pred, gt
    raise ValueError(color_space)


def mse_loss(pred, gt, color_space="linear"):
    """nerfs/losses.py:10-32 — F.mse_loss(mean) after color_space_transformer."""
    a, b = color_space_transformer(pred, gt, color_space)
    return F.mse_loss(a, b)


def psnr(mse):
    """an/utils.py:538-539 (image PSNR uses mse.clamp_min(1e-8), runtime_adapt.py:157)."""
    return -10.0 * math.log10(max(float(mse), 1e-8))


class OracleTrainer:
    """One reference-style train step (pipelines/online_stage/runtime_adapt.py:286-310):
    render → MSE (coarse + fine when hierarchical) → backward → clip_grad_norm_(1.0) → Adam.

    Param groups follow models/inr/meta_ngp.py:446-469 ('sigma' = trunk+heads, 'color' = colour MLP)
    with per-group lr (common/utils.py:16-76).

    amp="fp16": the use_amp=True body (runtime_adapt.py:290-310) — the MLPs under the autocast(float16) restatement
    of _lin, the loss scaled by ``loss_scale`` for the backward and the gradients unscaled (GradScaler.unscale_
    multiplies by 1/scale) before the clip; a step whose gradients hold an inf / nan is skipped, as GradScaler.step
    does (the returned loss is still the step's), and the scale follows GradScaler.update's defaults (torch.amp
    GradScaler: backoff_factor 0.5 on a skipped step, growth_factor 2.0 after growth_interval 2000 clean steps in a
    row), so multi-step oracle AMP runs keep the reference's scale trajectory."""

    def __init__(self, p_coarse, p_fine=None, lr_sigma=2e-3, lr_color=2e-3, betas=(0.9, 0.999),
                 eps=1e-8, grad_clip=1.0, color_space="linear", amp=None, loss_scale=65536.0):
        self.nets = [OrderedDict((k, v.clone().requires_grad_(True)) for k, v in p_coarse.items())]
        if p_fine is not None:
            self.nets.append(OrderedDict((k, v.clone().requires_grad_(True)) for k, v in p_fine.items()))
        sig, col = [], []
        for net in self.nets:
            for k, v in net.items():
                (col if k.startswith("color_mlp") else sig).append(v)
        self.params = sig + col
        self.opt = torch.optim.Adam([{"params": sig, "lr": lr_sigma}, {"params": col, "lr": lr_color}],
                                    betas=betas, eps=eps)
        self.grad_clip = grad_clip
        self.color_space = color_space
        self.amp = amp
        self.loss_scale = float(loss_scale) if amp else 1.0
        self._growth_tracker = 0  # GradScaler's count of consecutive finite steps

    def step(self, rays, gt, S, n_importance=0, training=True, u_strat=None, u_pdf=None, bg="white"):
        self.opt.zero_grad()
        pf = self.nets[1] if len(self.nets) > 1 else None
        rgb, depth, w, acc, ex = render_rays(self.nets[0], rays, S, training, u_strat, bg, pf,
                                             n_importance, u_pdf, amp=self.amp)
        loss = mse_loss(rgb, gt, self.color_space)
        if n_importance > 0:
            loss = loss + mse_loss(ex["rgb_coarse"], gt, self.color_space)
        (loss * self.loss_scale).backward()
        finite = True
        if self.amp:
            inv = 1.0 / self.loss_scale
            for q in self.params:
                if q.grad is not None:
                    q.grad.mul_(inv)
                    finite = finite and bool(torch.isfinite(q.grad).all())
        if self.grad_clip is not None:
            torch.nn.utils.clip_grad_norm_(self.params, self.grad_clip)
        if finite:
            self.opt.step()
        if self.amp:  # GradScaler.update (torch/amp/grad_scaler.py defaults)
            if not finite:
                self.loss_scale *= 0.5
                self._growth_tracker = 0
            else:
                self._growth_tracker += 1
                if self._growth_tracker == 2000:
                    self.loss_scale *= 2.0
                    self._growth_tracker = 0
        return float(loss.detach())
