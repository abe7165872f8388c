"""Typed wrappers over the C-ABI: allocate outputs with torch (caller-owned buffers), launch on the
current stream, raise on a non-zero status.  No autograd here (see ray_rendering / vanilla)."""
from __future__ import annotations

import ctypes
from typing import Sequence

import torch

from ._lib import check, lib, need, ptr, stream

F32 = torch.float32
_CS = {"linear": 0, "srgb": 1, "identity": 2}


def _empty(shape, like):
    return torch.empty(shape, dtype=F32, device=like.device)


def rays_gen(c2w, H, W, fx, fy, cx, cy, *, pix=None, near=None, far=None, aabb=None, center_pixels=True,
             images_u8=None, aabb_max_bound=1e10, aabb_invalid=1e10):
    """get_rays(get_ray_directions(...)) for a dense image (pix=None) or a batch of (img,row,col)."""
    need(c2w, "c2w")
    if c2w.dim() == 2:
        c2w = c2w[:3, :4].reshape(1, 3, 4).contiguous()
    c2w = c2w[..., :3, :4].contiguous()
    n_poses = c2w.shape[0]
    if pix is not None:
        need(pix, "pix", torch.int32)
        n = pix.shape[0]
    else:
        n = H * W
    if aabb is None and (near is None or far is None):
        raise ValueError("Provide near/far when scene_box is None")
    if aabb is not None:
        aabb = need(aabb.reshape(6).contiguous(), "aabb")
    rays = torch.empty((n, 8), dtype=F32, device=c2w.device)
    rgb = torch.empty((n, 3), dtype=F32, device=c2w.device) if images_u8 is not None else None
    if images_u8 is not None:
        need(images_u8, "images_u8", torch.uint8)
    st = lib().nerf_rays_gen(ptr(c2w), n_poses, ptr(pix), n, H, W, fx, fy, cx, cy, int(center_pixels),
                             float(near or 0.0), float(far or 0.0), ptr(aabb), aabb_max_bound, aabb_invalid,
                             ptr(images_u8), ptr(rays), ptr(rgb), stream())
    check(st, "nerf_rays_gen")
    return (rays, rgb) if images_u8 is not None else rays


def pick_pixels(n, n_images, H, W, seed, device, step_dev=None, seed_mul=0):
    """n random (image, row, col) triples of the counter RNG stream ``seed``; with ``step_dev`` (int64 device
    counter) the stream is seed + step_dev * seed_mul, read by the kernel (captured train-step graphs)."""
    pix = torch.empty((n, 3), dtype=torch.int32, device=device)
    if step_dev is not None:
        need(step_dev, "step_dev", torch.int64)
        check(lib().nerf_pick_pixels_dseed(n, n_images, H, W, ctypes.c_uint64(seed & (2**64 - 1)),
                                           ctypes.c_uint64(seed_mul & (2**64 - 1)), ptr(step_dev), ptr(pix),
                                           stream()), "nerf_pick_pixels_dseed")
        return pix
    check(lib().nerf_pick_pixels(n, n_images, H, W, ctypes.c_uint64(seed & (2**64 - 1)), ptr(pix), stream()),
          "nerf_pick_pixels")
    return pix


def clamp_near_far(rays, near=None, far=None, eps=1e-6, invalid_value=float("inf")):
    need(rays, "rays")
    rays = rays.clone()
    valid = torch.empty(rays.shape[0], dtype=torch.uint8, device=rays.device)
    check(lib().nerf_clamp_near_far(ptr(rays), rays.shape[0], int(near is not None), float(near or 0.0),
                                    int(far is not None), float(far or 0.0), eps, invalid_value, ptr(valid),
                                    stream()), "nerf_clamp_near_far")
    return rays, valid.bool()


def rays_ndc(rays, H, W, focal, near_plane=1.0):
    need(rays, "rays")
    out = torch.empty_like(rays)
    check(lib().nerf_rays_ndc(ptr(rays), rays.shape[0], H, W, focal, near_plane, ptr(out), stream()), "nerf_rays_ndc")
    return out


def sample_stratified(rays, S, randomized, u=None, seed=0):
    need(rays, "rays")
    if u is not None:
        need(u, "u")
    t = _empty((rays.shape[0], S), rays)
    check(lib().nerf_sample_stratified(ptr(rays), rays.shape[0], S, int(bool(randomized)), ptr(u),
                                       ctypes.c_uint64(seed & (2**64 - 1)), ptr(t), stream()),
          "nerf_sample_stratified")
    return t


def build_xd(rays, t):
    need(rays, "rays"), need(t, "t")
    n, S = t.shape
    xd = _empty((n * S, 6), rays)
    check(lib().nerf_build_xd(ptr(rays), ptr(t), n, S, ptr(xd), stream()), "nerf_build_xd")
    return xd


def sample_pdf(t, w, n_imp, u=None, det=False, seed=0):
    need(t, "t"), need(w, "weights")
    if u is not None:
        need(u, "u")
    n, S = t.shape
    out = _empty((n, S + n_imp), t)
    check(lib().nerf_sample_pdf(ptr(t), ptr(w), n, S, n_imp, ptr(u), int(bool(det)),
                                ctypes.c_uint64(seed & (2**64 - 1)), ptr(out), stream()), "nerf_sample_pdf")
    return out


def freq_encode(x, L, include_input=True):
    need(x, "x")
    D = x.shape[-1]
    flat = x.reshape(-1, D)
    od = D * (2 * L + (1 if include_input else 0))
    out = _empty((flat.shape[0], od), x)
    check(lib().nerf_freq_encode(ptr(flat), flat.shape[0], D, L, int(include_input), ptr(out), od, stream()),
          "nerf_freq_encode")
    return out.view(*x.shape[:-1], od)


# ------------------------------------------------------------------ MLP


PRECISIONS = ("fp32", "bf16", "fp16")
# the 16-bit builds of the fused MLP kernels (include/nerf_amd.h): bf16 (configs[2], autocast(bfloat16)) and fp16 (the
# reference's autocast(float16) operands and rounding points, runtime_adapt.py:291-310)
_H16 = {"bf16": "bf16", "fp16": "f16"}
# bf16 path selection (include/nerf_amd.h): 0 = the fused production kernels; the layered launches are their
# bitwise references.  A workspace's backward must use the NERF_BF16_LAYERED_BWD bit of its training forward.
BF16_LAYERED_FWD = 1
BF16_LAYERED_BWD = 2


def _check_precision(precision):
    if precision not in PRECISIONS:
        raise ValueError(f"precision must be one of {PRECISIONS}, got {precision!r}")


def mlp_workspace_bytes(M, training, precision="fp32"):
    _check_precision(precision)
    if precision in _H16:
        return getattr(lib(), f"nerf_mlp_workspace_bytes_{_H16[precision]}")(M, int(training))
    return lib().nerf_mlp_workspace_bytes(M, int(training))


def mlp_workspace_bytes_2s(M):
    """Workspace of the two-stream fp32 backward (nerf_mlp_bwd_2s): one input-gradient buffer per trunk layer."""
    return lib().nerf_mlp_workspace_bytes_2s(M)


def mlp_workspace(M, training, device, precision="fp32"):
    return torch.empty(mlp_workspace_bytes(M, training, precision), dtype=torch.uint8, device=device)


def _events_arg(events):
    if events is None:
        return None
    arr = (ctypes.c_void_p * len(events))(*[ctypes.c_void_p(e.cuda_event) for e in events])
    return arr


# fp32 GEMM engine flags (include/nerf_amd.h): 0 = bf16 split products (default), NATIVE_FP32 = fp32 MFMA kernels
MLP_NATIVE_FP32 = 1
MLP_NATIVE_DGRAD = 2  # backward only: input-gradient GEMMs on the fp32 MFMA (default: split, small-term accumulators)


def mlp_fwd(w_packed, x_d, ws, training, out=None, events=None, precision="fp32", bf16_flags=0, fp32_flags=0):
    need(w_packed, "packed weights"), need(x_d, "x_d")
    _check_precision(precision)
    M = x_d.shape[0]
    if out is None:
        out = _empty((M, 4), x_d)
    if precision in _H16:
        fn = f"nerf_mlp_fwd_{_H16[precision]}"
        check(getattr(lib(), fn)(ptr(w_packed), ptr(x_d), M, ptr(out), ptr(ws), ws.numel(), int(training),
                                 int(bf16_flags), _events_arg(events), stream()), fn)
        return out
    check(lib().nerf_mlp_fwd_ex(ptr(w_packed), ptr(x_d), M, ptr(out), ptr(ws), ws.numel(), int(training),
                                int(fp32_flags) & MLP_NATIVE_FP32,  # MLP_NATIVE_DGRAD is a backward-only flag
                                _events_arg(events), stream()), "nerf_mlp_fwd_ex")
    return out


def mlp_bwd(w_packed, M, d_rgb_sigma, ws, d_w=None, accumulate=False, events=None, precision="fp32", bf16_flags=0,
            wgrad_stream=None, sync=None, fp32_flags=0):
    """wgrad_stream (fp32 only): run the weight-gradient GEMMs there (nerf_mlp_bwd_2s; sync = 10 torch.cuda.Events,
    ws from mlp_workspace_bytes_2s); d_w is complete in the current stream's order either way."""
    need(w_packed, "packed weights"), need(d_rgb_sigma, "d_rgb_sigma")
    _check_precision(precision)
    if d_w is None:
        d_w = torch.empty_like(w_packed)
        accumulate = False
    if precision in _H16:
        fn = f"nerf_mlp_bwd_{_H16[precision]}"
        check(getattr(lib(), fn)(ptr(w_packed), M, ptr(d_rgb_sigma), ptr(d_w), int(accumulate), ptr(ws),
                                 ws.numel(), int(bf16_flags), _events_arg(events), stream()), fn)
        return d_w
    if wgrad_stream is not None:
        if sync is None or len(sync) < 10:
            raise ValueError("nerf_mlp_bwd_2s needs 10 sync events")
        for e in sync:  # torch creates an event's HIP handle at its first record
            if not e.cuda_event:
                e.record()
        check(lib().nerf_mlp_bwd_2s_ex(ptr(w_packed), M, ptr(d_rgb_sigma), ptr(d_w), int(accumulate), ptr(ws),
                                       ws.numel(), int(fp32_flags), _events_arg(events), stream(),
                                       ctypes.c_void_p(wgrad_stream.cuda_stream), _events_arg(sync)),
              "nerf_mlp_bwd_2s_ex")
        return d_w
    check(lib().nerf_mlp_bwd_ex(ptr(w_packed), M, ptr(d_rgb_sigma), ptr(d_w), int(accumulate), ptr(ws), ws.numel(),
                                int(fp32_flags), _events_arg(events), stream()), "nerf_mlp_bwd_ex")
    return d_w


# ------------------------------------------------------------------ compositing


def composite_fwd(rgb_sigma, t, bg=None, sigma_scale=1.0, gt=None, color_space="linear", inv_count=None,
                  loss_sum=None, outs=None):
    need(rgb_sigma, "rgb_sigma"), need(t, "t")
    n, S = t.shape
    if bg is not None:
        need(bg, "bg")
    if outs is None:
        rgb, depth, w, acc = _empty((n, 3), t), _empty((n,), t), _empty((n, S), t), _empty((n,), t)
    else:
        rgb, depth, w, acc = outs
    d_rgb = None
    if gt is not None:
        need(gt, "gt")
        d_rgb = _empty((n, 3), t)
        if loss_sum is None:
            loss_sum = torch.zeros(1, dtype=F32, device=t.device)
        if inv_count is None:
            inv_count = 1.0 / (3 * n)
    cs = _CS.get(color_space)
    if cs is None:
        raise ValueError(f"Invalid color_space={color_space!r}; use 'linear'|'srgb'|'identity'")
    check(lib().nerf_composite_fwd(ptr(rgb_sigma), ptr(t), ptr(bg), n, S, float(sigma_scale), ptr(rgb), ptr(depth),
                                   ptr(w), ptr(acc), ptr(gt), cs, float(inv_count or 0.0), ptr(loss_sum),
                                   ptr(d_rgb), stream()), "nerf_composite_fwd")
    if gt is not None:
        return rgb, depth, w, acc, loss_sum, d_rgb
    return rgb, depth, w, acc


def composite_bwd(rgb_sigma, t, bg, g_rgb, g_depth=None, g_acc=None, g_w=None, sigma_scale=1.0, out=None):
    need(rgb_sigma, "rgb_sigma"), need(t, "t"), need(g_rgb, "g_rgb")
    n, S = t.shape
    if rgb_sigma.numel() != n * S * 4 or rgb_sigma.shape[-1] != 4:   # (N,S,4) or the MLP's (N*S,4)
        raise ValueError(f"rgb_sigma must hold ({n},{S},4), got {tuple(rgb_sigma.shape)}")
    if tuple(g_rgb.shape) != (n, 3):
        raise ValueError(f"g_rgb must be ({n},3), got {tuple(g_rgb.shape)}")
    for x, name, shape in ((bg, "bg", (n, 3)), (g_depth, "g_depth", (n,)), (g_acc, "g_acc", (n,)),
                           (g_w, "g_w", (n, S))):
        if x is not None:
            need(x, name)
            if tuple(x.shape) != shape:
                raise ValueError(f"{name} must be {shape}, got {tuple(x.shape)}")
    if out is None:
        out = torch.empty_like(rgb_sigma)
    else:
        need(out, "out")
    check(lib().nerf_composite_bwd(ptr(rgb_sigma), ptr(t), ptr(bg), n, S, float(sigma_scale), ptr(g_rgb),
                                   ptr(g_depth), ptr(g_acc), ptr(g_w), ptr(out), stream()), "nerf_composite_bwd")
    return out


# ------------------------------------------------------------------ optimiser


def grad_sqnorm(g, partials=None):
    if partials is None:
        partials = torch.empty(256, dtype=F32, device=g.device)
    check(lib().nerf_grad_sqnorm(ptr(g), g.numel(), ptr(partials), stream()), "nerf_grad_sqnorm")
    return partials


def adam(p, g, m, v, seg_off: Sequence[int], seg_lr: Sequence[float], step, betas=(0.9, 0.999), eps=1e-8,
         weight_decay=0.0, partials=None, max_norm=0.0):
    """nerf_adam; ``step`` an int, or an int64 device tensor holding the step count (nerf_adam_dstep)."""
    off = (ctypes.c_int64 * len(seg_off))(*seg_off)
    lr = (ctypes.c_double * len(seg_lr))(*seg_lr)
    if isinstance(step, torch.Tensor):
        need(step, "step", torch.int64)
        check(lib().nerf_adam_dstep(ptr(p), ptr(g), ptr(m), ptr(v), p.numel(), off, lr, len(seg_lr), betas[0],
                                    betas[1], eps, weight_decay, ptr(step), ptr(partials), max_norm, stream()),
              "nerf_adam_dstep")
        return
    check(lib().nerf_adam(ptr(p), ptr(g), ptr(m), ptr(v), p.numel(), off, lr, len(seg_lr), betas[0], betas[1], eps,
                          weight_decay, step, ptr(partials), max_norm, stream()), "nerf_adam")


def packed_points(rays, ray_idx, t0, t1):
    """nerf_packed_points: x_d (M,6) = [o + d (t0+t1)/2, d] of packed intervals."""
    M = ray_idx.numel()
    xd = torch.empty((M, 6), dtype=F32, device=rays.device)
    check(lib().nerf_packed_points(ptr(rays), ptr(ray_idx.to(torch.int32).contiguous()), ptr(t0), ptr(t1), M, ptr(xd),
                                   stream()), "nerf_packed_points")
    return xd
