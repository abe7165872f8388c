"""CPU restatement of the reference's Instant-NGP expert — TEST INFRASTRUCTURE ONLY.

Same rules as ``nerf_oracle.py``: only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module, and only as the checker.  The product path
(``nerf-sys_amd/nerf_amd/ngp.py`` + ``csrc/ngp.hip``) never imports it.

Restates, in plain PyTorch on the CPU (autograd supplies the reference gradients), the torch
fallbacks the reference runs when tiny-cuda-nn is absent (paths relative to
``/root/reference/adaptive_nerf``):

* ``components_from_spherical_harmonics`` / ``SHEncoder.forward``   models/encodings.py:27-81, :133-151
* ``HashGridEncoder`` (ctor :175-270, ``_hash`` :288-297, ``_gather`` :299-311,
  ``_torch_forward`` :313-381)                                       models/encodings.py
* ``MetaNGP`` forward (``_world_to_unit`` :166-169, ``_enc_xyz`` :171-174, ``_enc_dir`` :176-179,
  ``color`` :182-201, ``density`` :203-239, ``forward`` :241-255, ctor :21-107)
                                                                     models/inr/meta_ngp.py
* ``MetaLinear.forward`` (x W^T + b)                                 models/metamodule/metamodule.py:140-156

Parity is PINNED against golden vectors produced by importing the reference
(``tools/gen_golden.py`` → ``tests/golden/ngp.npz``).  tiny-cuda-nn's own HashGrid (which keeps
the coarse levels dense and computes in fp16) is NOT what the reference runs here and is
**parity unpinned** (no source in the image); this restatement follows the torch fallback.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import torch

SH_C = (0.28209479177387814, 0.4886025119029199, 1.0925484305920792, 0.9461746957575601,
        0.31539156525251999, 0.5462742152960396, 0.5900435899266435, 2.890611442640554,
        0.4570457994644658, 0.3731763325901154, 1.445305721320277, 2.5033429417967046,
        1.7701307697799304, 0.6690465435572892, 0.10578554691520431, 0.47308734787878004,
        0.6258357354491761)


def sh_components(degree, d):
    """models/encodings.py:27-81 — real SH up to `degree` of (assumed unit) directions."""
    x, y, z = d[..., 0], d[..., 1], d[..., 2]
    xx, yy, zz = x * x, y * y, z * z
    c = d.new_zeros((*d.shape[:-1], (degree + 1) ** 2))
    c[..., 0] = 0.28209479177387814
    if degree > 0:
        c[..., 1] = 0.4886025119029199 * y
        c[..., 2] = 0.4886025119029199 * z
        c[..., 3] = 0.4886025119029199 * x
    if degree > 1:
        c[..., 4] = 1.0925484305920792 * x * y
        c[..., 5] = 1.0925484305920792 * y * z
        c[..., 6] = 0.9461746957575601 * zz - 0.31539156525251999
        c[..., 7] = 1.0925484305920792 * x * z
        c[..., 8] = 0.5462742152960396 * (xx - yy)
    if degree > 2:
        c[..., 9] = 0.5900435899266435 * y * (3 * xx - yy)
        c[..., 10] = 2.890611442640554 * x * y * z
        c[..., 11] = 0.4570457994644658 * y * (5 * zz - 1)
        c[..., 12] = 0.3731763325901154 * z * (5 * zz - 3)
        c[..., 13] = 0.4570457994644658 * x * (5 * zz - 1)
        c[..., 14] = 1.445305721320277 * z * (xx - yy)
        c[..., 15] = 0.5900435899266435 * x * (xx - 3 * yy)
    if degree > 3:
        c[..., 16] = 2.5033429417967046 * x * y * (xx - yy)
        c[..., 17] = 1.7701307697799304 * y * z * (3 * xx - yy)
        c[..., 18] = 0.9461746957575601 * x * y * (7 * zz - 1)
        c[..., 19] = 0.6690465435572892 * y * z * (7 * zz - 3)
        c[..., 20] = 0.10578554691520431 * (35 * zz * zz - 30 * zz + 3)
        c[..., 21] = 0.6690465435572892 * x * z * (7 * zz - 3)
        c[..., 22] = 0.47308734787878004 * (xx - yy) * (7 * zz - 1)
        c[..., 23] = 1.7701307697799304 * x * z * (xx - 3 * yy)
        c[..., 24] = 0.6258357354491761 * (xx * (xx - 3 * yy) - yy * (3 * xx - yy))
    return c


def sh_encode(d, levels=4):
    """SHEncoder.forward (models/encodings.py:133-151): normalise (clamp 1e-9), then components."""
    d = d / d.norm(dim=-1, keepdim=True).clamp_min(1e-9)
    return sh_components(levels - 1, d)


def freq_encode(x, n_freq, include_input=True):
    """FrequencyEncoder.torch_forward (models/encodings.py:437-444)."""
    bands = 2.0 ** torch.arange(n_freq, dtype=torch.float32)
    xe = x[..., None] * bands.to(x.dtype)
    pe = torch.cat([torch.cos(xe), torch.sin(xe)], -1).reshape(*x.shape[:-1], x.shape[-1] * 2 * n_freq)
    return torch.cat([x, pe], -1) if include_input else pe


def hash_resolutions(levels, min_res, max_res):
    """HashGridEncoder ctor (models/encodings.py:196-210): growth factor in float64, the per-level
    resolutions floor(min_res * growth**arange(L)) evaluated in float32 as the reference does."""
    g = 1.0 if levels <= 1 else float(math.exp((math.log(max_res) - math.log(min_res)) / (levels - 1)))
    lv = torch.arange(levels, dtype=torch.float32)
    return torch.floor(min_res * (g ** lv)).to(torch.int32), g


def hash_index(ix, iy, iz, log2_T):
    """HashGridEncoder._hash (models/encodings.py:288-297): int64 products with the primes
    [1, 2654435761, 805459861], XOR, modulo 2^log2_T."""
    return ((ix.to(torch.int64) * 1) ^ (iy.to(torch.int64) * 2654435761)
            ^ (iz.to(torch.int64) * 805459861)) % (2 ** log2_T)


def hash_encode(table, x01, res, log2_T, F, interpolation="Linear"):
    """HashGridEncoder._torch_forward (models/encodings.py:313-381).  table (L*T, F)."""
    L = res.numel()
    T = 2 ** log2_T
    offs = torch.arange(L, dtype=torch.int64) * T
    scaled = x01[..., None, :] * res.to(x01.dtype).view(*([1] * (x01.ndim - 1)), L, 1)

    def gather(ix, iy, iz):
        return table[hash_index(ix, iy, iz, log2_T) + offs]

    if interpolation == "Nearest":
        idx = torch.round(scaled).to(torch.int64)
        return gather(idx[..., 0], idx[..., 1], idx[..., 2]).reshape(*x01.shape[:-1], L * F)
    fl = torch.floor(scaled)
    fr = scaled - fl
    fl = fl.to(torch.int64)
    ce = fl + 1
    f000 = gather(fl[..., 0], fl[..., 1], fl[..., 2])
    f001 = gather(fl[..., 0], fl[..., 1], ce[..., 2])
    f010 = gather(fl[..., 0], ce[..., 1], fl[..., 2])
    f011 = gather(fl[..., 0], ce[..., 1], ce[..., 2])
    f100 = gather(ce[..., 0], fl[..., 1], fl[..., 2])
    f101 = gather(ce[..., 0], fl[..., 1], ce[..., 2])
    f110 = gather(ce[..., 0], ce[..., 1], fl[..., 2])
    f111 = gather(ce[..., 0], ce[..., 1], ce[..., 2])
    wx, wy, wz = fr[..., 0:1], fr[..., 1:2], fr[..., 2:3]
    if interpolation == "Smoothstep":
        wx = wx * wx * (3 - 2 * wx)
        wy = wy * wy * (3 - 2 * wy)
        wz = wz * wz * (3 - 2 * wz)
    c00 = f000 * (1 - wx) + f100 * wx
    c01 = f001 * (1 - wx) + f101 * wx
    c10 = f010 * (1 - wx) + f110 * wx
    c11 = f011 * (1 - wx) + f111 * wx
    c0 = c00 * (1 - wy) + c10 * wy
    c1 = c01 * (1 - wy) + c11 * wy
    return (c0 * (1 - wz) + c1 * wz).flatten(start_dim=-2)


def ngp_param_shapes(in_dim, hidden=64, sigma_depth=2, geo_feat_dim=15, color_hidden=64, color_depth=3,
                     dir_dim=16):
    """Parameter names/shapes of MetaNGP (models/inr/meta_ngp.py:81-105) minus the hash table."""
    s = OrderedDict()
    last = in_dim
    for i in range(sigma_depth):
        s[f"sigma_trunk.{i}.linear.weight"] = (hidden, last)
        s[f"sigma_trunk.{i}.linear.bias"] = (hidden,)
        last = hidden
    s["sigma_head.weight"] = (1, last)
    s["sigma_head.bias"] = (1,)
    s["geo_head.weight"] = (geo_feat_dim, last)
    s["geo_head.bias"] = (geo_feat_dim,)
    last = geo_feat_dim + dir_dim
    for j in range(color_depth):
        s[f"color_mlp.{j}.linear.weight"] = (color_hidden, last)
        s[f"color_mlp.{j}.linear.bias"] = (color_hidden,)
        last = color_hidden
    s[f"color_mlp.{color_depth}.weight"] = (3, last)
    s[f"color_mlp.{color_depth}.bias"] = (3,)
    return s


def _lin(x, p, name):
    return x.matmul(p[name + ".weight"].t()) + p[name + ".bias"]


class _TruncExp(torch.autograd.Function):
    """models/trunc_exp.py:43-57 — gradient exp(clamp(x)) also outside the clamp."""

    @staticmethod
    def forward(ctx, x):
        xc = x.clamp(-88.722839111, 88.722839111)
        ctx.save_for_backward(xc)
        return torch.exp(xc)

    @staticmethod
    def backward(ctx, g):
        (xc,) = ctx.saved_tensors
        return g * torch.exp(xc)


def ngp_forward(p, table, x_d, aabb, res, log2_T, F, **kw):
    """MetaNGP.forward (models/inr/meta_ngp.py:241-255) -> (M,4) [rgb, sigma], with the reference's
    trunc_exp autograd.  kw: sigma_depth, color_depth, dir_encoding, interpolation, use_sigmoid_rgb, enc_eps."""
    x, d = x_d[..., :3], x_d[..., 3:6]
    sd, cd = kw.get("sigma_depth", 2), kw.get("color_depth", 3)
    extent = aabb[1] - aabb[0]
    x01 = ((x - aabb[0]) / extent).clamp(kw.get("enc_eps", 1e-6), 1.0 - kw.get("enc_eps", 1e-6))
    h = hash_encode(table, x01, res, log2_T, F, kw.get("interpolation", "Linear"))
    for i in range(sd):
        h = torch.relu(_lin(h, p, f"sigma_trunk.{i}.linear"))
    sigma = _TruncExp.apply(_lin(h, p, "sigma_head"))
    geo = _lin(h, p, "geo_head")
    dn = d / d.norm(dim=-1, keepdim=True).clamp_min(1e-9)
    d_enc = sh_encode(dn, 4) if kw.get("dir_encoding", "spherical") == "spherical" else freq_encode(dn, 4)
    c = torch.cat([geo, d_enc], -1)
    for j in range(cd):
        c = torch.relu(_lin(c, p, f"color_mlp.{j}.linear"))
    c = _lin(c, p, f"color_mlp.{cd}")
    rgb = torch.sigmoid(c) if kw.get("use_sigmoid_rgb", True) else c
    return torch.cat([rgb, sigma], -1)


ngp_forward_ad = ngp_forward
