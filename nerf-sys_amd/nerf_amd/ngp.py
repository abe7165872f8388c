"""The Instant-NGP expert on the HIP kernels: ``HashGridEncoder``, ``SHEncoder`` and
``InstantNGP`` — drop-in mirrors of the reference's torch backends

    HashGridEncoder   models/encodings.py:158-381   (torch fallback: int64 hash, every level hashed)
    SHEncoder         models/encodings.py:84-151    (real SH, degree levels-1)
    MetaNGP           models/inr/meta_ngp.py:15-255, get_param_groups :446-469

with the same constructor arguments, parameter names (``xyz_encoder.hash_table``,
``sigma_trunk.{i}.linear.*``, ``sigma_head.*``, ``geo_head.*``, ``color_mlp.{j}.linear.*``,
``color_mlp.{D}.*``), the expert contract ``expert(x_d (M,6), params=None) -> (M,4)`` and the MetaModule
fast-weights surface (the hash table is not a fast weight, as in the reference: HashGridEncoder is not a
MetaModule, metamodule.py:20-30).

Compute: ``nerf_hash_encode`` (gather, world->unit mapping fused) -> ``nerf_ngp_fwd`` (all MLP layers in
one fused fp32-MFMA kernel) ; backward ``nerf_ngp_bwd`` (forward recomputed on chip, weight gradients
reduced per workgroup) -> ``nerf_hash_encode_bwd`` (fp32 atomics into the table gradient).  No CPU
fallback: every op requires HIP tensors.  ``use_occ`` builds an occupancy grid (``occupancy.OccGridEstimator``,
§8f row 2) with MetaNGP's marching / update / premark methods; ``render_rays`` then takes the packed
occupancy renderer once ``occ_ready``.
"""
from __future__ import annotations

import contextlib
import ctypes
import math
import warnings
from collections import OrderedDict
from typing import Dict, Optional

import torch
import torch.nn as nn
from torch.autograd.function import once_differentiable

from ._lib import check, lib, need, ptr, stream
from .vanilla import VanillaNeRF

_INTERP = {"Nearest": 0, "Linear": 1, "Smoothstep": 2}


class NerfHashGrid(ctypes.Structure):
    _fields_ = [("levels", ctypes.c_int32), ("features_per_level", ctypes.c_int32),
                ("log2_hashmap_size", ctypes.c_int32), ("interpolation", ctypes.c_int32),
                ("resolutions", ctypes.c_int32 * 32)]


class NerfNgpNet(ctypes.Structure):
    _fields_ = [("in_dim", ctypes.c_int32), ("hidden", ctypes.c_int32), ("sigma_depth", ctypes.c_int32),
                ("geo_feat_dim", ctypes.c_int32), ("color_hidden", ctypes.c_int32),
                ("color_depth", ctypes.c_int32), ("dir_encoding", ctypes.c_int32), ("sh_levels", ctypes.c_int32),
                ("use_sigmoid_rgb", ctypes.c_int32), ("generic_kernels", ctypes.c_int32)]


def _addr(s):
    return ctypes.c_void_p(ctypes.addressof(s))


class _Timing:
    """Optional HIP-event timing of the expert's launches on the current stream (benches): no host sync."""

    def __init__(self):
        self.enabled = False
        self.records = []

    def start(self, name, rows=0):
        if not self.enabled:
            return None
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        return (name, e0, e1, rows)

    def stop(self, h):
        if h is not None:
            h[2].record()
            self.records.append(h)

    def collect(self):
        """-> {name: [(ms, rows) per launch]}"""
        torch.cuda.synchronize()
        out = {}
        for name, e0, e1, rows in self.records:
            if isinstance(rows, torch.Tensor):  # device-sized launches: the (lo, hi) row range on the device
                r = rows.cpu()
                rows = int(r[1]) - int(r[0])
            out.setdefault(name, []).append((e0.elapsed_time(e1), rows))
        self.records = []
        return out


TIMING = _Timing()


# ------------------------------------------------------------------------------------------ kernel wrappers

def hash_encode(grid: NerfHashGrid, table, x, aabb=None, enc_eps=1e-6, out_stride=None):
    """nerf_hash_encode: x (M, >=3) rows (pitch = x.stride(0)); aabb: host sequence of 6 floats or None."""
    need(table, "hash_table")
    if x.stride(-1) != 1:
        x = x.contiguous()
    M = x.shape[0]
    od = grid.levels * grid.features_per_level
    os_ = out_stride or od
    out = torch.empty((M, os_), dtype=torch.float32, device=x.device)
    ab = (ctypes.c_float * 6)(*[float(v) for v in aabb]) if aabb is not None else None
    check(lib().nerf_hash_encode(_addr(grid), ptr(table), ptr(x), x.stride(0), M, ab, float(enc_eps), ptr(out),
                                 os_, stream()), "nerf_hash_encode")
    return out


def hash_encode_bwd(grid: NerfHashGrid, x, d_out, n_table_rows, aabb=None, enc_eps=1e-6, d_table=None):
    if x.stride(-1) != 1:
        x = x.contiguous()
    need(d_out, "d_out")
    if d_table is None:
        d_table = torch.zeros((n_table_rows, grid.features_per_level), dtype=torch.float32, device=x.device)
    ab = (ctypes.c_float * 6)(*[float(v) for v in aabb]) if aabb is not None else None
    check(lib().nerf_hash_encode_bwd(_addr(grid), ptr(x), x.stride(0), x.shape[0], ab, float(enc_eps), ptr(d_out),
                                     d_out.stride(0), ptr(d_table), stream()), "nerf_hash_encode_bwd")
    return d_table


def sh_encode(d, levels=4):
    if d.stride(-1) != 1:
        d = d.contiguous()
    need(d if d.is_contiguous() else d.contiguous(), "d")
    out = torch.empty((d.shape[0], levels * levels), dtype=torch.float32, device=d.device)
    check(lib().nerf_sh_encode(ptr(d), d.stride(0), d.shape[0], int(levels), ptr(out), levels * levels, stream()),
          "nerf_sh_encode")
    return out


def ngp_fwd(net: NerfNgpNet, w_packed, enc, x_d, out=None):
    """nerf_ngp_fwd: enc (M, >=in_dim), x_d (M,6) -> rgb_sigma (M,4)."""
    M = x_d.shape[0]
    if out is None:
        out = torch.empty((M, 4), dtype=torch.float32, device=x_d.device)
    check(lib().nerf_ngp_fwd(_addr(net), ptr(w_packed), ptr(enc), enc.stride(0), ptr(x_d), M, ptr(out), stream()),
          "nerf_ngp_fwd")
    return out


E_UNSUPPORTED = -5


def ngp_fwd_enc(net: NerfNgpNet, grid: NerfHashGrid, table, w_packed, x_d, aabb=None, enc_eps=1e-6):
    """nerf_ngp_fwd_enc: x_d (M, 6) -> (rgb_sigma (M, 4), enc (M, L*F)) in one launch, or None when the expert's
    shape has no fused kernel (the caller then runs hash_encode + ngp_fwd)."""
    x_d = x_d.contiguous()
    M = x_d.shape[0]
    od = grid.levels * grid.features_per_level
    enc = torch.empty((M, od), dtype=torch.float32, device=x_d.device)
    out = torch.empty((M, 4), dtype=torch.float32, device=x_d.device)
    ab = (ctypes.c_float * 6)(*[float(v) for v in aabb]) if aabb is not None else None
    rc = lib().nerf_ngp_fwd_enc(_addr(net), _addr(grid), ptr(table), ptr(w_packed), ptr(x_d), M, ab, float(enc_eps),
                                ptr(enc), od, ptr(out), stream())
    if rc == E_UNSUPPORTED:
        return None
    check(rc, "nerf_ngp_fwd_enc")
    return out, enc


def ngp_density_enc(net: NerfNgpNet, grid: NerfHashGrid, table, w_packed, x, aabb=None, enc_eps=1e-6):
    """nerf_ngp_density_enc: world points (M, >=3) -> sigma (M,) in one launch (encoding in LDS), or None when
    the expert's shape has no fused kernel (the caller then runs hash_encode + ngp_density)."""
    if x.stride(-1) != 1:
        x = x.contiguous()
    M = x.shape[0]
    out = torch.empty(M, dtype=torch.float32, device=x.device)
    ab = (ctypes.c_float * 6)(*[float(v) for v in aabb]) if aabb is not None else None
    rc = lib().nerf_ngp_density_enc(_addr(net), _addr(grid), ptr(table), ptr(w_packed), ptr(x), x.stride(0), M, ab,
                                    float(enc_eps), ptr(out), stream())
    if rc == E_UNSUPPORTED:
        return None
    check(rc, "nerf_ngp_density_enc")
    return out


def ngp_density(net: NerfNgpNet, w_packed, enc):
    """nerf_ngp_density: enc (M, >=in_dim) -> sigma (M,) (trunk + sigma head only)."""
    M = enc.shape[0]
    out = torch.empty(M, dtype=torch.float32, device=enc.device)
    check(lib().nerf_ngp_density(_addr(net), ptr(w_packed), ptr(enc), enc.stride(0), M, ptr(out), stream()),
          "nerf_ngp_density")
    return out


_WS = {}


def ngp_workspace(net: NerfNgpNet, M, device):
    need_b = max(int(lib().nerf_ngp_workspace_bytes(_addr(net), M)), 16)
    # one buffer per (device, stream): launches on different streams never share a workspace
    key = (str(device), torch.cuda.current_stream(device).cuda_stream)
    ws = _WS.get(key)
    if ws is None or ws.numel() < need_b:
        ws = torch.empty(need_b, dtype=torch.uint8, device=device)
        _WS[key] = ws
    return ws


def ngp_bwd(net: NerfNgpNet, w_packed, enc, x_d, d_rgb_sigma, d_enc=None, d_w=None, accumulate=False):
    """nerf_ngp_bwd -> (d_enc (M, enc pitch), d_w (packed))."""
    M = x_d.shape[0]
    if d_enc is None:
        d_enc = torch.empty_like(enc)
    if d_w is None:
        d_w = torch.empty_like(w_packed)
    ws = ngp_workspace(net, M, x_d.device)
    check(lib().nerf_ngp_bwd(_addr(net), ptr(w_packed), ptr(enc), enc.stride(0), ptr(x_d), M, ptr(d_rgb_sigma),
                             ptr(d_enc), ptr(d_w), int(accumulate), ptr(ws), ws.numel(), stream()), "nerf_ngp_bwd")
    return d_enc, d_w


def ngp_bwd_hash(net: NerfNgpNet, grid: NerfHashGrid, w_packed, enc, x_d, d_rgb_sigma, d_table, aabb=None,
                 enc_eps=1e-6, d_w=None, accumulate=False):
    """nerf_ngp_bwd_hash: MLP backward + table scatter (d_table += ...) in one launch -> d_w, or None when the
    expert's shape has no fused kernel (the caller then runs ngp_bwd + hash_encode_bwd)."""
    M = x_d.shape[0]
    if d_w is None:
        d_w = torch.empty_like(w_packed)
    ws = ngp_workspace(net, M, x_d.device)
    ab = (ctypes.c_float * 6)(*[float(v) for v in aabb]) if aabb is not None else None
    rc = lib().nerf_ngp_bwd_hash(_addr(net), _addr(grid), ptr(w_packed), ptr(enc), enc.stride(0), ptr(x_d), M,
                                 ptr(d_rgb_sigma), ab, float(enc_eps), ptr(d_table), ptr(d_w), int(accumulate),
                                 ptr(ws), ws.numel(), stream())
    if rc == E_UNSUPPORTED:
        return None
    check(rc, "nerf_ngp_bwd_hash")
    return d_w


# ------------------------------------------------------------------------------------------ encoders

def level_resolutions(levels, min_res, max_res):
    """HashGridEncoder ctor (models/encodings.py:196-210): growth factor in float64, resolutions
    floor(min_res * growth**arange(L)) in float32 — the same torch expression, host side."""
    g = 1.0 if levels <= 1 else float(math.exp((math.log(max_res) - math.log(min_res)) / (levels - 1)))
    lv = torch.arange(levels, dtype=torch.float32)
    return torch.floor(min_res * (g ** lv)).to(torch.int32), g


class _HashEncodeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, table, grid, aabb, eps):
        ctx.grid, ctx.aabb, ctx.eps = grid, aabb, eps
        ctx.save_for_backward(x)
        ctx.rows = table.shape[0]
        return hash_encode(grid, table.detach(), x, aabb, eps)

    @staticmethod
    @once_differentiable
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        if ctx.needs_input_grad[0]:
            raise NotImplementedError("HashGridEncoder (HIP): no gradient w.r.t. positions")
        d_table = hash_encode_bwd(ctx.grid, x, g.contiguous(), ctx.rows, ctx.aabb, ctx.eps)
        return None, d_table, None, None, None


class HashGridEncoder(nn.Module):
    """models/encodings.py:158-381 (torch backend semantics).  forward(x (...,3) in [0,1]) -> (..., L*F)."""

    def __init__(self, levels: int = 16, min_res: int = 16, max_res: int = 4096, log2_hashmap_size: int = 19,
                 features_per_level: int = 2, hash_init_scale: float = 1e-3, implementation: str = "tcnn",
                 interpolation: Optional[str] = None) -> None:
        super().__init__()
        self.levels = int(levels)
        self.min_res = int(min_res)
        self.max_res = int(max_res)
        self.features_per_level = int(features_per_level)
        self.log2_hashmap_size = int(log2_hashmap_size)
        self.hash_init_scale = float(hash_init_scale)
        self.hash_table_size = 2 ** self.log2_hashmap_size
        if interpolation is not None and interpolation not in _INTERP:
            warnings.warn(f"[HashGridEncoder] interpolation '{interpolation}' not supported; using 'Linear'.",
                          RuntimeWarning)
            interpolation = "Linear"
        self.interpolation = interpolation
        res, self.growth_factor = level_resolutions(self.levels, self.min_res, self.max_res)
        self.register_buffer("level_resolutions", res, persistent=False)
        self.register_buffer("level_offsets", torch.arange(self.levels, dtype=torch.int64) * self.hash_table_size,
                             persistent=False)
        self._out_dim = self.levels * self.features_per_level
        T = self.hash_table_size * self.levels
        self.hash_table = nn.Parameter((torch.rand(T, self.features_per_level) * 2 - 1) * self.hash_init_scale)
        g = NerfHashGrid()
        g.levels, g.features_per_level, g.log2_hashmap_size = self.levels, self.features_per_level, self.log2_hashmap_size
        g.interpolation = _INTERP[self.interpolation or "Linear"]
        for i, r in enumerate(res.tolist()):
            g.resolutions[i] = int(r)
        self.grid = g

    @property
    def out_dim(self) -> int:
        return self._out_dim

    def get_out_dim(self) -> int:
        return self._out_dim

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        assert x.shape[-1] == 3, f"Expected (...,3), got {tuple(x.shape)}"
        flat = x.reshape(-1, 3).float().contiguous()
        y = _HashEncodeFn.apply(flat, self.hash_table, self.grid, None, 0.0)
        return y.view(*x.shape[:-1], self._out_dim)


class SHEncoder(nn.Module):
    """models/encodings.py:84-151: forward(d (...,3)) -> (..., levels^2) (directions normalised inside)."""

    def __init__(self, levels: int = 4, implementation: str = "tcnn") -> None:
        super().__init__()
        if levels <= 0 or levels > 5:
            raise ValueError(f"Supported levels ∈ [1, 5], got {levels}")
        self.levels = int(levels)
        self.degree = self.levels - 1
        self._out_dim = self.levels ** 2

    @property
    def out_dim(self) -> int:
        return self._out_dim

    def forward(self, d: torch.Tensor) -> torch.Tensor:
        assert d.shape[-1] == 3, f"Expected (...,3); got {tuple(d.shape)}"
        y = sh_encode(d.reshape(-1, 3).float().contiguous(), self.levels)
        return y.view(*d.shape[:-1], self._out_dim)


# ------------------------------------------------------------------------------------------ MetaNGP


class NgpLayout:
    """Packed layout of one MetaNGP network (nerf_ngp_layout) + the index map of its named tensors."""

    def __init__(self, net: NerfNgpNet, shapes: "OrderedDict[str, tuple]", sigma_depth: int, color_depth: int):
        n = ctypes.c_int32(0)
        total = int(lib().nerf_ngp_layout(_addr(net), None, ctypes.c_void_p(ctypes.addressof(n))))
        if total < 0:
            raise ValueError("unsupported MetaNGP configuration for the fused HIP MLP (every width <= 64, "
                             "1+geo_feat_dim <= 32, geo+dir <= 64, <= 12 layers, LDS plan <= 160 KB)")
        tbl = (ctypes.c_int64 * (4 * n.value))()
        lib().nerf_ngp_layout(_addr(net), tbl, ctypes.c_void_p(ctypes.addressof(n)))
        self.total = total
        t = [(tbl[4 * i], tbl[4 * i + 1], tbl[4 * i + 2]) for i in range(n.value)]
        place = {}
        for i in range(sigma_depth):
            place[f"sigma_trunk.{i}.linear.weight"] = (2 * i, 0)
            place[f"sigma_trunk.{i}.linear.bias"] = (2 * i + 1, 0)
        h = sigma_depth
        place["sigma_head.weight"] = (2 * h, 0)
        place["sigma_head.bias"] = (2 * h + 1, 0)
        place["geo_head.weight"] = (2 * h, 1)
        place["geo_head.bias"] = (2 * h + 1, 1)
        for j in range(color_depth):
            place[f"color_mlp.{j}.linear.weight"] = (2 * (h + 1 + j), 0)
            place[f"color_mlp.{j}.linear.bias"] = (2 * (h + 1 + j) + 1, 0)
        place[f"color_mlp.{color_depth}.weight"] = (2 * (h + 1 + color_depth), 0)
        place[f"color_mlp.{color_depth}.bias"] = (2 * (h + 1 + color_depth) + 1, 0)
        self.names = list(shapes)
        idx = []
        for name in self.names:
            ti, r0 = place[name]
            off, _, cols = t[ti]
            shp = shapes[name]
            r = shp[0]
            c = shp[1] if len(shp) == 2 else 1
            idx.append((off + torch.arange(r0, r0 + r).view(-1, 1) * cols + torch.arange(c).view(1, -1)).reshape(-1))
        self.index = torch.cat(idx)
        self._dev = {}
        self.tensors_table = t
        # Adam groups inside the packed MLP: 'sigma' = trunk + heads, 'color' = colour MLP (meta_ngp.py:446-469)
        self.color_start = t[2 * (sigma_depth + 1)][0]

    def device_index(self, device):
        key = str(device)
        if key not in self._dev:
            self._dev[key] = self.index.to(device)
        return self._dev[key]

    def pack(self, tensors):
        return _PackFn.apply(self, *tensors)

    def pack_raw(self, tensors):
        if _PACK_SCOPE["depth"]:
            key = (id(self), tuple((t.data_ptr(), t._version) for t in tensors))
            hit = _PACK_SCOPE["cache"].get(key)
            if hit is not None:
                return hit.view(-1)  # a fresh tensor object: each autograd use gets its own node
        flat = torch.cat([x.detach().reshape(-1).to(torch.float32) for x in tensors])
        out = torch.zeros(self.total, dtype=torch.float32, device=flat.device).index_copy(
            0, self.device_index(flat.device), flat)
        if _PACK_SCOPE["depth"]:
            _PACK_SCOPE["cache"][key] = out
        return out

    def flat_grad_target(self, tensors):
        """(flat gradient buffer, element positions) when every tensor's .grad is a contiguous view of ONE
        FlatAdam gradient buffer (tag ``_nerf_flat_grad``), else None."""
        gs = [t.grad for t in tensors]
        if not all(getattr(t, "_nerf_flat_grad", False) and g is not None and g.is_contiguous() for t, g in
                   zip(tensors, gs)):
            return None
        base = gs[0]._base
        if base is None or any(g._base is not base for g in gs):
            return None
        key = ("flat", base.data_ptr(), tuple(g.data_ptr() for g in gs))
        if key not in self._dev:
            b0 = base.data_ptr()
            self._dev[key] = torch.cat([torch.arange((g.data_ptr() - b0) // 4, (g.data_ptr() - b0) // 4 + g.numel())
                                        for g in gs]).to(base.device)
        return base, self._dev[key]


_PACK_SCOPE = {"depth": 0, "cache": {}}


@contextlib.contextmanager
def pack_scope():
    """Within one render call the experts' parameters cannot change, so the visibility pass (sigma only) and the
    forward pack each expert's MLP once (keyed on the tensors' storage and version counters); the cache is dropped
    when the outermost scope exits."""
    _PACK_SCOPE["depth"] += 1
    try:
        yield
    finally:
        _PACK_SCOPE["depth"] -= 1
        if _PACK_SCOPE["depth"] == 0:
            _PACK_SCOPE["cache"].clear()


class _PackFn(torch.autograd.Function):
    """Packs a MetaNGP's named tensors into the fused kernel's layout.  Backward: the packed gradient goes back to
    the tensors' layout with ONE gather; for FlatAdam-owned parameters it is added straight into the flat gradient
    buffer (one index_add instead of one autograd accumulation launch per tensor), returning no per-tensor grads."""

    @staticmethod
    def forward(ctx, layout, *tensors):
        ctx.layout = layout
        ctx.tensors = tensors
        return layout.pack_raw(tensors)

    @staticmethod
    @once_differentiable
    def backward(ctx, d_w):
        layout, tensors = ctx.layout, ctx.tensors
        need_all = all(ctx.needs_input_grad[1:])
        g = d_w.index_select(0, layout.device_index(d_w.device))
        tgt = layout.flat_grad_target(tensors) if need_all else None
        if tgt is not None:
            base, pos = tgt
            base.index_add_(0, pos, g)
            return (None,) * (1 + len(tensors))
        out, o = [], 0
        for t, need_i in zip(tensors, ctx.needs_input_grad[1:]):
            k = t.numel()
            out.append(g[o:o + k].view_as(t) if need_i else None)
            o += k
        return (None, *out)


class _NgpFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x_d, table, w_packed, model):
        x_d = x_d.contiguous().float()
        M = x_d.shape[0]
        fused = None
        if M:
            h = TIMING.start("fwd_enc", M)
            fused = ngp_fwd_enc(model.net_struct, model.xyz_encoder.grid, table.detach(), w_packed, x_d,
                                model._aabb_host, model._eps)
            TIMING.stop(h)
        if fused is not None:
            out, enc = fused
        else:
            h = TIMING.start("hash_fwd", M)
            enc = hash_encode(model.xyz_encoder.grid, table.detach(), x_d, model._aabb_host, model._eps)
            TIMING.stop(h)
            h = TIMING.start("mlp_fwd", M)
            out = ngp_fwd(model.net_struct, w_packed, enc, x_d) if M else x_d.new_empty((0, 4))
            TIMING.stop(h)
        ctx.model = model
        ctx.rows = table.shape[0]
        ctx.table = table  # the parameter itself: FlatAdam-owned tables take their gradient in place
        ctx.save_for_backward(x_d, enc, w_packed)
        return out

    @staticmethod
    @once_differentiable
    def backward(ctx, g):
        x_d, enc, w_packed = ctx.saved_tensors
        model = ctx.model
        if ctx.needs_input_grad[0]:
            raise NotImplementedError("InstantNGP (HIP): no gradient w.r.t. sample positions x_d")
        g = g.contiguous().float()
        if x_d.shape[0] == 0:
            return None, torch.zeros_like(model.xyz_encoder.hash_table), torch.zeros_like(w_packed), None
        d_table = None
        if ctx.needs_input_grad[1]:
            # MLP backward + table scatter in one launch (production shape): straight into a FlatAdam-owned
            # table's .grad view, else into a fresh zero gradient
            t = ctx.table
            flat = getattr(t, "_nerf_flat_grad", False) and t.grad is not None
            tgt = t.grad if flat else torch.zeros((ctx.rows, model.xyz_encoder.grid.features_per_level),
                                                  dtype=torch.float32, device=x_d.device)
            h = TIMING.start("bwd_hash", x_d.shape[0])
            d_w = ngp_bwd_hash(model.net_struct, model.xyz_encoder.grid, w_packed, enc, x_d, g, tgt,
                               model._aabb_host, model._eps)
            TIMING.stop(h)
            if d_w is not None:
                if flat:
                    _table_grad_ready(t)
                return None, (None if flat else tgt), d_w, None
        h = TIMING.start("mlp_bwd", x_d.shape[0])
        d_enc, d_w = ngp_bwd(model.net_struct, w_packed, enc, x_d, g)
        TIMING.stop(h)
        if ctx.needs_input_grad[1]:
            h = TIMING.start("hash_bwd", x_d.shape[0])
            t = ctx.table
            if getattr(t, "_nerf_flat_grad", False) and t.grad is not None:
                # the table's .grad is a view of FlatAdam's flat buffer: scatter-add straight into it instead of
                # a zeroed (rows, F) tensor that autograd would then add (saves ~4 x 134 MB of HBM per expert)
                hash_encode_bwd(model.xyz_encoder.grid, x_d, d_enc, ctx.rows, model._aabb_host, model._eps,
                                d_table=t.grad)
                _table_grad_ready(t)
            else:
                d_table = hash_encode_bwd(model.xyz_encoder.grid, x_d, d_enc, ctx.rows, model._aabb_host,
                                          model._eps)
            TIMING.stop(h)
        return None, d_table, d_w, None


def _table_grad_ready(t):
    """A FlatAdam-owned table's gradient is complete in stream order (its only writer, this expert's backward, has
    been enqueued): FlatAdam's bucketed exchange starts that table's all-reduce now (optim.FlatAdam)."""
    cb = getattr(t, "_nerf_grad_ready", None)
    if cb is not None:
        cb(t)


class _Block(nn.Module):
    def __init__(self, i, o):
        super().__init__()
        self.linear = nn.Linear(i, o)


class InstantNGP(nn.Module):
    """MetaNGP (models/inr/meta_ngp.py:15-255) on the HIP kernels; same constructor and parameter names."""

    def __init__(self, *, occ_conf: Optional[Dict] = None, scene_box=None, hidden: int = 64, sigma_depth: int = 2,
                 color_hidden: int = 64, geo_feat_dim: int = 15, color_depth: int = 3, use_sigmoid_rgb: bool = True,
                 hash_enc_conf: Optional[Dict] = None, dir_encoding: str = "spherical", **kwargs) -> None:
        super().__init__()
        occ_conf = occ_conf or {}
        aabb = scene_box.aabb if hasattr(scene_box, "aabb") else scene_box
        aabb = torch.as_tensor(aabb, dtype=torch.float32).reshape(2, 3).cpu()
        if not bool((aabb[0] < aabb[1]).all()):
            raise ValueError(f"AABB invalid: min>=max ({aabb[0]} vs {aabb[1]})")
        self.register_buffer("aabb_extent", aabb[1] - aabb[0])
        self.register_buffer("enc_eps", torch.tensor(1e-6, dtype=torch.float32), persistent=False)
        self._aabb_host = [float(v) for v in aabb.reshape(-1).tolist()]
        self._eps = float(torch.tensor(1e-6, dtype=torch.float32))
        self.scene_box = scene_box
        self.use_occ = bool(occ_conf.get("use_occ", False))
        self.occ_ready = False
        self.use_bg_nerf = False
        self.dim_out = 4
        self.geo_feat_dim = int(geo_feat_dim)
        self.use_sigmoid_rgb = bool(use_sigmoid_rgb)
        hc = hash_enc_conf or {}
        self.xyz_encoder = HashGridEncoder(levels=hc.get("levels", 4), min_res=hc.get("min_res", 16),
                                           max_res=hc.get("max_res", 4096),
                                           log2_hashmap_size=hc.get("log2_hashmap_size", 19),
                                           features_per_level=hc.get("features_per_level", 2),
                                           interpolation=hc.get("interpolation", "Linear"))
        in_xyz = self.xyz_encoder.out_dim
        dir_encoding = dir_encoding.lower()
        if dir_encoding == "spherical":
            self.dir_encoder = SHEncoder(levels=4)
            dir_dim, dir_mode = 16, 0
        elif dir_encoding == "frequency":
            from .encodings import FrequencyEncoder
            self.dir_encoder = FrequencyEncoder(in_dim=3, pe_dim=4, include_input=True, use_pi=False)
            dir_dim, dir_mode = 27, 1
        else:
            raise ValueError(f"Unsupported dir_encoding: {dir_encoding}")
        self.sigma_depth = max(int(sigma_depth), 0)
        self.color_depth = max(int(color_depth), 0)
        trunk, last = [], in_xyz
        for _ in range(self.sigma_depth):
            trunk.append(_Block(last, hidden))
            last = hidden
        self.sigma_trunk = nn.ModuleList(trunk)
        self.sigma_head = nn.Linear(last, 1)
        with torch.no_grad():
            self.sigma_head.bias.fill_(-1.0)
        self.geo_head = nn.Linear(last, self.geo_feat_dim)
        cm, last = [], self.geo_feat_dim + dir_dim
        for _ in range(self.color_depth):
            cm.append(_Block(last, color_hidden))
            last = color_hidden
        cm.append(nn.Linear(last, 3))
        self.color_mlp = nn.ModuleList(cm)
        net = NerfNgpNet()
        net.in_dim, net.hidden, net.sigma_depth = in_xyz, int(hidden), self.sigma_depth
        net.geo_feat_dim, net.color_hidden, net.color_depth = self.geo_feat_dim, int(color_hidden), self.color_depth
        net.dir_encoding, net.sh_levels, net.use_sigmoid_rgb = dir_mode, 4, int(self.use_sigmoid_rgb)
        self.net_struct = net
        shapes = OrderedDict((n, tuple(p.shape)) for n, p in self.named_parameters() if not n.startswith("xyz_encoder."))
        self.layout = NgpLayout(net, shapes, self.sigma_depth, self.color_depth)
        self._subdict_cache = {}
        if self.use_occ:  # meta_ngp.py:108-145
            from .occupancy import OccGridEstimator
            diag = float((aabb[1] - aabb[0]).norm())
            rss = occ_conf.get("render_step_size")
            self.render_step_size = float(rss) if rss is not None else diag / 1000.0
            self.occ_thre = float(occ_conf.get("occ_thre", 1e-2))
            self.alpha_thre = float(occ_conf.get("alpha_thre", 1e-2))
            self.cone_angle = float(occ_conf.get("cone_angle", 1.0 / 256.0))
            self.near_plane = float(occ_conf.get("near_plane", 0.05))
            self.far_plane = float(occ_conf.get("far_plane", 1e3))
            self.occ_update_interval = int(occ_conf.get("update_interval", 16))
            self.occ_warmup_steps = int(occ_conf.get("warmup_steps", 256))
            self.occ_cosine_anneal = bool(occ_conf.get("cosine_anneal", True))
            self.occ_alpha_thre_start = float(occ_conf.get("alpha_thre_start", 0.0))
            self.occ_alpha_thre_end = float(occ_conf.get("alpha_thre_end", self.alpha_thre))
            self.occ_ema_decay = float(occ_conf.get("ema_decay", 0.95))
            self.occ_resolution = int(occ_conf.get("resolution", 128))
            self.occ_levels = int(occ_conf.get("levels", 4))
            self.register_buffer("scene_aabb", torch.cat([aabb[0], aabb[1]]).flatten())
            self.occ_grid = OccGridEstimator(roi_aabb=self.scene_aabb, resolution=self.occ_resolution,
                                             levels=self.occ_levels)
            self.occ_frozen = bool(occ_conf.get("occ_frozen", False))
            self.occ_ready = bool(occ_conf.get("occ_ready", False))
            self.num_occ_updates = 0
            self.occ_premarked = False

    # ---- density / occupancy (meta_ngp.py:203-239, 245-258, 318-443)
    def density(self, x: torch.Tensor, params=None, return_feats: bool = False):
        """sigma (...,1) at world points (the fused kernel evaluates the whole network; directions are unused
        by sigma).  return_feats is not supported (geo features stay on chip)."""
        if return_feats:
            raise NotImplementedError("density(return_feats=True): geo features are not materialised")
        shp = x.shape[:-1]
        xf = x.reshape(-1, 3).float()
        w = self.packed(params)
        if not (torch.is_grad_enabled() and (w.requires_grad or self.xyz_encoder.hash_table.requires_grad)):
            # no graph needed (visibility filter, occupancy update): sigma branch only
            with torch.no_grad():
                h = TIMING.start("density_enc", xf.shape[0])
                sig = ngp_density_enc(self.net_struct, self.xyz_encoder.grid, self.xyz_encoder.hash_table.detach(),
                                      w.detach(), xf, self._aabb_host, self._eps)
                TIMING.stop(h)
                if sig is not None:
                    return sig.view(*shp, 1)
                h = TIMING.start("hash_fwd", xf.shape[0])
                enc = hash_encode(self.xyz_encoder.grid, self.xyz_encoder.hash_table.detach(), xf, self._aabb_host,
                                  self._eps)
                TIMING.stop(h)
                h = TIMING.start("mlp_density", xf.shape[0])
                sig = ngp_density(self.net_struct, w.detach(), enc)
                TIMING.stop(h)
                return sig.view(*shp, 1)
        xd = torch.cat([xf, torch.zeros_like(xf)], -1)
        xd[:, 5] = 1.0
        return self.forward(xd, params=params)[:, 3:4].view(*shp, 1)

    def _anneal_alpha_thre(self, step: int) -> None:
        if step < self.occ_warmup_steps:
            t = step / max(1, self.occ_warmup_steps - 1)
            if self.occ_cosine_anneal:
                c = 0.5 * (1 - math.cos(math.pi * t))
                self.alpha_thre = (1 - c) * self.occ_alpha_thre_start + c * self.occ_alpha_thre_end
            else:
                self.alpha_thre = (1 - t) * self.occ_alpha_thre_start + t * self.occ_alpha_thre_end
        else:
            self.alpha_thre = self.occ_alpha_thre_end

    @torch.no_grad()
    def maybe_update_occ_grid(self, step: int, params=None) -> None:
        if not (self.training and self.use_occ and not self.occ_frozen):
            return
        self.occ_ready = step >= self.occ_warmup_steps
        self._anneal_alpha_thre(step)
        self.occ_grid.update_every_n_steps(
            step=step, occ_eval_fn=lambda x: self.density(x, params=params).squeeze(-1) * self.render_step_size,
            occ_thre=self.occ_thre, ema_decay=self.occ_ema_decay, warmup_steps=self.occ_warmup_steps,
            n=self.occ_update_interval)
        self.num_occ_updates += 1

    @torch.no_grad()
    def premark_invisible_cells_from(self, K, c2w_rdf, width: int, height: int, near_plane: float = 0.05) -> None:
        """premark_invisible_cells (meta_ngp.py:318-347) from stacked intrinsics (n,3,3) and RDF c2w (n,3,4)."""
        if not self.use_occ or self.occ_premarked:
            return
        self.occ_grid.mark_invisible_cells(K=K, c2w=c2w_rdf, width=width, height=height, near_plane=near_plane)
        self.occ_premarked = True

    @torch.no_grad()
    def occupancy_marching_packed(self, rays, *, params=None, render_step_size=None, alpha_thre=None,
                                  cone_angle=None):
        """occupancy_marching (meta_ngp.py:384-443) -> (ray_idx int32, t0, t1, offsets int32 (N+1))."""
        if getattr(self, "occ_grid", None) is None:
            raise RuntimeError("MetaNGP: occ_grid missing")
        rays = rays.contiguous().float()
        o, d = rays[:, :3], rays[:, 3:6]
        sigma_fn = None
        if self.training:
            def sigma_fn(t_starts, t_ends, ray_indices):
                mids = 0.5 * (t_starts + t_ends)
                x = o[ray_indices] + d[ray_indices] * mids[:, None]
                return self.density(x, params=params).squeeze(-1)
        return self.occ_grid.sampling_packed(
            o, d, sigma_fn=sigma_fn, near_plane=self.near_plane, far_plane=self.far_plane, t_min=rays[:, 6],
            t_max=rays[:, 7], render_step_size=self.render_step_size if render_step_size is None else render_step_size,
            stratified=self.training, cone_angle=self.cone_angle if cone_angle is None else cone_angle,
            alpha_thre=self.alpha_thre if alpha_thre is None else alpha_thre)

    def occupancy_marching(self, rays, *, params=None, render_step_size=None, alpha_thre=None, cone_angle=None):
        ri, t0, t1, _ = self.occupancy_marching_packed(rays, params=params, render_step_size=render_step_size,
                                                       alpha_thre=alpha_thre, cone_angle=cone_angle)
        return ri.long(), t0, t1

    # ---- MetaModule surface (models/metamodule/metamodule.py:20-69): the hash table is not a meta parameter
    def meta_named_parameters(self, prefix: str = "", recurse: bool = True):
        for n, p in self.named_parameters(prefix=prefix, recurse=recurse):
            if not n[len(prefix):].lstrip(".").startswith("xyz_encoder."):
                yield n, p

    def meta_parameters(self, recurse: bool = True):
        for _, p in self.meta_named_parameters(recurse=recurse):
            yield p

    get_subdict = VanillaNeRF.get_subdict

    def get_param_groups(self):
        """models/inr/meta_ngp.py:446-469."""
        return {"encoding": {"params": list(self.xyz_encoder.parameters())},
                "sigma": {"params": list(self.sigma_trunk.parameters()) + list(self.sigma_head.parameters())
                          + list(self.geo_head.parameters())},
                "color": {"params": list(self.color_mlp.parameters())}}

    def tensors(self, params=None):
        own = dict(self.named_parameters())
        if params is None:
            return [own[n] for n in self.layout.names]
        return [params.get(n, own[n]) for n in self.layout.names]

    def packed(self, params=None):
        return self.layout.pack(self.tensors(params))

    def _fused_ok(self) -> bool:
        """Whether the one-launch kernels (fwd_enc, density_enc, bwd_hash) cover this expert's shape: each entry point
        answers NERF_E_UNSUPPORTED before it looks at its buffers, so a zero-row call probes it."""
        v = self.__dict__.get("_fused_ok_v")
        if v is None:
            L, g, n = lib(), self.xyz_encoder.grid, self.net_struct
            od = g.levels * g.features_per_level
            rc1 = L.nerf_ngp_fwd_enc(_addr(n), _addr(g), None, None, None, 0, None, 0.0, None, od, None, stream())
            rc2 = L.nerf_ngp_density_enc(_addr(n), _addr(g), None, None, None, 3, 0, None, 0.0, None, stream())
            rc3 = L.nerf_ngp_bwd_hash(_addr(n), _addr(g), None, None, od, None, 0, None, None, 0.0, None,
                                      ctypes.c_void_p(16), 1, None, 0, stream())
            v = self.__dict__["_fused_ok_v"] = (rc1 == 0 and rc2 == 0 and rc3 == 0)
        return v

    def load_reference_state(self, state: Dict[str, torch.Tensor]):
        with torch.no_grad():
            for n, p in self.named_parameters():
                p.copy_(state[n].to(p.device, p.dtype))
        return self

    def forward(self, x_d: torch.Tensor, params=None) -> torch.Tensor:
        assert x_d.shape[-1] == 6, f"Expected (...,6) [xyz,dir], got {x_d.shape}"
        shp = x_d.shape[:-1]
        from . import second_order as so
        so.refuse("the Instant-NGP expert")
        out = _NgpFn.apply(x_d.reshape(-1, 6), self.xyz_encoder.hash_table, self.packed(params), self)
        return out.view(*shp, 4)


MetaNGP = InstantNGP
