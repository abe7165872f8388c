"""The vanilla NeRF expert: ``expert(x_d (M,6), params=None) -> (M,4)`` on the HIP MLP kernels.

Mirrors ``MetaNeRF(encoding_dir="frequency")`` (models/inr/meta_vanilla.py:13-154) — 8x256 ReLU trunk,
skip cat([h, enc]) at layer 4, sigma via trunc_exp, 15-d geo feature, colour MLP 42->128->3 with
sigmoid — behind the container contract of models/inr/meta_ngp.py:226-241, with the MetaModule
fast-weights surface (models/metamodule/metamodule.py:20-69): parameter names, ``meta_named_parameters``,
``get_subdict`` and a ``params=`` dict that replaces any subset of the module's own tensors.

Gradients flow by PyTorch autograd to whatever tensors were used (module parameters or explicit
fast-weight tensors), through ``VanillaMLPFn`` whose weights are explicit inputs (packed once per call
into the kernel layout by differentiable torch indexing).  Double backward (MAML second order,
pipelines/offline_stage/meta_core.py:57) runs the torch composite of second_order.py inside ``second_order()``.
"""
from __future__ import annotations

import math
import re
import warnings
from collections import OrderedDict
from typing import Dict, Optional

import torch
import torch.nn as nn
from torch.autograd.function import once_differentiable

from . import kernels as K
from ._lib import lib

PARAM_SHAPES = OrderedDict()
for _i in range(8):
    PARAM_SHAPES[f"trunk.{_i}.linear.weight"] = (256, 63 if _i == 0 else (319 if _i == 4 else 256))
    PARAM_SHAPES[f"trunk.{_i}.linear.bias"] = (256,)
PARAM_SHAPES["sigma_head.weight"] = (1, 256)
PARAM_SHAPES["sigma_head.bias"] = (1,)
PARAM_SHAPES["geo_head.weight"] = (15, 256)
PARAM_SHAPES["geo_head.bias"] = (15,)
PARAM_SHAPES["color_mlp.layer0.linear.weight"] = (128, 42)
PARAM_SHAPES["color_mlp.layer0.linear.bias"] = (128,)
PARAM_SHAPES["color_mlp.color_out.weight"] = (3, 128)
PARAM_SHAPES["color_mlp.color_out.bias"] = (3,)
NUM_PARAMS = sum(math.prod(s) for s in PARAM_SHAPES.values())  # 503,059


class PackedLayout:
    """Packed kernel layout (include/nerf_amd.h nerf_mlp_layout) and the index map from the
    reference-named tensors into it."""

    _inst = None

    def __init__(self):
        import ctypes
        tbl = (ctypes.c_int64 * (22 * 4))()
        self.total = int(lib().nerf_mlp_layout(tbl))
        self.table = [(tbl[4 * t], tbl[4 * t + 1], tbl[4 * t + 2], tbl[4 * t + 3]) for t in range(22)]
        # (tensor index, row offset) per reference parameter
        place = {}
        for i in range(8):
            place[f"trunk.{i}.linear.weight"] = (2 * i, 0)
            place[f"trunk.{i}.linear.bias"] = (2 * i + 1, 0)
        place["sigma_head.weight"] = (16, 0)
        place["geo_head.weight"] = (16, 1)
        place["sigma_head.bias"] = (17, 0)
        place["geo_head.bias"] = (17, 1)
        place["color_mlp.layer0.linear.weight"] = (18, 0)
        place["color_mlp.layer0.linear.bias"] = (19, 0)
        place["color_mlp.color_out.weight"] = (20, 0)
        place["color_mlp.color_out.bias"] = (21, 0)
        self.index = OrderedDict()  # name -> LongTensor (numel,) of packed positions (CPU)
        for name, shp in PARAM_SHAPES.items():
            t, r0 = place[name]
            off, rows, cols, _ = self.table[t]
            r = shp[0]
            c = shp[1] if len(shp) == 2 else 1
            rr = torch.arange(r0, r0 + r).view(-1, 1)
            cc = torch.arange(c).view(1, -1)
            self.index[name] = (off + rr * cols + cc).reshape(-1)
        self.all_index = torch.cat(list(self.index.values()))
        self._dev = {}
        # Adam param groups inside one packed net: 'sigma' = trunk + heads, 'color' = colour MLP
        self.color_start = self.table[18][0]

    @classmethod
    def get(cls):
        if cls._inst is None:
            cls._inst = PackedLayout()
        return cls._inst

    def index_on(self, device):
        key = str(device)
        if key not in self._dev:
            self._dev[key] = self.all_index.to(device)
        return self._dev[key]

    def pack(self, tensors):
        """Differentiable: list of tensors in PARAM_SHAPES order -> packed (total,) fp32."""
        flat = torch.cat([t.reshape(-1).to(torch.float32) for t in tensors])
        dev = flat.device
        return torch.zeros(self.total, dtype=torch.float32, device=dev).index_copy(0, self.index_on(dev), flat)

    def unpack(self, packed):
        """packed (total,) -> OrderedDict of reference-shaped views/copies."""
        out = OrderedDict()
        for name, shp in PARAM_SHAPES.items():
            out[name] = packed[self.index[name].to(packed.device)].view(shp)
        return out


def amp_precision() -> str:
    """The MLP precision the caller's autocast region asks for (else "fp32").  The reference trains under
    ``torch.cuda.amp.autocast(dtype=torch.float16)`` + GradScaler (pipelines/online_stage/runtime_adapt.py:290-310,
    configs/train.json "use_amp": true): autocast(float16) runs the fp16 build of the fused MLP kernels ("fp16": fp16
    operands, the reference's rounding points — include/nerf_amd.h nerf_mlp_fwd_f16), autocast(bfloat16) the bf16
    build ("bf16", configs[2]).  Compositing, loss and sampling stay fp32 either way: the reference's volume_render
    receives the expert's fp32 outputs (the heads add fp32 biases, metamodule.py:153-155)."""
    if torch.is_autocast_enabled("cuda"):
        dt = torch.get_autocast_dtype("cuda")
        if dt == torch.float16:
            return "fp16"
        if dt == torch.bfloat16:
            return "bf16"
    return "fp32"


class VanillaMLPFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x_d, w_packed, precision="fp32"):
        x_d = x_d.contiguous().float()
        M = x_d.shape[0]
        ws = K.mlp_workspace(M, True, x_d.device, precision)
        out = K.mlp_fwd(w_packed, x_d, ws, training=True, precision=precision)
        ctx.save_for_backward(w_packed)
        ctx.ws = ws
        ctx.M = M
        ctx.precision = precision
        return out

    @staticmethod
    @once_differentiable
    def backward(ctx, g):
        (w_packed,) = ctx.saved_tensors
        g = g.contiguous().float()
        d_w = K.mlp_bwd(w_packed, ctx.M, g, ctx.ws, precision=ctx.precision)
        ctx.ws = None
        if ctx.needs_input_grad[0]:
            raise NotImplementedError("gradient w.r.t. sample positions x_d is not supported by the HIP MLP")
        return None, d_w, None


def mlp_forward(x_d, w_packed, precision: Optional[str] = None):
    """x_d (M,6) -> (M,4) with a packed weight tensor; inference path when no grad is needed.  precision None
    follows the caller's autocast region (amp_precision)."""
    precision = amp_precision() if precision is None else precision
    if torch.is_grad_enabled() and w_packed.requires_grad:
        return VanillaMLPFn.apply(x_d, w_packed, precision)
    x_d = x_d.contiguous().float()
    ws = K.mlp_workspace(x_d.shape[0], False, x_d.device, precision)
    return K.mlp_fwd(w_packed.detach(), x_d, ws, training=False, precision=precision)


class _Block(nn.Module):
    def __init__(self, i, o):
        super().__init__()
        self.linear = nn.Linear(i, o)


class _ColorMLP(nn.Module):
    def __init__(self):
        super().__init__()
        self.layer0 = _Block(42, 128)
        self.color_out = nn.Linear(128, 3)


class VanillaNeRF(nn.Module):
    """HIP-backed equivalent of MetaNeRF(encoding_dir="frequency") with the (M,6)->(M,4) contract."""

    def __init__(self):
        super().__init__()
        self.trunk = nn.ModuleList([_Block(PARAM_SHAPES[f"trunk.{i}.linear.weight"][1], 256) for i in range(8)])
        self.sigma_head = nn.Linear(256, 1)
        self.geo_head = nn.Linear(256, 15)
        self.color_mlp = _ColorMLP()
        self.use_occ = False
        self.use_bg_nerf = False
        self.dim_out = 4
        self._subdict_cache = {}

    # ---- MetaModule surface (models/metamodule/metamodule.py:20-69)
    def meta_named_parameters(self, prefix: str = "", recurse: bool = True):
        for n, p in self.named_parameters(prefix=prefix, recurse=recurse):
            yield n, p

    def meta_parameters(self, recurse: bool = True):
        for _, p in self.meta_named_parameters(recurse=recurse):
            yield p

    def get_subdict(self, params: Optional[Dict[str, torch.Tensor]], key: Optional[str] = None):
        if params is None:
            return None
        names = tuple(params.keys())
        ck = (key, names)
        if ck not in self._subdict_cache:
            if key is None:
                self._subdict_cache[ck] = list(names)
            else:
                rx = re.compile(rf"^{re.escape(key)}\.(.+)")
                self._subdict_cache[ck] = [rx.sub(r"\1", k) for k in names if rx.match(k)]
        sub = self._subdict_cache[ck]
        if not sub:
            warnings.warn(f"Module `{type(self).__name__}` has no parameter for submodule `{key}` in `params`. "
                          "Using default parameters.", stacklevel=2)
            return None
        return OrderedDict((n, params[f"{key}.{n}"]) for n in sub)

    def get_param_groups(self):
        """models/inr/meta_ngp.py:446-469 grouping (no encoder parameters for the frequency PE)."""
        sig = [p for n, p in self.named_parameters() if not n.startswith("color_mlp")]
        col = [p for n, p in self.named_parameters() if n.startswith("color_mlp")]
        return {"sigma": {"params": sig}, "color": {"params": col}}

    # ---- packing
    def tensors(self, params=None):
        own = dict(self.named_parameters())
        if params is None:
            return [own[n] for n in PARAM_SHAPES]
        return [params.get(n, own[n]) for n in PARAM_SHAPES]

    def packed(self, params=None):
        return PackedLayout.get().pack(self.tensors(params))

    def load_reference_state(self, state: Dict[str, torch.Tensor]):
        with torch.no_grad():
            for n, p in self.named_parameters():
                p.copy_(state[n].to(p.device, p.dtype))
        return self

    def forward(self, x_d: torch.Tensor, params=None) -> torch.Tensor:
        assert x_d.shape[-1] == 6, f"Expected (...,6) [xyz,dir], got {tuple(x_d.shape)}"
        shp = x_d.shape[:-1]
        from . import second_order as so
        if so.active():  # create_graph=True inner loop: the differentiable torch composite (second_order.py)
            return so.vanilla_forward(self, x_d.reshape(-1, 6), params).view(*shp, 4)
        out = mlp_forward(x_d.reshape(-1, 6), self.packed(params))
        return out.view(*shp, 4)


class HierarchicalNeRF(nn.Module):
    """A coarse + fine pair behind ONE model object, for callers that only pass ``model`` (the reference's
    compute_mse_loss(P, model, data), nerfs/losses.py:10-32): ``model(x_d, params)`` is the coarse expert and
    ``render_rays(model, ..., n_importance=k)`` renders the fine pass with ``model.fine``.  Parameter groups
    merge both nets ('sigma' / 'color', models/inr/meta_ngp.py:446-469)."""

    def __init__(self, coarse: Optional[VanillaNeRF] = None, fine: Optional[VanillaNeRF] = None):
        super().__init__()
        self.coarse = coarse if coarse is not None else VanillaNeRF()
        self.fine = fine if fine is not None else VanillaNeRF()
        self.use_occ = False
        self.use_bg_nerf = False
        self.dim_out = 4

    def get_param_groups(self):
        gc, gf = self.coarse.get_param_groups(), self.fine.get_param_groups()
        return {k: {"params": gc[k]["params"] + gf[k]["params"]} for k in gc}

    def forward(self, x_d: torch.Tensor, params=None) -> torch.Tensor:
        return self.coarse(x_d, params=params)


_EXP_MAX = {torch.float16: 11.089866488, torch.bfloat16: 88.722839111, torch.float32: 88.722839111,
            torch.float64: 709.782712893}


class _TruncExpFn(torch.autograd.Function):
    """models/trunc_exp.py:43-57 (used only for volume_render(raw_sigma=True); the MLP applies it in-kernel)."""

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


def trunc_exp_torch(x):
    return _TruncExpFn.apply(x)
