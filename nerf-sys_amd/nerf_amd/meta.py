"""Meta-learning inner / outer updates over the HIP render path — mirrors
adaptive_nerf/pipelines/offline_stage/meta_core.py.

``task_adapt`` runs the reference's inner loop (:14-68): fast weights, the loss of ``compute_loss`` through
``render_rays`` (every op a HIP kernel behind autograd), ``torch.autograd.grad`` over the fast tensors, and
the functional SGD step ``w - inner_lr * g`` for all fast tensors in ONE launch (nerf_sgd_multi). The step is
an autograd Function whose backward is the identity to ``w`` (``g`` is a constant: first order), so the outer
``loss.backward()`` of FOMAML reaches the module parameters exactly as through the reference's tensor ops.
Second-order MAML (``create_graph=True``) needs double backward through the HIP kernels and is refused
(SURVEY.md §8b gradient contract).

``reptile_meta_update`` (:145-176) is one nerf_reptile_update call over every matching tensor; ``meta_update`` /
``maml_meta_update`` / ``clip_all_grads`` / ``extract_module_params`` / ``snapshot_params`` follow :74-205.
"""
from __future__ import annotations

import ctypes
from collections import OrderedDict
from typing import List, Optional

import torch

from ._lib import check, lib, ptr, stream
from .losses import compute_fim_loss, compute_mse_loss


def _ptr_array(tensors):
    return (ctypes.c_void_p * max(len(tensors), 1))(*[None if t is None else t.data_ptr() for t in tensors])


class _SgdStep(torch.autograd.Function):
    """out_i = w_i - lr * g_i (nerf_sgd_multi); d out_i / d w_i = I, g_i constant (first order)."""

    @staticmethod
    def forward(ctx, lr, grads, *ws):
        outs = [torch.empty_like(w) for w in ws]
        n = len(ws)
        for s in range(0, n, 64):
            w_c, g_c, o_c = ws[s:s + 64], grads[s:s + 64], outs[s:s + 64]
            numel = (ctypes.c_int64 * len(w_c))(*[w.numel() for w in w_c])
            check(lib().nerf_sgd_multi(len(w_c), _ptr_array(w_c), _ptr_array(g_c), _ptr_array(o_c), numel,
                                       float(lr), stream()), "nerf_sgd_multi")
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gouts):
        return (None, None) + tuple(gouts)


def sgd_update(fast: "OrderedDict[str, torch.Tensor]", grads, inner_lr: float) -> "OrderedDict[str, torch.Tensor]":
    """meta_core.py:61-64: {n: w if g is None else w - inner_lr * g} in one HIP launch per 64 tensors."""
    names = list(fast.keys())
    ws, gs = [], []
    for n, g in zip(names, grads):
        w = fast[n]
        if w.dtype != torch.float32 or not w.is_cuda or not w.is_contiguous():
            raise ValueError(f"fast weight {n!r} must be a contiguous fp32 device tensor")
        if g is not None:
            g = g.to(w.dtype).contiguous()
            if g.shape != w.shape:
                raise ValueError(f"gradient of {n!r} has shape {tuple(g.shape)}, expected {tuple(w.shape)}")
        ws.append(w)
        gs.append(g)
    outs = _SgdStep.apply(float(inner_lr), gs, *ws)
    return OrderedDict((n, w if g is None else o) for n, w, g, o in zip(names, ws, gs, outs))


def compute_loss(P, model, data, params=None, active_module=None, **kwargs):
    """nerfs/losses.py:154-166 dispatcher.  P.fim routes to compute_fim_loss, which (as in the reference, where no
    module defines ``fisher_store``) returns the per-ray MSE mean of one render; kwargs go to it only, as there."""
    if getattr(P, "fim", False):
        return compute_fim_loss(P, model, data, params, active_module, **kwargs)
    return compute_mse_loss(P, model, data, params, active_module)


def extract_module_params(submodule, copy: bool = True) -> "OrderedDict[str, torch.Tensor]":
    """meta_core.py:196-205: reptile copies detached leaves; (fo)MAML injects the module parameters."""
    if copy:
        return OrderedDict((n, p.detach().clone().requires_grad_(True)) for n, p in submodule.meta_named_parameters())
    return OrderedDict((n, p) for n, p in submodule.meta_named_parameters())


def snapshot_params(model):
    """meta_core.py:208-210."""
    return {n: p.detach().clone() for n, p in model.meta_named_parameters()}


def task_adapt(P, model, support, inner_lr, iterations, active_module: Optional[int] = None):
    """meta_core.py:14-68. Returns (fast OrderedDict, [detached loss per iteration]).

    P.algo "fomaml" / "reptile" (first order) run on the HIP kernels.  Like the reference (:30-38) each inner forward
    then runs under autocast(fp16) when P.use_amp (default True) and a GPU is present: vanilla experts take the fp16
    build of their MLP kernels (vanilla.amp_precision); the Instant-NGP kernels stay fp32.  Any other algo ("maml")
    is second order (create_graph=True, no autocast, :28-29): the inner losses run the torch composite of
    second_order.py and the update is the reference's tensor expression, so the graph reaches the outer backward."""
    from .second_order import second_order
    algo = str(getattr(P, "algo", "")).lower()
    first_order = algo in ("fomaml", "reptile")
    base = model.submodules[active_module] if active_module is not None else model
    fast = extract_module_params(base, copy=(algo == "reptile"))
    losses = []
    amp_enabled = bool(getattr(P, "use_amp", True)) and torch.cuda.is_available() and first_order
    for _ in range(int(iterations)):
        if first_order:
            with torch.autocast("cuda", dtype=torch.float16, enabled=amp_enabled):
                loss = compute_loss(P, model, support, params=fast, active_module=active_module)
            grads = torch.autograd.grad(loss, tuple(fast.values()), create_graph=False, allow_unused=True)
            fast = sgd_update(fast, grads, inner_lr)
        else:
            with second_order():
                loss = compute_loss(P, model, support, params=fast, active_module=active_module)
                grads = torch.autograd.grad(loss, tuple(fast.values()), create_graph=True, allow_unused=True)
            fast = OrderedDict((n, w if g is None else (w - inner_lr * g.to(w.dtype)))
                               for (n, w), g in zip(fast.items(), grads))
        losses.append(loss.detach())
    return fast, losses


@torch.no_grad()
def reptile_meta_update(P, model, fast_list: List["OrderedDict[str, torch.Tensor]"]):
    """meta_core.py:145-176: theta += P.lr * mean_f(fast_f - theta) per tensor named in the fast lists, skipped
    when the mean delta has a non-finite element or is all zero. Returns the updated names."""
    if len(fast_list) == 0:
        raise ValueError("Reptile update called with empty fast_list")
    names, thetas, fasts = [], [], []
    for name, p in model.meta_named_parameters():
        f = [fl.get(name) for fl in fast_list]
        if any(v is None for v in f):
            # the reference accumulates each fast list's own keys; a name missing from some list still gets
            # the sum of the others over n = len(fast_list) — kept identical by treating it as theta there
            if all(v is None for v in f):
                continue
            f = [p if v is None else v for v in f]
        if p.dtype != torch.float32 or not p.is_cuda or not p.is_contiguous():
            raise ValueError(f"parameter {name!r} must be a contiguous fp32 device tensor")
        names.append(name)
        thetas.append(p)
        fasts.append([v.detach().to(p.dtype).contiguous() for v in f])
    if not names:
        return []
    n_fast = len(fast_list)
    flags = torch.empty(2 * len(names), dtype=torch.int32, device=thetas[0].device)
    flat_fast = [v for fl in fasts for v in fl]
    numel = (ctypes.c_int64 * len(names))(*[t.numel() for t in thetas])
    check(lib().nerf_reptile_update(len(names), _ptr_array(thetas), _ptr_array(flat_fast), n_fast, numel,
                                    float(P.lr), ptr(flags), flags.numel() * 4, stream()), "nerf_reptile_update")
    f = flags.view(-1, 2).cpu()
    updated = [n for n, (bad, nz) in zip(names, f.tolist()) if not bad and nz]
    print("Reptile meta-update: updated %d parameter tensors: %s"
          % (len(updated), ", ".join(updated) if updated else "<none>"))
    return updated


def clip_all_grads(optimizer, grad_clip=1.0):
    """meta_core.py:182-192."""
    if grad_clip is None:
        return
    params = [p for g in optimizer.param_groups for p in g["params"] if p.grad is not None]
    if params:
        torch.nn.utils.clip_grad_norm_(params, grad_clip)


def maml_meta_update(optimizer, loss_out, grad_clip=1.0):
    """meta_core.py:119-142 (fp32 branch): backward of the query loss, clip, step; a non-finite loss is skipped.
    A FlatAdam optimiser clips inside its own step (nerf_grad_sqnorm + nerf_adam)."""
    if not torch.isfinite(loss_out):
        print(f"[WARN] Skipping meta-update: non-finite loss_out={loss_out.item()}")
        return
    if hasattr(optimizer, "param_groups"):
        optimizer.zero_grad(set_to_none=True)
        loss_out.backward()
        clip_all_grads(optimizer, grad_clip)
    else:
        optimizer.zero_grad()
        loss_out.backward()
    optimizer.step()


def meta_update(P, model, optimizer, loss_out=None, scheduler=None, fast_list=None):
    """meta_core.py:74-116 (without the debug prints)."""
    algo = P.algo.lower()
    if algo in ("maml", "fomaml"):
        maml_meta_update(optimizer, loss_out, grad_clip=getattr(P, "grad_clip", 1.0))
    elif algo == "reptile":
        reptile_meta_update(P, model, fast_list=fast_list)
    else:
        raise ValueError(f"Unsupported algo {algo!r}")
    if scheduler is not None:
        scheduler.step()
