"""The reference's Mixture-of-Experts container on the HIP kernels.

Mirrors ``MetaContainer`` (models/inr/meta_container.py:21-503): the same constructor, parameter names
(``submodules.{k}.*``, ``bg_mlp.0.*``, ``bg_mlp.2.*``), ``forward(x, params=None, active_module=None)``
with soft (boundary_margin > 1) or hard routing, ``background_color(d)``, ``get_param_groups()`` and the
fast-weights surface.  Compute per call:

  nerf_moe_route (weights (M,K)) -> nerf_moe_dispatch (expert-major row lists; ONE host read of the K+1
  offsets, as the reference's .nonzero() syncs) -> per expert: nerf_gather_rows -> expert forward (HIP
  expert kernels) -> nerf_moe_combine in expert order (the reference's index_add_ summation order);
  backward: nerf_moe_combine_bwd per expert (routing is no-grad in the reference too).
  background_color: nerf_bg_mlp_fwd / nerf_bg_mlp_bwd (SH + 2-layer MLP fused, one thread per ray).

Occupancy rendering of the whole container (``render_container_occ``, SURVEY §8f rows 2+3) runs on the HIP
kernels: per-expert AABB prefilter + marching, per-ray segment union on the GPU, soft sigma/rgb blend, one
packed integration.  Not mirrored: the ``density`` / ``color`` split queries; ``bg_encoding="fourier"``
fails in the reference's constructor (FrequencyEncoder without in_dim) and raises here.
"""
from __future__ import annotations

import ctypes
from collections import OrderedDict
from typing import Dict, List, Optional

import torch
import torch.nn as nn
from torch.autograd.function import once_differentiable

from ._lib import check, lib, ptr, stream
from .ngp import InstantNGP, SHEncoder
from .vanilla import VanillaNeRF


def build_expert(nerf_variant: str, **nerf_kwargs) -> nn.Module:
    """meta_container.py:14-18."""
    if nerf_variant == "instant":
        return InstantNGP(**nerf_kwargs)
    return VanillaNeRF()


# ------------------------------------------------------------------ kernel wrappers

def moe_route(x, centroids_host, boundary_margin, cluster_2d):
    M, K = x.shape[0], len(centroids_host) // 3
    W = torch.empty((M, K), dtype=torch.float32, device=x.device)
    c = (ctypes.c_float * len(centroids_host))(*centroids_host)
    check(lib().nerf_moe_route(ptr(x), x.stride(0), M, c, K, int(cluster_2d), float(boundary_margin), ptr(W),
                               stream()), "nerf_moe_route")
    return W


def moe_dispatch(W, eps=0.0, host_offsets=True):
    """-> (offsets (K+1): host list, or the device int32 tensor when host_offsets is False; idx (device int32,
    expert-major))."""
    M, K = W.shape
    offs = torch.empty(K + 1, dtype=torch.int32, device=W.device)
    idx = torch.empty(max(M * K, 1), dtype=torch.int32, device=W.device)
    wsb = int(lib().nerf_moe_dispatch_workspace_bytes(M, K))
    ws = torch.empty(wsb, dtype=torch.uint8, device=W.device)
    check(lib().nerf_moe_dispatch(ptr(W), M, K, float(eps), ptr(offs), ptr(idx), ptr(ws), wsb, stream()),
          "nerf_moe_dispatch")
    return (offs.cpu().tolist() if host_offsets else offs), idx


def gather_rows(src, idx, cols=None):
    n = idx.numel()
    cols = cols or src.shape[1]
    dst = torch.empty((n, cols), dtype=torch.float32, device=src.device)
    check(lib().nerf_gather_rows(ptr(src), src.stride(0), ptr(idx), n, cols, ptr(dst), cols, stream()),
          "nerf_gather_rows")
    return dst


class _MixFn(torch.autograd.Function):
    """out = sum_k (in expert order) index_add(sel_k, y_k * W[sel_k, k])."""

    @staticmethod
    def forward(ctx, W, N, C, sels, ks, *ys):
        out = torch.zeros((N, C), dtype=torch.float32, device=W.device)
        K = W.shape[1]
        for k, sel, y in zip(ks, sels, ys):
            y = y.contiguous().float()
            check(lib().nerf_moe_combine(ptr(y), y.shape[0], C, ptr(sel), ptr(W), K, k, ptr(out), stream()),
                  "nerf_moe_combine")
        ctx.save_for_backward(W, *sels)
        ctx.ks, ctx.C = ks, C
        return out

    @staticmethod
    @once_differentiable
    def backward(ctx, g):
        W, *sels = ctx.saved_tensors
        g = g.contiguous().float()
        K = W.shape[1]
        grads = []
        for k, sel in zip(ctx.ks, sels):
            dy = torch.empty((sel.numel(), ctx.C), dtype=torch.float32, device=g.device)
            check(lib().nerf_moe_combine_bwd(ptr(g), sel.numel(), ctx.C, ptr(sel), ptr(W), K, k, ptr(dy), stream()),
                  "nerf_moe_combine_bwd")
            grads.append(dy)
        return (None, None, None, None, None, *grads)


class _BgFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, d, w_packed, H):
        d = d.contiguous().float()
        N = d.shape[0]
        out = torch.empty((N, 3), dtype=torch.float32, device=d.device)
        check(lib().nerf_bg_mlp_fwd(ptr(d), d.stride(0), N, ptr(w_packed), H, ptr(out), stream()), "nerf_bg_mlp_fwd")
        ctx.save_for_backward(d, w_packed)
        ctx.H = H
        return out

    @staticmethod
    @once_differentiable
    def backward(ctx, g):
        d, w = ctx.saved_tensors
        N = d.shape[0]
        dw = torch.empty_like(w)
        wsb = int(lib().nerf_bg_mlp_workspace_bytes(N, ctx.H))
        ws = torch.empty(wsb, dtype=torch.uint8, device=d.device)
        check(lib().nerf_bg_mlp_bwd(ptr(d), d.stride(0), N, ptr(w), ctx.H, ptr(g.contiguous().float()), ptr(dw),
                                    ptr(ws), wsb, stream()), "nerf_bg_mlp_bwd")
        if ctx.needs_input_grad[0]:
            raise NotImplementedError("background MLP (HIP): no gradient w.r.t. directions")
        return None, dw, None


class _BlendFn(torch.autograd.Function):
    """sigma / rgb of the routed experts blended BEFORE integration (ray_rendering.py:441-471)."""

    @staticmethod
    def forward(ctx, W, M, sels, ks, *ys):
        s = torch.zeros(M, dtype=torch.float32, device=W.device)
        c = torch.zeros((M, 3), dtype=torch.float32, device=W.device)
        K = W.shape[1]
        ys = [y.contiguous().float() for y in ys]
        for k, sel, y in zip(ks, sels, ys):
            check(lib().nerf_moe_blend(ptr(y), y.shape[0], ptr(sel), ptr(W), K, k, ptr(s), ptr(c), stream()),
                  "nerf_moe_blend")
        rs = torch.empty((M, 4), dtype=torch.float32, device=W.device)
        check(lib().nerf_moe_blend_finish(ptr(s), ptr(c), M, ptr(rs), stream()), "nerf_moe_blend_finish")
        ctx.save_for_backward(W, s, rs, *sels, *ys)
        ctx.ks, ctx.n = ks, len(ks)
        return rs

    @staticmethod
    @once_differentiable
    def backward(ctx, g):
        W, s, rs, *rest = ctx.saved_tensors
        sels, ys = rest[:ctx.n], rest[ctx.n:]
        g = g.contiguous().float()
        K = W.shape[1]
        grads = []
        for k, sel, y in zip(ctx.ks, sels, ys):
            dy = torch.empty_like(y)
            check(lib().nerf_moe_blend_bwd(ptr(y), y.shape[0], ptr(sel), ptr(W), K, k, ptr(s), ptr(rs), ptr(g), ptr(dy),
                                           stream()), "nerf_moe_blend_bwd")
            grads.append(dy)
        return (None, None, None, None, *grads)


MARCH_STAGE_CAP = 512  # staged segments per (expert, ray) pair: K*N*512*8 B (67 MB at 4 x 4096 pairs)


def vis_thresholds(model, alpha_thre=None):
    """Per-expert visibility thresholds min(alpha_thre, mean occupancy) (nerfacc sampling's alpha_thre clamp,
    ray_rendering.py:397-422) in ONE persistent device tensor, recomputed in place only when a grid or alpha_thre
    changed (the grids update every 16 steps) — not with 4 reductions and a host->device copy every step.  In place,
    so a captured train-step graph (graph_step.py) reads the current values after an eager occupancy update."""
    subs = list(model.submodules)
    athr = [ex.alpha_thre for ex in subs] if alpha_thre is None else list(alpha_thre)
    key = (tuple((ex.occ_grid.gen, ex.occ_grid.occs._version, ex.occ_grid.occs.data_ptr()) for ex in subs),
           tuple(athr))
    st = model.__dict__.setdefault("_vis_thr_state", {"key": None, "buf": None})
    if st["key"] != key:
        dev = subs[0].occ_grid.occs.device
        occ_mean = torch.stack([ex.occ_grid.occs.mean() for ex in subs]).float()
        val = torch.minimum(occ_mean, torch.tensor(athr, dtype=torch.float32, device=dev))
        if st["buf"] is None or st["buf"].shape != val.shape:
            st["buf"] = val.contiguous()
        else:
            st["buf"].copy_(val)
        st["key"] = key
    return st["buf"]


def _march_experts(model, rays, sub_params, render_step_size, alpha_thre, cone_angle, before_sync=None):
    """Every expert's occupancy marching (MetaNGP.occupancy_marching, meta_ngp.py:384-443, on the rays that hit its
    box, ray_rendering.py:397-422) in ONE launch pair: count -> scan -> ONE host read of the K+1 expert boundaries
    -> write.  In training, the visibility filter (nerfacc render_visibility_from_density with alpha_thre =
    min(alpha_thre, mean occupancy) per expert) runs over all experts' segments at once and compacts in place of
    the per-expert host reads: the compacted offsets are pos[offsets], sizes stay on the device.
    Returns (ray_idx, t0, t1, offsets (K*N+1)) or (None,)*4 when no expert produced a sample."""
    from . import kernels as K_
    from .occupancy import exclusive_scan
    subs = list(model.submodules)
    K, N, dev = len(subs), rays.shape[0], rays.device
    ex0 = subs[0]
    for ex in subs[1:]:
        if (ex.near_plane, ex.far_plane) != (ex0.near_plane, ex0.far_plane):
            raise ValueError("experts with different near/far planes")
    cone = [ex.cone_angle if cone_angle is None else cone_angle for ex in subs]
    if len(set(cone)) != 1:
        raise ValueError("experts with different cone angles")
    grids = (type(ex0.occ_grid.grid) * K)(*[ex.occ_grid.grid for ex in subs])
    bins = (ctypes.c_void_p * K)(*[ex.occ_grid.binaries.data_ptr() for ex in subs])
    boxes = (ctypes.c_float * (6 * K))(*[float(v) for ex in subs for v in ex._aabb_host])
    steps = (ctypes.c_float * K)(*[float(ex.render_step_size if render_step_size is None else render_step_size)
                                   for ex in subs])
    training = bool(ex0.training)
    seed = int(torch.randint(0, 2 ** 62, (1,)).item())
    L = lib()
    counts = torch.empty(K * N, dtype=torch.int32, device=dev)
    args = (grids, bins, boxes, steps, K, ptr(rays), N, float(ex0.near_plane), float(ex0.far_plane), float(cone[0]),
            int(training), ctypes.c_uint64(seed), 8192)
    # staged march: the count pass keeps each (expert, ray) pair's first MARCH_STAGE_CAP segments, so the write pass
    # is a copy (pairs with more segments are marched again)
    stage = torch.empty(K * N * MARCH_STAGE_CAP * 2, dtype=torch.float32, device=dev)
    check(L.nerf_occ_march_multi_staged(*args, ptr(counts), ptr(stage), MARCH_STAGE_CAP, None, None, None, None,
                                        stream()), "nerf_occ_march_multi_staged(count)")
    offs = exclusive_scan(counts)
    if before_sync is not None:
        before_sync()
    bounds = offs[::N].cpu().tolist()                  # the one host read: K+1 expert boundaries
    M = bounds[-1]
    if getattr(model, "device_sized", False) and "_dev_sizes" not in model.__dict__:
        model.__dict__["_dev_sizes"] = _DevSizes(M)    # seeds the device-sized path's capacity (next calls)
    if M == 0:
        return None, None, None, None
    ri = torch.empty(M, dtype=torch.int32, device=dev)
    t0 = torch.empty(M, dtype=torch.float32, device=dev)
    t1 = torch.empty(M, dtype=torch.float32, device=dev)
    check(L.nerf_occ_march_multi_staged(*args, ptr(counts), ptr(stage), MARCH_STAGE_CAP, ptr(offs), ptr(ri), ptr(t0),
                                        ptr(t1), stream()), "nerf_occ_march_multi_staged(emit)")
    del stage
    athr = [ex.alpha_thre if alpha_thre is None else alpha_thre for ex in subs]
    if training:
        # visibility (nerfacc sampling with sigma_fn, early_stop_eps 1e-4): sigma of every sample from its expert
        with torch.no_grad():
            xd = K_.packed_points(rays, ri, t0, t1)
            sig = torch.empty(M, dtype=torch.float32, device=dev)
            for k, ex in enumerate(subs):
                a, b = bounds[k], bounds[k + 1]
                if b > a:
                    sig[a:b] = ex.density(xd[a:b, :3], params=sub_params[k]).view(-1)
            # per-expert thresholds min(alpha_thre, mean occupancy): recomputed only when a grid or alpha_thre
            # changed (the grids update every 16 steps), not with 4 reductions and a host->device copy every step
            thr = vis_thresholds(model, athr)
            keep = torch.empty(M, dtype=torch.int32, device=dev)
            check(L.nerf_packed_visibility_groups(ptr(t0), ptr(t1), ptr(sig), ptr(offs), K * N, N, 1e-4,
                                                  float(max(athr)), ptr(thr), ptr(keep), stream()),
                  "nerf_packed_visibility_groups")
            pos = exclusive_scan(keep)
            ri2 = torch.empty(M, dtype=torch.int32, device=dev)
            t02 = torch.empty(M, dtype=torch.float32, device=dev)
            t12 = torch.empty(M, dtype=torch.float32, device=dev)
            check(L.nerf_packed_compact(ptr(keep), ptr(pos), M, ptr(ri), ptr(t0), ptr(t1), ptr(ri2), ptr(t02),
                                        ptr(t12), None, stream()), "nerf_packed_compact")
            offs = pos[offs.long()].contiguous()          # segment j now starts at pos[offsets[j]]
            ri, t0, t1 = ri2, t02, t12
    return ri, t0, t1, offs


# ------------------------------------------------------------------ device-sized (sync-free) container step
#
# The host-sized path above reads two sizes per call on the host (the marched sample count, and the merged count with
# the K+1 expert offsets), and every launch after such a read waits for the host to catch up: ~0.9 ms of idle GPU per
# train step.  The device-sized path sizes every buffer for a CAPACITY of samples and every kernel
# after the march reads its row count from device memory (nerf_*_n / _rng entry points), so the host never waits and
# runs ahead of the GPU.  The capacity follows the sample counts of earlier steps: each call copies its counts to
# pinned host memory without waiting, a later call reads them once they have landed (event query, no sync) and keeps
# the capacity at >= 2x the largest count seen (power of two).  A step whose march would exceed the capacity keeps
# the first CAP samples (per (expert, ray) pair in order) and is counted in model.dev_overflows (never observed in
# the bench: the counts move by a few percent per step).  The first call of a model runs the host-sized path, which
# seeds the capacity.  Outputs equal the host-sized path's (tests/test_gpu_moe.py): the same kernels on the same
# rows; only the experts' weight-gradient slab partition (a persistent grid sized by the capacity) moves the fp32
# summation order of the MLP weight gradients.


class _DevSizes:
    """Capacity bookkeeping of one model's device-sized renders (see above)."""

    def __init__(self, first_total, min_cap=1 << 16):
        self.min_cap = int(min_cap)
        self.max_seen = int(first_total)
        self.cap = self._cap_for(self.max_seen)
        self.pending = []          # (event, pinned int32 march total, capacity it ran with)
        self.overflows = 0
        self.calls = 0
        # frozen (a captured train-step graph, graph_step.py): the capacity no longer moves and no host copy / event
        # is issued; the largest march total is kept on the device (max_dev) and read after the replays
        self.frozen = False
        self.max_dev = None

    def freeze(self, cap=None, device=None):
        """Fix the capacity (default: the current one) for graph capture."""
        self.poll()
        if cap is not None:
            self.cap = max(int(cap), self.cap)
        self.frozen = True
        self.max_dev = torch.zeros(1, dtype=torch.int32, device=device)

    def frozen_report(self):
        """(largest march total seen by the frozen steps, whether it exceeded the capacity) — one host read."""
        mx = int(self.max_dev.item()) if self.max_dev is not None else 0
        return mx, mx > self.cap

    def _cap_for(self, total):
        return max(self.min_cap, 1 << (max(1, 2 * int(total)) - 1).bit_length())

    def poll(self):
        if self.frozen:
            return self.cap
        keep = []
        for ev, host, cap in self.pending:
            if ev.query():
                tot = int(host[0])
                if tot > cap:
                    self.overflows += 1
                self.max_seen = max(self.max_seen, tot)
            else:
                keep.append((ev, host, cap))
        self.pending = keep[-8:]
        self.cap = max(self.cap, self._cap_for(self.max_seen))
        return self.cap

    def record(self, total_dev, cap):
        if self.frozen:
            torch.maximum(self.max_dev, total_dev.view(1), out=self.max_dev)
            self.calls += 1
            return
        host = torch.empty(1, dtype=torch.int32, pin_memory=True)
        host.copy_(total_dev.view(1), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.pending.append((ev, host, cap))
        self.calls += 1


def _ngp_dev_ok(model):
    """The device-sized path covers containers of production-shape Instant-NGP experts (the fused kernels)."""
    from .ngp import InstantNGP
    return all(isinstance(sub, InstantNGP) and sub._fused_ok() for sub in model.submodules)


class _NgpFnDev(torch.autograd.Function):
    """The expert's forward / backward on its gathered rows 0 .. rng[1] - rng[0] - 1 of capacity-sized buffers."""

    @staticmethod
    def forward(ctx, x_d, rng, table, w_packed, sub):
        from .ngp import TIMING, _addr
        cap = x_d.shape[0]
        g = sub.xyz_encoder.grid
        od = g.levels * g.features_per_level
        enc = torch.empty((cap, od), dtype=torch.float32, device=x_d.device)
        out = torch.empty((cap, 4), dtype=torch.float32, device=x_d.device)
        ab = (ctypes.c_float * 6)(*sub._aabb_host)
        h = TIMING.start("fwd_enc", rng)
        check(lib().nerf_ngp_fwd_enc_n(_addr(sub.net_struct), _addr(g), ptr(table.detach()), ptr(w_packed), ptr(x_d),
                                       cap, ptr(rng), ab, float(sub._eps), ptr(enc), od, ptr(out), stream()),
              "nerf_ngp_fwd_enc_n")
        TIMING.stop(h)
        ctx.sub, ctx.table = sub, table
        ctx.save_for_backward(x_d, enc, w_packed, rng)
        return out

    @staticmethod
    @once_differentiable
    def backward(ctx, gr):
        from .ngp import TIMING, _addr, _table_grad_ready, ngp_workspace
        x_d, enc, w_packed, rng = ctx.saved_tensors
        sub, t = ctx.sub, ctx.table
        cap = x_d.shape[0]
        gr = gr.contiguous().float()
        flat = getattr(t, "_nerf_flat_grad", False) and t.grad is not None
        tgt = t.grad if flat else torch.zeros_like(t)
        d_w = torch.empty_like(w_packed)
        ws = ngp_workspace(sub.net_struct, cap, x_d.device)
        ab = (ctypes.c_float * 6)(*sub._aabb_host)
        h = TIMING.start("bwd_hash", rng)
        check(lib().nerf_ngp_bwd_hash_n(_addr(sub.net_struct), _addr(sub.xyz_encoder.grid), ptr(w_packed), ptr(enc),
                                        enc.stride(0), ptr(x_d), cap, ptr(rng), ptr(gr), ab, float(sub._eps),
                                        ptr(tgt), ptr(d_w), 0, ptr(ws), ws.numel(), stream()), "nerf_ngp_bwd_hash_n")
        TIMING.stop(h)
        if flat:
            _table_grad_ready(t)
        return None, None, (None if flat else tgt), d_w, None


class _BlendFnDev(torch.autograd.Function):
    """_BlendFn over capacity-sized rows: expert k's rows pair with idx entries rngs[k][0] .., the mix is finished for
    the first *m_dev rows."""

    @staticmethod
    def forward(ctx, W, m_dev, idx, rngs, ks, *ys):
        cap, K = W.shape
        s = torch.zeros(cap, dtype=torch.float32, device=W.device)
        c = torch.zeros((cap, 3), dtype=torch.float32, device=W.device)
        L = lib()
        for k, rng, y in zip(ks, rngs, ys):
            check(L.nerf_moe_blend_rng(ptr(y), cap, ptr(idx), ptr(rng), ptr(W), K, k, ptr(s), ptr(c), stream()),
                  "nerf_moe_blend_rng")
        rs = torch.empty((cap, 4), dtype=torch.float32, device=W.device)
        check(L.nerf_moe_blend_finish_n(ptr(s), ptr(c), cap, ptr(m_dev), ptr(rs), stream()), "nerf_moe_blend_finish_n")
        ctx.save_for_backward(W, s, rs, idx, *rngs, *ys)
        ctx.ks, ctx.n = ks, len(ks)
        return rs

    @staticmethod
    @once_differentiable
    def backward(ctx, g):
        W, s, rs, idx, *rest = ctx.saved_tensors
        rngs, ys = rest[:ctx.n], rest[ctx.n:]
        g = g.contiguous().float()
        cap, K = W.shape
        grads = []
        for k, rng, y in zip(ctx.ks, rngs, ys):
            dy = torch.empty_like(y)
            check(lib().nerf_moe_blend_bwd_rng(ptr(y), cap, ptr(idx), ptr(rng), ptr(W), K, k, ptr(s), ptr(rs), ptr(g),
                                               ptr(dy), stream()), "nerf_moe_blend_bwd_rng")
            grads.append(dy)
        return (None, None, None, None, None, *grads)


def _march_experts_dev(model, rays, sub_params, render_step_size, alpha_thre, cone_angle, sizes):
    """_march_experts without the host read: the packed arrays hold sizes.cap samples; the offsets are clamped to it.
    Returns (ray_idx, t0, t1, offsets (K*N+1), cap)."""
    from .ngp import TIMING, _addr
    from .occupancy import exclusive_scan
    subs = list(model.submodules)
    K, N, dev = len(subs), rays.shape[0], rays.device
    ex0 = subs[0]
    for ex in subs[1:]:
        if (ex.near_plane, ex.far_plane) != (ex0.near_plane, ex0.far_plane):
            raise ValueError("experts with different near/far planes")
    cone = [ex.cone_angle if cone_angle is None else cone_angle for ex in subs]
    if len(set(cone)) != 1:
        raise ValueError("experts with different cone angles")
    grids = (type(ex0.occ_grid.grid) * K)(*[ex.occ_grid.grid for ex in subs])
    bins = (ctypes.c_void_p * K)(*[ex.occ_grid.binaries.data_ptr() for ex in subs])
    boxes = (ctypes.c_float * (6 * K))(*[float(v) for ex in subs for v in ex._aabb_host])
    steps = (ctypes.c_float * K)(*[float(ex.render_step_size if render_step_size is None else render_step_size)
                                   for ex in subs])
    training = bool(ex0.training)
    L = lib()
    # model.step_seed = (int64 device step counter, base, mul): the jitter seed base + step * mul is read on the
    # device (a captured train-step graph replays with the counter it advances); else one host draw per call
    ss = getattr(model, "step_seed", None)
    seed = int(ss[1]) if ss is not None else int(torch.randint(0, 2 ** 62, (1,)).item())
    counts = torch.empty(K * N, dtype=torch.int32, device=dev)
    args = (grids, bins, boxes, steps, K, ptr(rays), N, float(ex0.near_plane), float(ex0.far_plane), float(cone[0]),
            int(training), ctypes.c_uint64(seed), 8192)
    stage = torch.empty(K * N * MARCH_STAGE_CAP * 2, dtype=torch.float32, device=dev)

    def march(*rest):
        if ss is None:
            return L.nerf_occ_march_multi_staged(*args, *rest, stream())
        return L.nerf_occ_march_multi_staged_dseed(*args, *rest, ptr(ss[0]), ctypes.c_uint64(int(ss[2])), stream())

    check(march(ptr(counts), ptr(stage), MARCH_STAGE_CAP, None, None, None, None), "nerf_occ_march_multi_staged(count)")
    offs = exclusive_scan(counts)
    cap = sizes.poll()
    sizes.record(offs[K * N:], cap)
    offs.clamp_(max=cap)
    ri = torch.empty(cap, dtype=torch.int32, device=dev)
    t0 = torch.empty(cap, dtype=torch.float32, device=dev)
    t1 = torch.empty(cap, dtype=torch.float32, device=dev)
    check(march(ptr(counts), ptr(stage), MARCH_STAGE_CAP, ptr(offs), ptr(ri), ptr(t0), ptr(t1)),
          "nerf_occ_march_multi_staged(emit)")
    del stage
    athr = [ex.alpha_thre if alpha_thre is None else alpha_thre for ex in subs]
    if training:
        with torch.no_grad():
            m_dev = offs[K * N:]
            xd = torch.empty((cap, 6), dtype=torch.float32, device=dev)
            check(L.nerf_packed_points_n(ptr(rays), ptr(ri), ptr(t0), ptr(t1), cap, ptr(m_dev), ptr(xd), stream()),
                  "nerf_packed_points_n")
            sig = torch.empty(cap, dtype=torch.float32, device=dev)
            bounds = offs[::N].contiguous()            # K+1 expert boundaries, on the device
            for k, ex in enumerate(subs):
                w = ex.packed(sub_params[k]).detach()
                ab = (ctypes.c_float * 6)(*ex._aabb_host)
                h = TIMING.start("density_enc", bounds[k:k + 2])
                check(L.nerf_ngp_density_enc_rng(_addr(ex.net_struct), _addr(ex.xyz_encoder.grid),
                                                 ptr(ex.xyz_encoder.hash_table.detach()), ptr(w), ptr(xd), 6, cap,
                                                 ptr(bounds[k:k + 2]), ab, float(ex._eps), ptr(sig), stream()),
                      "nerf_ngp_density_enc_rng")
                TIMING.stop(h)
            thr = vis_thresholds(model, athr)
            keep = torch.zeros(cap, dtype=torch.int32, device=dev)
            check(L.nerf_packed_visibility_groups(ptr(t0), ptr(t1), ptr(sig), ptr(offs), K * N, N, 1e-4,
                                                  float(max(athr)), ptr(thr), ptr(keep), stream()),
                  "nerf_packed_visibility_groups")
            pos = exclusive_scan(keep)
            ri2 = torch.empty(cap, dtype=torch.int32, device=dev)
            t02 = torch.empty(cap, dtype=torch.float32, device=dev)
            t12 = torch.empty(cap, dtype=torch.float32, device=dev)
            check(L.nerf_packed_compact(ptr(keep), ptr(pos), cap, ptr(ri), ptr(t0), ptr(t1), ptr(ri2), ptr(t02),
                                        ptr(t12), None, stream()), "nerf_packed_compact")
            offs = pos[offs.long()].contiguous()
            ri, t0, t1 = ri2, t02, t12
    return ri, t0, t1, offs, cap


def _render_container_occ_dev(model, rays, params, bg_color_default, render_step_size, alpha_thre, cone_angle):
    from .ray_rendering import _get_bg_rgb
    from .occupancy import exclusive_scan, render_packed
    rays = rays.contiguous().float()
    N = rays.shape[0]
    dev = rays.device
    d = rays[:, 3:6]
    K = len(model.submodules)
    sub_params = ([model.get_subdict(params, f"submodules.{k}") for k in range(K)] if params is not None
                  else [None] * K)
    ws = [sub.packed(sub_params[k]) for k, sub in enumerate(model.submodules)]  # (cached by pack_scope)
    bg = _get_bg_rgb(model, d, params, rays, N, bg_color_default)
    sizes = model.__dict__["_dev_sizes"]
    ri_all, t0_all, t1_all, offs_all, cap = _march_experts_dev(model, rays, sub_params, render_step_size, alpha_thre,
                                                               cone_angle, sizes)
    t0s = (ctypes.c_void_p * K)(*([t0_all.data_ptr()] * K))
    t1s = (ctypes.c_void_p * K)(*([t1_all.data_ptr()] * K))
    ofs = (ctypes.c_void_p * K)(*[offs_all[k * N:].data_ptr() for k in range(K)])
    L = lib()
    cnt = torch.empty(max(N, 1), dtype=torch.int32, device=dev)
    check(L.nerf_segments_union(t0s, t1s, ofs, K, N, ptr(cnt), None, None, None, None, stream()),
          "nerf_segments_union(count)")
    moff = exclusive_scan(cnt[:N])
    cap2 = 2 * cap  # a ray's union of its experts' sorted boundary lists has < 2x their segments
    ri = torch.empty(cap2, dtype=torch.int32, device=dev)
    t0 = torch.empty(cap2, dtype=torch.float32, device=dev)
    t1 = torch.empty(cap2, dtype=torch.float32, device=dev)
    check(L.nerf_segments_union(t0s, t1s, ofs, K, N, None, ptr(moff), ptr(ri), ptr(t0), ptr(t1), stream()),
          "nerf_segments_union(write)")
    m_dev = moff[N:]
    xm = torch.empty((cap2, 6), dtype=torch.float32, device=dev)
    check(L.nerf_packed_points_n(ptr(rays), ptr(ri), ptr(t0), ptr(t1), cap2, ptr(m_dev), ptr(xm), stream()),
          "nerf_packed_points_n")
    with torch.no_grad():
        W = torch.empty((cap2, K), dtype=torch.float32, device=dev)
        c = (ctypes.c_float * len(model._cent_host))(*model._cent_host)
        check(L.nerf_moe_route_n(ptr(xm), 6, cap2, ptr(m_dev), c, K, int(model.cluster_2d),
                                 float(model.boundary_margin), ptr(W), stream()), "nerf_moe_route_n")
        offs_dev = torch.empty(K + 1, dtype=torch.int32, device=dev)
        idx = torch.empty(cap2 * K, dtype=torch.int32, device=dev)
        wsb = int(L.nerf_moe_dispatch_workspace_bytes(cap2, K))
        wsd = torch.empty(wsb, dtype=torch.uint8, device=dev)
        check(L.nerf_moe_dispatch_n(ptr(W), cap2, ptr(m_dev), K, 1e-8, ptr(offs_dev), ptr(idx), ptr(wsd), wsb,
                                    stream()), "nerf_moe_dispatch_n")
    ks, rngs, ys = [], [], []
    for k, sub in enumerate(model.submodules):
        rng = offs_dev[k:k + 2]
        xk = torch.empty((cap2, 6), dtype=torch.float32, device=dev)
        check(L.nerf_gather_rows_rng(ptr(xm), 6, ptr(idx), ptr(rng), cap2, 6, ptr(xk), 6, stream()),
              "nerf_gather_rows_rng")
        ys.append(_NgpFnDev.apply(xk, rng, sub.xyz_encoder.hash_table, ws[k], sub))
        ks.append(k)
        rngs.append(rng)
    rs = _BlendFnDev.apply(W, m_dev, idx, rngs, ks, *ys)
    rgb, depth, w, acc = render_packed(rs, t0, t1, moff, bg)
    return rgb, depth, w[:, None], acc


def render_container_occ(model, rays, *, params=None, bg_color_default="white", chunk=1_000_000,
                         render_step_size=None, alpha_thre=None, cone_angle=None):
    """render_rays_occ for the full container (nerfs/ray_rendering.py:384-481): per-expert AABB prefilter and
    occupancy marching, per-ray union of the experts' segments (GPU; a per-ray Python loop in the reference),
    routing at the segment midpoints, experts evaluated only where their weight > 1e-8, sigma / rgb blended
    before ONE packed integration.  Returns rgb (N,3), depth (N,), weights (M,1), acc (N,)."""
    from .ngp import pack_scope
    with pack_scope():
        if getattr(model, "device_sized", False) and _ngp_dev_ok(model) and "_dev_sizes" in model.__dict__:
            return _render_container_occ_dev(model, rays, params, bg_color_default, render_step_size, alpha_thre,
                                             cone_angle)
        return _render_container_occ(model, rays, params, bg_color_default, chunk, render_step_size, alpha_thre,
                                     cone_angle)


def _render_container_occ(model, rays, params, bg_color_default, chunk, render_step_size, alpha_thre, cone_angle):
    from . import kernels as K_
    from .occupancy import exclusive_scan, render_packed
    from .ray_rendering import _get_bg_rgb
    rays = rays.contiguous().float()
    N = rays.shape[0]
    dev = rays.device
    d = rays[:, 3:6]
    K = len(model.submodules)
    sub_params = ([model.get_subdict(params, f"submodules.{k}") for k in range(K)] if params is not None
                  else [None] * K)
    if K > 8:
        raise ValueError("occupancy marching / segment union support at most 8 experts")
    early = {}

    def before_sync():
        # host work that needs no marched sizes, issued while the march's count pass runs on the GPU (before the
        # host read of the packed sizes): each Instant-NGP expert's packed MLP (cached by pack_scope for this render;
        # other expert types do not cache, so packing them here would only be repeated in their forward) and the
        # background
        from .ngp import InstantNGP
        for k, sub in enumerate(model.submodules):
            if isinstance(sub, InstantNGP):
                sub.packed(sub_params[k])
        early["bg"] = _get_bg_rgb(model, d, params, rays, N, bg_color_default)

    ri_all, t0_all, t1_all, offs_all = _march_experts(model, rays, sub_params, render_step_size, alpha_thre,
                                                      cone_angle, before_sync=before_sync)
    if offs_all is None:
        acc = rays.new_zeros(N)
        return early["bg"], acc.clone(), torch.zeros(1, 1, device=dev, dtype=rays.dtype), acc
    # expert k's segments: offsets[k*N : (k+1)*N + 1] index the shared t0 / t1 arrays
    t0s = (ctypes.c_void_p * K)(*([t0_all.data_ptr()] * K))
    t1s = (ctypes.c_void_p * K)(*([t1_all.data_ptr()] * K))
    ofs = (ctypes.c_void_p * K)(*[offs_all[k * N:].data_ptr() for k in range(K)])
    L = lib()
    cnt = torch.empty(max(N, 1), dtype=torch.int32, device=dev)
    check(L.nerf_segments_union(t0s, t1s, ofs, K, N, ptr(cnt), None, None, None, None, stream()),
          "nerf_segments_union(count)")
    moff = exclusive_scan(cnt[:N])
    # the merged count stays on the device: the union, its points, the routing and the dispatch run over a
    # capacity (a ray's union of k sorted boundary lists has < 2x their segments), then ONE host read brings
    # the merged count and the K+1 expert offsets together
    cap = 2 * int(t0_all.numel())
    ri = torch.empty(cap, dtype=torch.int32, device=dev)
    t0 = torch.empty(cap, dtype=torch.float32, device=dev)
    t1 = torch.empty(cap, dtype=torch.float32, device=dev)
    check(L.nerf_segments_union(t0s, t1s, ofs, K, N, None, ptr(moff), ptr(ri), ptr(t0), ptr(t1), stream()),
          "nerf_segments_union(write)")
    m_dev = moff[N:]
    xm = torch.empty((cap, 6), dtype=torch.float32, device=dev)
    check(L.nerf_packed_points_n(ptr(rays), ptr(ri), ptr(t0), ptr(t1), cap, ptr(m_dev), ptr(xm), stream()),
          "nerf_packed_points_n")
    with torch.no_grad():
        W = torch.empty((cap, K), dtype=torch.float32, device=dev)
        c = (ctypes.c_float * len(model._cent_host))(*model._cent_host)
        check(L.nerf_moe_route_n(ptr(xm), 6, cap, ptr(m_dev), c, K, int(model.cluster_2d),
                                 float(model.boundary_margin), ptr(W), stream()), "nerf_moe_route_n")
        offs_dev, idx = moe_dispatch(W, 1e-8, host_offsets=False)
    host = torch.cat([m_dev, offs_dev]).cpu().tolist()
    M, offs = host[0], host[1:]
    if M == 0:
        acc = rays.new_zeros(N)
        return early["bg"], acc.clone(), torch.zeros(1, 1, device=dev, dtype=rays.dtype), acc
    ri, t0, t1, xm, W = ri[:M], t0[:M], t1[:M], xm[:M], W[:M]
    ks, sels, ys = [], [], []
    for k, sub in enumerate(model.submodules):
        n_k = offs[k + 1] - offs[k]
        if n_k == 0:
            continue
        sel = idx[offs[k]:offs[k + 1]]
        xk = gather_rows(xm, sel, 6)
        yk = torch.cat([sub(xk[s:s + chunk], params=sub_params[k]) for s in range(0, n_k, chunk)], 0)
        ks.append(k)
        sels.append(sel)
        ys.append(yk)
    rs = _BlendFn.apply(W, M, sels, ks, *ys)
    rgb, depth, w, acc = render_packed(rs, t0, t1, moff, early["bg"])
    return rgb, depth, w[:, None], acc


# ------------------------------------------------------------------ the container


class MetaContainer(nn.Module):
    def __init__(self, num_submodules: int, centroids: torch.Tensor, aabb: torch.Tensor,
                 nerf_variant: str = "instant", boundary_margin: float = 1.0, cluster_2d: bool = True,
                 joint_training: bool = False, use_bg_nerf: bool = True, bg_hidden: int = 32,
                 bg_encoding: str = "spherical", occ_conf: Optional[Dict] = None, **nerf_kwargs):
        super().__init__()
        assert num_submodules > 0
        assert centroids.ndim == 2 and centroids.size(0) == num_submodules
        assert boundary_margin >= 1.0
        if num_submodules > 32:
            raise ValueError("at most 32 experts (nerf_moe_route)")
        occ_conf = occ_conf or {}
        aabb = torch.as_tensor(aabb, dtype=torch.float32)
        self.register_buffer("scene_aabb_vec", torch.cat([aabb[0], aabb[1]], dim=0).float(), persistent=True)
        self.register_buffer("centroids", torch.as_tensor(centroids).to(torch.float32), persistent=True)
        self._cent_host = [float(v) for v in self.centroids[:, :3].reshape(-1).tolist()]
        self.use_occ = bool(occ_conf.get("use_occ", False))
        self.boundary_margin = float(boundary_margin)
        self.cluster_2d = bool(cluster_2d)
        self.joint_training = bool(joint_training)
        self._coord_idx = (1, 2) if self.cluster_2d else (0, 1, 2)
        self.nerf_variant = nerf_variant
        self.dim_out = 4
        boxes = nerf_kwargs.pop("expert_box_list")
        base = {**nerf_kwargs, "occ_conf": occ_conf}
        self.submodules = nn.ModuleList([build_expert(nerf_variant, **{**base, "scene_box": b}) for b in boxes])
        self.use_bg_nerf = bool(use_bg_nerf)
        if self.use_bg_nerf:
            if bg_encoding != "spherical":
                raise ValueError("bg_encoding='fourier' is broken in the reference (FrequencyEncoder without "
                                 "in_dim, meta_container.py:83-86); use 'spherical'")
            self.bg_dir_enc = SHEncoder(levels=4, implementation="tcnn")
            self.bg_hidden_dim = int(bg_hidden)
            if not 1 <= self.bg_hidden_dim <= 64:
                raise ValueError("bg_hidden must be in [1, 64] (nerf_bg_mlp_fwd)")
            self.bg_mlp = nn.Sequential(nn.Linear(self.bg_dir_enc.out_dim, self.bg_hidden_dim, bias=True), nn.ReLU(),
                                        nn.Linear(self.bg_hidden_dim, 3, bias=True), nn.Sigmoid())
        self._subdict_cache = {}

    # ---- routing (meta_container.py:97-134)
    def _routing(self, pts: torch.Tensor):
        assert pts.dim() == 2 and pts.shape[-1] == 3, "pts must be (N,3)"
        W = moe_route(pts.contiguous().float(), self._cent_host, self.boundary_margin, self.cluster_2d)
        if self.boundary_margin > 1.0:
            return W, None
        return None, W.argmax(dim=1)

    # ---- forward (meta_container.py:266-330)
    def forward(self, x: torch.Tensor, params: Optional[OrderedDict] = None,
                active_module: Optional[int] = None) -> torch.Tensor:
        assert x.dim() == 2 and x.shape[-1] >= 6, "x must be (N,D>=6)"
        K = len(self.submodules)
        sub_params = ([self.get_subdict(params, f"submodules.{k}") for k in range(K)] if params is not None
                      else [None] * K)
        if active_module is not None:
            return self.submodules[active_module](x, params=sub_params[active_module])
        from . import second_order as so
        so.refuse("a container's expert mix (pass active_module)")
        x = x.contiguous().float()
        N = x.shape[0]
        with torch.no_grad():
            W = moe_route(x, self._cent_host, self.boundary_margin, self.cluster_2d)
            offs, idx = moe_dispatch(W, 0.0)
        ks, sels, ys = [], [], []
        for k, sub in enumerate(self.submodules):
            n_k = offs[k + 1] - offs[k]
            if n_k == 0:
                if self.joint_training:
                    _ = sub(x[:0], params=sub_params[k])
                continue
            sel = idx[offs[k]:offs[k + 1]]
            yk = sub(gather_rows(x, sel, 6), params=sub_params[k])
            ks.append(k)
            sels.append(sel)
            ys.append(yk)
        if not ys:
            return x.new_zeros(N, self.dim_out)
        return _MixFn.apply(W, N, ys[0].shape[-1], sels, ks, *ys)

    # ---- background (meta_container.py:334-363)
    def _bg_packed(self):
        l0, l2 = self.bg_mlp[0], self.bg_mlp[2]
        return torch.cat([l0.weight.reshape(-1), l0.bias, l2.weight.reshape(-1), l2.bias]).float()

    def background_color(self, d: torch.Tensor) -> torch.Tensor:
        if not self.use_bg_nerf:
            raise RuntimeError("background_color called but use_bg_nerf=False")
        if d.dim() not in (2, 3):
            raise ValueError(f"background_color expects (N,3) or (B,N,3), got {tuple(d.shape)}")
        flat = d.reshape(-1, 3)
        rgb = _BgFn.apply(flat, self._bg_packed(), self.bg_hidden_dim)
        return rgb.view(*d.shape[:-1], 3)

    # ---- occupancy surface (not built)
    @property
    def occ_ready(self) -> bool:
        return all(getattr(sub, "occ_ready", False) for sub in self.submodules)

    def maybe_update_expert_occupancies(self, step: int, params=None) -> None:
        """meta_container.py:368-372."""
        for k, sub in enumerate(self.submodules):
            sub.maybe_update_occ_grid(step, self.get_subdict(params, f"submodules.{k}") if params is not None
                                      else None)

    def freeze_expert_occupancies(self, flag: bool) -> None:
        for sub in self.submodules:
            sub.occ_frozen = flag

    # ---- MetaModule surface
    def meta_named_parameters(self, prefix: str = "", recurse: bool = True):
        for k, sub in enumerate(self.submodules):
            for n, p in sub.meta_named_parameters(prefix=f"{prefix}submodules.{k}"):
                yield n, p

    def meta_parameters(self, recurse: bool = True):
        for _, p in self.meta_named_parameters(recurse=recurse):
            yield p

    get_subdict = VanillaNeRF.get_subdict

    def get_param_groups(self) -> Dict[str, Dict]:
        """meta_container.py:458-503."""
        enc: List = []
        sig: List = []
        col: List = []
        bg: List = []
        for sub in self.submodules:
            if hasattr(sub, "get_param_groups"):
                g = sub.get_param_groups()
                enc += list(g.get("encoding", {}).get("params", []))
                sig += list(g.get("sigma", {}).get("params", []))
                col += list(g.get("color", {}).get("params", []))
            else:
                sig += list(sub.parameters())
        if self.use_bg_nerf:
            bg += list(self.bg_dir_enc.parameters()) + list(self.bg_mlp.parameters())
        groups = {}
        for name, ps in (("encoding", enc), ("sigma", sig), ("color", col), ("background", bg)):
            if ps:
                groups[name] = {"params": ps}
        return groups

    def load_reference_state(self, state: Dict[str, torch.Tensor]):
        with torch.no_grad():
            for n, p in self.named_parameters():
                p.copy_(state[n].to(p.device, p.dtype))
        return self
