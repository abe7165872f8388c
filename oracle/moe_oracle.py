"""CPU restatement of the reference's MoE container — TEST INFRASTRUCTURE ONLY.

Same rules as ``nerf_oracle.py``: only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module, and only as the checker.  The product path
(``nerf-sys_amd/nerf_amd/container.py`` + ``csrc/moe.hip``) never imports it.

Restates ``MetaContainer`` (``/root/reference/adaptive_nerf/models/inr/meta_container.py``):
* ``_routing`` (:97-134): distances to the centroids on the clustering coordinates ((y, z) when
  ``cluster_2d``), soft inverse-distance weights inside ``boundary_margin`` x the nearest distance
  (margin > 1), else hard argmin;
* ``forward`` (:266-330): experts evaluated on the rows they are routed to, mixed with
  ``index_add_(w_k * y_k)`` in expert order (soft) or ``index_copy_`` (hard);
* ``background_color`` (:334-363): ``bg_mlp(SHEncoder(normalize(d)))``, Linear-ReLU-Linear-Sigmoid;
* ``get_param_groups`` (:458-503).
Pinned against golden vectors produced by importing the reference (``tools/gen_golden.py`` ->
``tests/golden/moe.npz``).  Distances are computed directly (sqrt of the sum of squares); torch.cdist
switches to the |x|^2 - 2xc + |c|^2 matrix form above 25 rows, so weights agree to fp32 rounding
(ties in the argmin / margin mask are measure-zero on the fixtures).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .ngp_oracle import sh_encode


def routing(pts, centroids, boundary_margin=1.0, cluster_2d=True):
    """meta_container.py:97-134 -> (weights (N,K) or None, hard (N,) or None)."""
    idx = [1, 2] if cluster_2d else [0, 1, 2]
    xc = pts[:, idx].float()
    cc = centroids[:, :3][:, idx].float()
    dist = (xc[:, None, :] - cc[None, :, :]).pow(2).sum(-1).sqrt()
    if boundary_margin > 1.0:
        dist = dist.clamp_min(1e-6)
        invd = 1.0 / dist
        mind = dist.min(dim=1, keepdim=True).values
        mask = dist <= (boundary_margin * mind)
        invd = invd * mask
        denom = invd.sum(dim=1, keepdim=True).clamp_min(1e-6)
        return invd / denom, None
    return None, dist.argmin(dim=1)


def container_forward(experts, x, centroids, boundary_margin=1.0, cluster_2d=True):
    """meta_container.py:266-330: experts = list of callables x (m,6) -> (m,4)."""
    N = x.shape[0]
    with torch.no_grad():
        w, hard = routing(x[:, :3], centroids, boundary_margin, cluster_2d)
    out = None
    for k, ex in enumerate(experts):
        sel = ((w[:, k] > 0) if w is not None else (hard == k)).nonzero(as_tuple=False).squeeze(1)
        if sel.numel() == 0:
            continue
        yk = ex(x.index_select(0, sel))
        if out is None:
            out = x.new_zeros(N, yk.shape[-1])
        if w is not None:
            out = out.index_add(0, sel, yk * w.index_select(0, sel)[:, k:k + 1])
        else:
            out = out.index_copy(0, sel, yk)
    return out if out is not None else x.new_zeros(N, 4)


def background_color(d, W1, b1, W2, b2, sh_levels=4):
    """meta_container.py:334-363 with bg_encoding='spherical': F.normalize, SHEncoder(levels=4), MLP."""
    dn = F.normalize(d, dim=-1)
    enc = sh_encode(dn, sh_levels)
    h = torch.relu(enc.matmul(W1.t()) + b1)
    return torch.sigmoid(h.matmul(W2.t()) + b2)
