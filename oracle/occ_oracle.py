"""CPU restatement of the occupancy-grid renderer — TEST INFRASTRUCTURE ONLY.  **Parity unpinned.**

Same rules as ``nerf_oracle.py``: only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module, and only as the checker.

The reference renders Instant-NGP experts with nerfacc 0.5.3 (``requirements.txt:6``): ``OccGridEstimator``
(``sampling``, ``update_every_n_steps``, ``mark_invisible_cells``), ``render_weight_from_density``,
``accumulate_along_rays`` and ``pack_info`` (call sites ``nerfs/ray_rendering.py:349-558``,
``models/inr/meta_ngp.py:108-145, 318-443``).  nerfacc's source is not in the image and no reference test
pins it, so this module restates the PUBLISHED algorithms (nerfacc docs / Instant-NGP paper), and the
build's HIP kernels are checked against this restatement plus known-answer properties:

* transmittance ``T_i = exp(-sum_{j<i} sigma_j dt_j)``, ``alpha_i = 1 - exp(-sigma_i dt_i)``,
  ``w_i = T_i alpha_i`` over packed per-ray segments (``render_weight_from_density``);
* ``accumulate_along_rays``: per-ray sums of ``w_i * v_i``;
* visibility: keep samples with ``T_i >= early_stop_eps`` and ``alpha_i >= alpha_thre``;
* occupancy marching over a multi-level grid (level l covers the ROI box scaled by 2^l about its centre):
  step ``dt = clamp(t * cone_angle, step, 1e10)``; a sample ``[t, t+dt)`` is emitted when the cell holding
  its midpoint (finest level containing it) is occupied; empty cells are skipped to the first step of
  the ``dt`` lattice past the cell's exit.
"""
from __future__ import annotations

import math

import torch


def level_aabbs(roi, levels):
    roi = torch.as_tensor(roi, dtype=torch.float32).reshape(6)
    c = (roi[:3] + roi[3:]) * 0.5
    h = (roi[3:] - roi[:3]) * 0.5
    return torch.stack([torch.cat([c - h * 2 ** l, c + h * 2 ** l]) for l in range(levels)])


def march(o, d, near, far, binaries, roi, R, step, cone_angle=0.0, max_steps=4096):
    """Per-ray occupancy marching (restated algorithm above).  binaries (L,R,R,R) bool.
    Returns (ray_indices, t0, t1) packed, ray-major."""
    L = binaries.shape[0]
    roi = torch.as_tensor(roi, dtype=torch.float32).reshape(6)
    c = (roi[:3] + roi[3:]) * 0.5
    h = (roi[3:] - roi[:3]) * 0.5
    ri, t0s, t1s = [], [], []
    for r in range(o.shape[0]):
        oo, dd = o[r].double(), d[r].double()
        t, tf = float(near[r]), float(far[r])
        # clip to the outermost level's box
        lo, hi = (c - h * 2 ** (L - 1)).double(), (c + h * 2 ** (L - 1)).double()
        tmin, tmax = -math.inf, math.inf
        for a in range(3):
            if abs(float(dd[a])) < 1e-12:
                if not (lo[a] <= oo[a] <= hi[a]):
                    tmin, tmax = 1.0, 0.0
                continue
            ta, tb = float((lo[a] - oo[a]) / dd[a]), float((hi[a] - oo[a]) / dd[a])
            tmin, tmax = max(tmin, min(ta, tb)), min(tmax, max(ta, tb))
        t, tf = max(t, tmin), min(tf, tmax)
        n = 0
        while t < tf and n < max_steps:
            n += 1
            dt = min(max(t * cone_angle, step), 1e10)
            mid = t + 0.5 * dt
            if mid >= tf:
                break
            p = oo + dd * mid
            s = float(((p - c.double()).abs() / h.double()).max())
            lvl = 0 if s <= 1.0 else int(math.ceil(math.log2(s)))
            if lvl >= L:
                break
            mn = (c - h * 2 ** lvl).double()
            sz = (h * 2 ** (lvl + 1)).double()
            cell = ((p - mn) / sz * R).floor().clamp(0, R - 1).long()
            if bool(binaries[lvl, cell[0], cell[1], cell[2]]):
                ri.append(r)
                t0s.append(t)
                t1s.append(t + dt)
                t = t + dt
            else:
                cmin = mn + cell.double() * sz / R
                cmax = cmin + sz / R
                te = math.inf
                for a in range(3):
                    if abs(float(dd[a])) > 1e-12:
                        te = min(te, float(((cmax[a] if dd[a] > 0 else cmin[a]) - oo[a]) / dd[a]))
                k = max(1, math.ceil((te - t) / dt))
                t = t + k * dt
    return (torch.tensor(ri, dtype=torch.int64), torch.tensor(t0s, dtype=torch.float32),
            torch.tensor(t1s, dtype=torch.float32))


def packed_weights(t0, t1, sigmas, ray_indices, n_rays):
    """render_weight_from_density: (weights, trans, alphas)."""
    sdt = sigmas * (t1 - t0)
    alphas = 1.0 - torch.exp(-sdt)
    trans = torch.empty_like(sdt)
    for r in range(n_rays):
        sel = (ray_indices == r).nonzero().squeeze(1)
        if sel.numel():
            cs = torch.cumsum(sdt[sel], 0)
            trans[sel] = torch.exp(-(cs - sdt[sel]))
    return trans * alphas, trans, alphas


def accumulate(weights, values, ray_indices, n_rays):
    """accumulate_along_rays."""
    v = weights[:, None] if values is None else weights[:, None] * values
    out = torch.zeros(n_rays, v.shape[1], dtype=v.dtype)
    return out.index_add(0, ray_indices, v)


def visibility(t0, t1, sigmas, ray_indices, n_rays, early_stop_eps=1e-4, alpha_thre=0.0):
    _, trans, alphas = packed_weights(t0, t1, sigmas, ray_indices, n_rays)
    vis = trans >= early_stop_eps
    if alpha_thre > 0:
        vis = vis & (alphas >= alpha_thre)
    return vis


def render_packed(rgb_sigma, t0, t1, ray_indices, n_rays, bg=None):
    """render_expert_occ's integration (nerfs/ray_rendering.py:537-557): rgb, depth, weights, acc."""
    w, _, _ = packed_weights(t0, t1, rgb_sigma[:, 3], ray_indices, n_rays)
    rgb = accumulate(w, rgb_sigma[:, :3], ray_indices, n_rays)
    tm = 0.5 * (t0 + t1)
    depth = accumulate(w, tm[:, None], ray_indices, n_rays).squeeze(-1)
    acc = accumulate(w, None, ray_indices, n_rays).squeeze(-1)
    if bg is not None:
        rgb = rgb + (1.0 - acc)[:, None] * bg
    return rgb, depth, w, acc
