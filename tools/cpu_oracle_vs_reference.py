#!/usr/bin/env python3
"""BASELINE.md §3 gate: the CPU oracle (bench.py's `cpu_baseline`, a restatement of the reference's PyTorch
path) must run within +-10 % of the reference's own CPU speed on C1.  Runs ONLY in the build container, where
/root/reference exists: the reference is IMPORTED (never copied), with the three import-only stubs of
tools/gen_golden.py, and its MetaNeRF wrapped in gen_golden's 6-line (M,6)->(M,4) adapter.

Workload (BASELINE.json configs[0], "C1"): a 100x100 crop of an 800x800 Blender-style view (10,000 rays),
64 stratified samples, coarse network only, one train step = render_rays -> MSE (linear colour space) ->
backward -> clip_grad_norm_(1.0) -> Adam (an/pipelines/online_stage/runtime_adapt.py:286-310).  Both sides get
the same seeded weights, rays, ground truth and thread count; timing = one warm-up step, then the median of
`--steps` steps, alternating reference / oracle so host drift hits both alike.

  PYTHONDONTWRITEBYTECODE=1 python tools/cpu_oracle_vs_reference.py [--steps 5] [--threads 8]

Writes profiles/r02/cpu_oracle_vs_reference.json.
"""
import argparse
import json
import os
import statistics
import sys
import time
from collections import OrderedDict

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]
REF = "/root/reference/adaptive_nerf"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    if not os.path.isdir(REF):
        print("reference absent; nothing to do")
        return
    sys.dont_write_bytecode = True
    from gen_golden import _install_stubs
    _install_stubs()
    sys.path.insert(0, REF)
    torch.set_num_threads(a.threads)
    from nerfs import ray_rendering as rr          # noqa: E402
    from nerfs import ray_sampling as rs           # noqa: E402
    from nerfs.losses import compute_mse_loss      # noqa: E402
    from models.inr.meta_vanilla import MetaNeRF   # noqa: E402
    from oracle import nerf_oracle as O            # noqa: E402
    from types import SimpleNamespace

    class Adapter(torch.nn.Module):  # expert(x_d (M,6), params) -> (M,4), as tools/gen_golden.py
        def __init__(self, n):
            super().__init__(); self.net = n; self.use_occ = False; self.submodules = [n]

        def forward(self, x_d, params=None):
            o = self.net(x_d[:, :3], x_d[:, 3:6], params=params)
            return torch.cat([o["rgb"], o["sigma"]], -1)

    torch.manual_seed(0)
    net = MetaNeRF(encoding_dir="frequency")
    model = Adapter(net).train()
    state = OrderedDict((n, p.detach().clone()) for n, p in net.meta_named_parameters())
    # C1 rays: the centre 100x100 crop of an 800x800 Blender-style view (focal 1111.1, near 2 / far 6)
    H = W = 800
    focal = 0.5 * W / torch.tan(torch.tensor(0.5 * 0.6911112)).item()
    dirs = rs.get_ray_directions(H, W, focal, focal, W / 2, H / 2, center_pixels=True, device="cpu")
    sys.path.insert(0, os.path.join(ROOT, "nerf-sys_amd"))
    from nerf_amd.scene import hemisphere_poses  # noqa: E402  (pose generator only; no HIP call)
    rays = rs.get_rays(dirs, hemisphere_poses(1)[0], scene_box=None, near=2.0, far=6.0).view(H, W, 8)[350:450, 350:450]
    rays = rays.reshape(-1, 8).contiguous()
    g = torch.Generator().manual_seed(1)
    gt = torch.rand(rays.shape[0], 3, generator=g)
    P = SimpleNamespace(ray_samples=64, chunk_points=1 << 22, color_space="linear")
    sig = [p for n, p in net.named_parameters() if not n.startswith("color_mlp")]
    col = [p for n, p in net.named_parameters() if n.startswith("color_mlp")]
    opt = torch.optim.Adam([{"params": sig, "lr": 2e-3}, {"params": col, "lr": 2e-3}])

    def ref_step():
        opt.zero_grad()
        loss = compute_mse_loss(P, model, {"rays": rays, "rgbs": gt})
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        return float(loss)

    ot = O.OracleTrainer(state)

    def oracle_step():
        return ot.step(rays, gt, 64, n_importance=0, training=True)

    l_ref, l_or = ref_step(), oracle_step()  # warm-up (same start point: same weights, same batch)
    tr, to = [], []
    for _ in range(a.steps):
        t0 = time.perf_counter(); ref_step(); tr.append(time.perf_counter() - t0)
        t0 = time.perf_counter(); oracle_step(); to.append(time.perf_counter() - t0)
    mr, mo = statistics.median(tr), statistics.median(to)
    n = rays.shape[0]
    res = {"config": "C1: 100x100 crop (10,000 rays), 64 stratified samples, coarse net only, train step "
                     "(render_rays -> MSE -> backward -> clip -> Adam)",
           "threads": a.threads, "host": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].split(":", 1)[1].strip(),
           "reference_rays_per_s": round(n / mr, 1), "oracle_rays_per_s": round(n / mo, 1),
           "oracle_over_reference": round(mr / mo, 4), "within_10pct": abs(mr / mo - 1.0) <= 0.10,
           "first_step_loss": {"reference": l_ref, "oracle": l_or,
                               "note": "independent jitter draws (rand_like inside each path)"},
           "reference_step_s": [round(x, 3) for x in tr], "oracle_step_s": [round(x, 3) for x in to]}
    os.makedirs(os.path.join(ROOT, "profiles", "r02"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "r02", "cpu_oracle_vs_reference.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
