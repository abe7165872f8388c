#!/usr/bin/env python3
"""BASELINE.json configs[4]: "8-scene nerf_synthetic sweep, 4096-ray batches, 8xMI355X, report mean PSNR +
aggregate rays/sec vs roofline".

Eight Lego-style synthetic scenes (seeds 0..7 of nerf_amd.scene: different seeded sphere layouts and
hemisphere poses; nerf_synthetic itself is not in the image) are trained independently with the
benchmarked train step (4096 rays/step, 64 coarse + 128 fine, two 8x256 networks).  Under torchrun with W
ranks, rank r trains scenes r, r+W, ... on its own GPU — the scenes are independent, so there is no
collective on the data path; the per-scene results are gathered once at the end.  On one GPU the eight
scenes run back to back.

  python tools/sweep_scenes.py [--steps 1000] [--precision fp32|bf16] [--scenes 8]
  torchrun --nproc-per-node 8 tools/sweep_scenes.py ...

Prints one JSON line per scene and a summary: mean PSNR, aggregate rays/s (sum over GPUs of each GPU's
training throughput), and the aggregate MFMA-roofline fraction (FLOP/ray of SURVEY §8d).
"""
import argparse
import faulthandler
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nerf-sys_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

# a native fault (HIP runtime, profiler, ctypes) prints every thread's Python stack instead of a bare address list
faulthandler.enable(all_threads=True)

FLOP_PER_RAY = 769327104
PEAK = {"fp32": 157.3e12, "bf16": 2500e12}


def _psnr(coarse, fine, scene, S=64, NI=128):
    from nerf_amd.losses import image_psnr
    from nerf_amd.ray_rendering import render_image
    fx, fy, cx, cy = scene.intrinsics
    ps = []
    for v in range(scene.test_poses.shape[0]):
        img, _, _ = render_image(coarse, H=scene.H, W=scene.W, fx=fx, fy=fy, cx=cx, cy=cy, c2w=scene.test_poses[v],
                                 near=scene.near, far=scene.far, ray_samples=S, n_importance=NI, fine_model=fine)
        ps.append(image_psnr(img, scene.test_images[v], "linear"))
    return sum(ps) / len(ps)


def train_scene(sid, *, steps, batch, train_views, test_views, precision, lr, dev, H=800, W=800,
                initial_psnr=False):
    """Train one seeded synthetic scene with the benchmarked step; returns its record (PSNR over the held-out
    views, train-loop rays/s, the per-step loss trajectory)."""
    from nerf_amd.scene import make_blender_scene
    from nerf_amd.trainer import NeRFTrainer, RayBatcher
    from nerf_amd.vanilla import VanillaNeRF
    torch.manual_seed(sid)
    scene = make_blender_scene(n_train=train_views, n_test=test_views, H=H, W=W, seed=sid, device=dev)
    coarse, fine = VanillaNeRF().to(dev), VanillaNeRF().to(dev)
    rec = {"scene_seed": sid}
    if initial_psnr:
        rec["psnr_init"] = round(_psnr(coarse.eval(), fine.eval(), scene), 3)
    tr = NeRFTrainer(coarse, fine, n_samples=64, n_importance=128, lr_sigma=lr, lr_color=lr, device=dev,
                     precision=precision)
    rb = RayBatcher(scene, dev)
    losses = torch.zeros(steps, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for step in range(steps):
        rays, gt = rb.batch(batch, seed=step)
        losses[step:step + 1].copy_(tr.step(rays, gt, seed=step))
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    tr.sync_to_modules()
    coarse.eval(), fine.eval()
    ls = losses.cpu().tolist()
    rec.update({"steps": steps, "train_s": round(el, 2), "rays_per_s": round(steps * batch / el, 1),
                "loss": round(ls[-1], 6), "psnr": round(_psnr(coarse, fine, scene), 3), "losses": ls})
    return rec


def summarize(results, batch, precision, world=1):
    """configs[4] summary: mean PSNR over the scenes, aggregate rays/s (every GPU trains its scenes concurrently; a
    GPU's rate = its rays / its training time; summed over GPUs) and the aggregate MFMA-roofline fraction."""
    per_gpu = {}
    for r in results:
        per_gpu.setdefault(r.get("rank", 0), []).append(r)
    agg = sum(sum(x["steps"] for x in rs) * batch / sum(x["train_s"] for x in rs) for rs in per_gpu.values())
    return {"config": "configs[4]: 8-scene synthetic sweep, 4096-ray batches, 64+128, 2 x (8x256 MLP)",
            "precision": precision, "n_gpus": world, "scenes": len(results), "batch": batch,
            "mean_psnr": round(sum(r["psnr"] for r in results) / len(results), 3),
            "aggregate_rays_per_s": round(agg, 1),
            "aggregate_mfma_frac": round(agg * FLOP_PER_RAY / (world * PEAK[precision]), 4),
            "data": "synthetic (seeded analytic scenes 0..7; nerf_synthetic not in the image)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenes", type=int, default=8)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--lr", type=float, default=2e-3)
    ap.add_argument("--train-views", type=int, default=100)
    ap.add_argument("--test-views", type=int, default=2)
    ap.add_argument("--size", type=int, default=800, help="image height = width")
    ap.add_argument("--precision", default="fp32", choices=["fp32", "bf16"])
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")  # only the final result gather crosses ranks
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    results = []
    for sid in range(rank, a.scenes, world):
        rec = train_scene(sid, steps=a.steps, batch=a.batch, train_views=a.train_views, test_views=a.test_views,
                          precision=a.precision, lr=a.lr, dev=dev, H=a.size, W=a.size)
        rec["rank"] = rank
        rec.pop("losses", None)
        print(json.dumps(rec), flush=True)
        results.append(rec)
        torch.cuda.empty_cache()
    if world > 1:
        allr = [None] * world
        dist.all_gather_object(allr, results)
        results = [r for rr in allr for r in rr]
    if rank == 0:
        print(json.dumps(summarize(results, a.batch, a.precision, world)), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
