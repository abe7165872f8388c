#!/usr/bin/env python3
"""Convergence run of the benchmarked train step: train the C2 workload (Lego-style 800x800 synthetic
scene, 4096 rays/step, 64 coarse + 128 fine, two 8x256 networks) on one GPU and report full-image PSNR on
held-out views at checkpoints — the "full-image PSNR" half of BASELINE.json's metric.

  python tools/train_psnr.py --steps 3000 --eval-every 1000 [--scene blender|llff] [--test-views 2]

Writes one JSON line per checkpoint to stdout (and --out): step, wall seconds of training so far
(excluding evaluation), loss, mean PSNR over the test views, rays/s.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nerf-sys_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="blender", choices=["blender", "llff"])
    ap.add_argument("--steps", type=int, default=3000)
    ap.add_argument("--eval-every", type=int, default=1000)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--samples", type=int, default=64)
    ap.add_argument("--importance", type=int, default=128)
    ap.add_argument("--lr", type=float, default=2e-3, help="sigma/color group lr (reference default, args.py:116-117)")
    ap.add_argument("--train-views", type=int, default=100)
    ap.add_argument("--test-views", type=int, default=2)
    ap.add_argument("--out", default=None)
    ap.add_argument("--precision", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--jitter-seed", type=int, default=0,
                    help="offset of the per-step jitter seeds (same batches, same initial weights): noise-band runs")
    a = ap.parse_args()

    from nerf_amd.scene import make_blender_scene, make_llff_scene
    from nerf_amd.trainer import NeRFTrainer, RayBatcher
    from nerf_amd.vanilla import VanillaNeRF
    from nerf_amd.ray_rendering import render_image
    from nerf_amd.losses import image_psnr

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    if a.scene == "blender":
        scene = make_blender_scene(n_train=a.train_views, n_test=a.test_views, seed=0, device=dev)
        ndc = None
    else:
        scene = make_llff_scene(n_train=min(a.train_views, 20), n_test=a.test_views, seed=0, device=dev)
        ndc = (scene.focal, 1.0)
    coarse, fine = VanillaNeRF().to(dev), VanillaNeRF().to(dev)
    tr = NeRFTrainer(coarse, fine, n_samples=a.samples, n_importance=a.importance, lr_sigma=a.lr, lr_color=a.lr,
                     device=dev, precision=a.precision)
    rb = RayBatcher(scene, dev)
    fx, fy, cx, cy = scene.intrinsics
    outf = open(a.out, "w") if a.out else None

    def evaluate():
        tr.sync_to_modules()
        coarse.eval(), fine.eval()
        ps = []
        for v in range(scene.test_poses.shape[0]):
            img, _, _ = render_image(coarse, H=scene.H, W=scene.W, fx=fx, fy=fy, cx=cx, cy=cy,
                                     c2w=scene.test_poses[v], near=scene.near, far=scene.far,
                                     ray_samples=a.samples, n_importance=a.importance, fine_model=fine, ndc=ndc)
            ps.append(image_psnr(img, scene.test_images[v], "linear"))
        coarse.train(), fine.train()
        return sum(ps) / len(ps)

    train_s = 0.0
    step = 0
    while step < a.steps:
        n = min(a.eval_every, a.steps - step)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            rays, gt = rb.batch(a.batch, seed=step)
            loss = tr.step(rays, gt, seed=step + a.jitter_seed * 1000003)
            step += 1
        torch.cuda.synchronize()
        train_s += time.perf_counter() - t0
        rec = {"scene": a.scene, "precision": a.precision, "jitter_seed": a.jitter_seed,
               "lib": os.path.basename(os.environ.get("NERF_AMD_LIB", "libnerf_amd.so")), "step": step, "train_s": round(train_s, 2), "loss": round(float(loss.item()), 6),
               "psnr": round(evaluate(), 3), "rays_per_s": round(step * a.batch / train_s, 1)}
        print(json.dumps(rec), flush=True)
        if outf:
            outf.write(json.dumps(rec) + "\n")
            outf.flush()


if __name__ == "__main__":
    main()
