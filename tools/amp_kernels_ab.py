#!/usr/bin/env python3
"""The reference's AMP loop body (bench.dropin_run: runtime_adapt.py:286-310, GradScaler) timed under
autocast(float16) — the fp16 build of the fused MLP kernels — and under autocast(bfloat16) — the bf16 build — on the
same C3 workload (4096 rays, 64 + 128, two nets), to price the fp16 build's rounding points.  Run it under
``rocprofv3 --kernel-trace --stats`` for the per-kernel split (the two builds' kernels live in different namespaces).

  python3 tools/amp_kernels_ab.py [--steps 40] [--warmup 10]"""
import argparse
import json
import os
import sys
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "nerf-sys_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=40)
ap.add_argument("--warmup", type=int, default=10)
args = ap.parse_args()
from nerf_amd.scene import make_blender_scene  # noqa: E402
from nerf_amd.trainer import RayBatcher  # noqa: E402

dev = torch.device("cuda", 0)
scene = make_blender_scene(n_train=8, n_test=1, H=800, W=800, seed=0, device=dev)
rb = RayBatcher(scene, dev)
a = SimpleNamespace(samples=64, importance=128, batch=4096, strong=False, steps=args.steps, warmup=args.warmup)
out = {}
for name, dt in (("fp16", torch.float16), ("bf16", torch.bfloat16), ("fp16_again", torch.float16)):
    r = bench.dropin_run(rb, dev, a, 1, 0, 4096, "bf16", amp_dtype=dt)
    out[name] = {"rays_per_s": r["value"], "ms_per_step": r["ms_per_step"], "final_loss": r["final_loss"]}
    print(name, out[name], flush=True)
print(json.dumps(out))
