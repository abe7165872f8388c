#!/usr/bin/env python3
"""Benchmark: rays/sec of the full NeRF train step (BASELINE.json configs[1]: Lego-style 800x800,
64 coarse + 128 fine hierarchical, fp32, two networks), data parallel over N GPUs (one process per
GPU, RCCL all-reduce of the flat gradient buffer), weak scaling (4096 rays per GPU per step).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...

Prints ONE JSON line on rank 0 (contract in the task statement), with
  roofline      — the dominant kernel (fine-net trunk GEMM class with the largest time share), its
                  algorithmic FLOP per launch / mean launch time from HIP events recorded by the
                  library inside the timed steps, against the fp32 MFMA peak (157.3 TFLOP/s);
  cpu_baseline  — the CPU oracle (a restatement of the reference's PyTorch path, pinned to its golden
                  vectors) running the same train step on a bounded sample on this host (rank 0, N=1).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "nerf-sys_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "rays/sec (train step) + full-image PSNR, 800×800 Lego, 64+128 samples"
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32, dense
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA (no sparsity)
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E peak
MAC_PER_EVAL = 500864
FLOP_PER_RAY = 769327104       # 6*MAC*(64 coarse + 192 fine evaluations), SURVEY.md §8(d)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=4096, help="rays per GPU per step")
    ap.add_argument("--samples", type=int, default=64)
    ap.add_argument("--importance", type=int, default=128)
    ap.add_argument("--train-views", type=int, default=100)
    ap.add_argument("--scene", default="blender", choices=["blender", "llff"],
                    help="blender = Lego-style 800x800 (configs[1]/[2]); llff = Fern-style 1008x756 NDC (configs[3])")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-psnr", action="store_true",
                    help="skip the full-image PSNR of one held-out view rendered after the timed steps")
    ap.add_argument("--no-overlap", action="store_true", help="run the coarse-net backward on the main stream")
    ap.add_argument("--precision", default="fp32", choices=["fp32", "bf16"],
                    help="MLP GEMM precision: fp32 = BASELINE configs[1] (default, the headline), bf16 = configs[2]")
    return ap.parse_args()


def cpu_baseline(seconds, S, NI):
    """The CPU oracle's train step (same op graph: 2 nets, 64+128, MSE, clip, Adam) on 128-ray batches."""
    from oracle import nerf_oracle as O
    torch.manual_seed(0)
    n = 128
    g = torch.Generator().manual_seed(0)
    o = torch.tensor([0.0, -4.0311, 0.5]).expand(n, 3)
    d = torch.nn.functional.normalize(torch.randn(n, 3, generator=g) * 0.15 + torch.tensor([0.0, 1.0, -0.12]), dim=-1)
    rays = torch.cat([o, d, torch.full((n, 1), 2.0), torch.full((n, 1), 6.0)], -1)
    gt = torch.rand(n, 3, generator=g)
    tr = O.OracleTrainer(O.init_vanilla_params(1), O.init_vanilla_params(2))
    tr.step(rays, gt, S, n_importance=NI)  # warm-up
    steps, t0 = 0, time.perf_counter()
    while True:
        tr.step(rays, gt, S, n_importance=NI)
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds or (steps >= 3 and el >= seconds * 0.5 and el / steps * (steps + 1) > seconds * 1.5):
            break
    return {"value": round(n * steps / el, 2), "unit": "rays/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"{steps} oracle train steps x {n} rays (64+128, 2 nets, fp32) in {el:.1f}s"}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from nerf_amd.scene import make_blender_scene, make_llff_scene
    from nerf_amd.trainer import NeRFTrainer, RayBatcher
    from nerf_amd.vanilla import VanillaNeRF

    torch.manual_seed(0)
    if a.scene == "llff":
        scene = make_llff_scene(n_train=min(a.train_views, 20), n_test=1, seed=0, device=dev)
    else:
        scene = make_blender_scene(n_train=a.train_views, n_test=1, H=800, W=800, seed=0, device=dev)
    coarse, fine = VanillaNeRF().to(dev), VanillaNeRF().to(dev)
    tr = NeRFTrainer(coarse, fine, n_samples=a.samples, n_importance=a.importance, world_size=world, device=dev,
                     overlap=not a.no_overlap, precision=a.precision)
    rb = RayBatcher(scene, dev)

    from nerf_amd.dp import shard_seed

    def one(step):
        sd = shard_seed(step, rank, world)  # disjoint per-rank ray batches
        rays, gt = rb.batch(a.batch, seed=sd)
        return tr.step(rays, gt, seed=sd)

    for s in range(a.warmup):
        loss = one(s)
    torch.cuda.synchronize()
    tr.enable_timing(a.steps)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(a.warmup, a.warmup + a.steps):
        loss = one(s)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    final_loss = float(loss.item())

    # ---- roofline of the dominant kernel: the trunk GEMM family (fwd / dgrad / wgrad classes take equal
    # shares of the step).  The fine forward shares the device with the coarse backward on the side stream,
    # so its wall durations are not per-kernel times; the fine backward runs alone.  The quoted kernel is the
    # dgrad GEMM (gemm_nt, ReLU-mask epilogue) at the fine net's M = 786,432 rows (12,288 blocks): per step 7
    # trunk launches (N = K = 256) + 1 head launch (N = 256, K = 32) -- exactly the launches the profiler's
    # per-(kernel, grid) average covers (tools/prof_summary.py).
    tm = tr.collect_timing()
    M = tm["M"]
    k256 = [1, 2, 3, 5, 6, 7]
    mean = lambda xs: sum(xs) / len(xs)
    cls = {
        "gemm_nt fwd (trunk 256x256, bias+ReLU)": mean([st[i] for st in tm["fwd"] for i in k256]),
        "gemm_wgrad (trunk 256x256, split-M)": mean([st[i] for st in tm["wgrad"] for i in k256]),
        "gemm_nt dgrad (trunk 256x256, ReLU mask)": mean([st[i - 1] for st in tm["dgrad"] for i in k256]),
    }
    dom = "gemm_nt dgrad (ReLU mask), fine net M=786432: 7 trunk 256x256 + 1 head 256x32 launches/step"
    flop_trunk, flop_head = 2.0 * M * 256 * 256, 2.0 * M * 256 * 32
    tot_ms = sum(sum(st) for st in tm["dgrad"]) + sum(tm["dgrad_head"])
    n_launch = sum(len(st) for st in tm["dgrad"]) + len(tm["dgrad_head"])
    tot_flop = flop_trunk * sum(len(st) for st in tm["dgrad"]) + flop_head * len(tm["dgrad_head"])
    ach = tot_flop / (tot_ms * 1e-3) / 1e12
    flops_launch = tot_flop / n_launch
    bf16 = a.precision == "bf16"
    traffic = None
    tpath = os.path.join(ROOT, "profiles", "traffic_bf16.json" if bf16 else "traffic.json")
    if os.path.exists(tpath):
        try:
            traffic = json.load(open(tpath)).get("gemm_nt dgrad (trunk 256x256, ReLU mask)")
        except Exception:
            traffic = None
    if bf16:
        # bf16 layers are HBM-bound: algorithmic bytes per launch = bf16 input-gradient rows in (K * 2 B) +
        # bf16 rows out (256 * 2 B) + the ReLU bitmask word row (32 B) per sample row
        by_trunk, by_head = M * (256 * 2 + 256 * 2 + 32.0), M * (32 * 2 + 256 * 2 + 32.0)
        tot_by = by_trunk * sum(len(st) for st in tm["dgrad"]) + by_head * len(tm["dgrad_head"])
        ach_gbs = tot_by / (tot_ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "kernel": dom.replace("gemm_nt", "gemm_nt_bf16"), "achieved": round(ach_gbs, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach_gbs / HBM_PEAK_GBS, 4), "traffic": traffic,
                "bytes_per_launch": tot_by / n_launch, "mfma_tflops": round(ach, 1),
                "mfma_frac_bf16": round(ach / BF16_MFMA_PEAK_TFLOPS, 4)}
    else:
        roof = {"bound": "mfma", "kernel": dom, "achieved": round(ach, 2), "peak": FP32_MFMA_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 4), "traffic": traffic,
                "flop_per_launch": flops_launch}
    roof.update({"mean_launch_ms": round(tot_ms / n_launch, 4), "classes_ms": {k: round(v, 4) for k, v in cls.items()}})
    peak_step = BF16_MFMA_PEAK_TFLOPS if bf16 else FP32_MFMA_PEAK_TFLOPS

    rays_total = a.batch * world * a.steps
    value = rays_total / el
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "rays/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "bf16" if bf16 else "f32", "data": "synthetic",
        "config": {"workload": ("Fern-style 1008x756 forward-facing NDC (synthetic analytic scene, 20 views)"
                                if a.scene == "llff" else "Lego-style 800x800 (synthetic analytic scene, 100 views)") +
                               ", 64 coarse + 128 fine hierarchical, 2 x (8x256 MLP), " +
                               ("bf16 MLP + fp32 compositing" if bf16 else "fp32") +
                               ", train step incl. ray gen + Adam",
                   "global_batch": a.batch * world, "rays_per_gpu": a.batch, "samples": [a.samples, a.importance],
                   "parallelism": f"dp{world}", "precision": a.precision},
        "roofline": roof,
        "step_mfma_frac": round(value * FLOP_PER_RAY / world / 1e12 / peak_step, 4),
        "final_loss": round(final_loss, 6),
    }
    if not a.no_psnr and rank == 0:
        from nerf_amd.ray_rendering import render_image
        tr.sync_to_modules()
        coarse.eval()
        fx, fy, cx, cy = scene.intrinsics
        img, _, _ = render_image(coarse, H=scene.H, W=scene.W, fx=fx, fy=fy, cx=cx, cy=cy, c2w=scene.test_poses[0],
                                 near=scene.near, far=scene.far, ray_samples=a.samples, n_importance=a.importance,
                                 fine_model=fine.eval(), ndc=(scene.focal, 1.0) if scene.ndc else None)
        from nerf_amd.losses import image_psnr
        out["psnr_after_steps"] = round(image_psnr(img, scene.test_images[0], "linear"), 3)
        out["psnr_note"] = ("held-out view after warmup+steps train steps (outside the timed region); "
                            "convergence: tools/train_psnr.py, profiles/r01/psnr_*.jsonl (fp32 28.1 dB / bf16 "
                            "28.1 dB after 3000 steps)")
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(a.cpu_seconds, a.samples, a.importance)
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()  # the other ranks wait for rank 0's PSNR render / report before tearing down
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
