#!/usr/bin/env python3
"""Bench of the Instant-NGP expert's train step (SURVEY.md §8f row 1 — a "next" row, not the headline
metric of bench.py): the reference's production expert (MetaNGP: 16-level hash grid, F=2, 2^20 entries
per level, max_res 4096, 64-wide sigma trunk x2, colour MLP 64 x2, SH directions; nerf_runner.py:103-121,
common/args.py) on the stratified renderer with 96 samples/ray (common/args.py:96), 4096 rays per step,
Lego-style 800x800 synthetic scene resident in HBM.

Prints one JSON line: rays/s, ms/step, per-kernel times from HIP events inside the timed steps, the
roofline of the dominant kernel against HBM peak with its algorithmic bytes per launch, and a CPU
baseline (the CPU oracle's train step, ``kind: port``) on a bounded sample.

  python tools/bench_ngp.py [--steps K] [--warmup W] [--batch N] [--samples S] [--no-cpu-baseline]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nerf-sys_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0
CONF = dict(hidden=64, sigma_depth=2, color_hidden=64, color_depth=2, dir_encoding="spherical",
            hash_enc_conf=dict(levels=16, features_per_level=2, log2_hashmap_size=20, min_res=16, max_res=4096,
                               interpolation="Linear"))
AABB = [[-1.5, -1.5, -1.5], [1.5, 1.5, 1.5]]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--samples", type=int, default=96)
    ap.add_argument("--train-views", type=int, default=100)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def cpu_baseline(seconds, S):
    """The CPU oracle's NGP train step (hash encode + MLPs + volume render + MSE + Adam) on 64-ray batches."""
    from collections import OrderedDict
    from oracle import nerf_oracle as O
    from oracle import ngp_oracle as NO
    torch.manual_seed(0)
    hc = CONF["hash_enc_conf"]
    L, F, log2T = hc["levels"], hc["features_per_level"], hc["log2_hashmap_size"]
    res, _ = NO.hash_resolutions(L, hc["min_res"], hc["max_res"])
    shapes = NO.ngp_param_shapes(L * F, 64, 2, 15, 64, 2, 16)
    p = OrderedDict((k, (torch.randn(s) * 0.1).requires_grad_(True)) for k, s in shapes.items())
    table = ((torch.rand(L * 2 ** log2T, F) * 2 - 1) * 1e-3).requires_grad_(True)
    aabb = torch.tensor(AABB)
    opt = torch.optim.Adam([{"params": [table], "lr": 1e-2}, {"params": list(p.values()), "lr": 2e-3}])
    n = 64
    g = torch.Generator().manual_seed(0)
    o = torch.tensor([0.0, -4.0311, 0.5]).expand(n, 3)
    d = torch.nn.functional.normalize(torch.randn(n, 3, generator=g) * 0.15 + torch.tensor([0.0, 1.0, -0.12]), dim=-1)
    rays = torch.cat([o, d, torch.full((n, 1), 2.0), torch.full((n, 1), 6.0)], -1)
    gt = torch.rand(n, 3, generator=g)

    def expert(x_d):
        return NO.ngp_forward(p, table, x_d, aabb, res, log2T, F, sigma_depth=2, color_depth=2)

    def step():
        rgb = O.render_rays(expert, rays, S, training=True)[0]
        loss = ((rgb.clamp(0, 1) - gt) ** 2).mean()
        opt.zero_grad()
        loss.backward()
        torch.nn.utils.clip_grad_norm_([table] + list(p.values()), 1.0)
        opt.step()

    step()
    steps, t0 = 0, time.perf_counter()
    while True:
        step()
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds or (steps >= 3 and el / steps * (steps + 1) > seconds * 1.5):
            break
    return {"value": round(n * steps / el, 2), "unit": "rays/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"{steps} oracle NGP train steps x {n} rays ({S} samples, fp32) in {el:.1f}s"}


def run(a, dev):
    """The NGP train-step bench on device ``dev``; returns the record (bench.py's ``ngp`` sub-record).  ``a`` carries
    steps, warmup, batch, samples, train_views, cpu_seconds, no_cpu_baseline."""
    from nerf_amd.ngp import InstantNGP
    from nerf_amd.ngp_trainer import NGPTrainer
    from nerf_amd.scene import make_blender_scene
    from nerf_amd.trainer import RayBatcher

    torch.manual_seed(0)
    scene = make_blender_scene(n_train=a.train_views, n_test=1, H=800, W=800, seed=0, device=dev)
    model = InstantNGP(occ_conf={}, scene_box=torch.tensor(AABB), **CONF)
    tr = NGPTrainer(model, n_samples=a.samples, device=dev)
    rb = RayBatcher(scene, dev)

    def one(step):
        rays, gt = rb.batch(a.batch, seed=step)
        return tr.step(rays, gt, seed=step)

    for s in range(a.warmup):
        loss = one(s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(a.warmup, a.warmup + a.steps):
        loss = one(s)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    # per-kernel timing in separate steps (events add no host sync, but keep the timed loop clean)
    per = {}
    for s in range(a.steps):
        tr.events = []
        one(a.warmup + a.steps + s)
        torch.cuda.synchronize()
        for name, e0, e1 in tr.events:
            per.setdefault(name, []).append(e0.elapsed_time(e1))
    tr.events = None
    ms = {k: sum(v) / len(v) for k, v in per.items()}
    hc = CONF["hash_enc_conf"]
    L, F = hc["levels"], hc["features_per_level"]
    M = a.batch * a.samples
    # algorithmic bytes per sample: positions 12 B; fwd gathers 8 corners x L x F fp32 + writes L*F fp32;
    # bwd reads d_enc L*F fp32 and read-modify-writes 8 x L x F fp32 in the table gradient
    # (fwd_enc / bwd_hash: the fused launches of the production shape, whose HBM side is the same gathers / atomics)
    by = {"hash_fwd": M * (12 + 8 * L * F * 4 + L * F * 4),
          "hash_bwd": M * (12 + L * F * 4 + 2 * 8 * L * F * 4)}
    by["fwd_enc"], by["bwd_hash"] = by["hash_fwd"], by["hash_bwd"]
    dom = max((k for k in by if k in ms), key=lambda k: ms[k])
    bk = "bwd_hash" if "bwd_hash" in ms else "hash_bwd"
    ach = by[dom] / (ms[dom] * 1e-3) / 1e9
    # the table-gradient scatter is bound by the memory-side float-atomic unit, not by HBM bytes: count the 64-B
    # atomic requests hash_bwd issues for one step's sample positions (tools/hash_requests.py)
    from nerf_amd import ngp_trainer as NT
    from hash_requests import ATOMIC_REQ_PEAK, count_requests
    seen = {}
    fname, xarg = ("ngp_bwd_hash", 4) if bk == "bwd_hash" else ("hash_encode_bwd", 1)
    orig = getattr(NT.G, fname)

    def spy(*args, **kw):
        seen.setdefault("x", args[xarg].detach().clone())
        return orig(*args, **kw)
    setattr(NT.G, fname, spy)
    one(a.warmup + 2 * a.steps)
    setattr(NT.G, fname, orig)
    nreq = count_requests(seen["x"], list(model.xyz_encoder.grid.resolutions)[:L],
                          hc["log2_hashmap_size"], model._aabb_host, model._eps)
    req_s = nreq / (ms[bk] * 1e-3)
    out = {
        "metric": "rays/sec (train step), Instant-NGP expert (SURVEY §8f row 1), 800x800 Lego-style, "
                  f"{a.samples} stratified samples",
        "value": round(a.batch * a.steps / el, 1), "unit": "rays/s", "n_gpus": 1, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 3), "higher_is_better": True,
        "dtype": "f32", "data": "synthetic",
        "config": {"workload": "MetaNGP production expert (16 levels x F=2, 2^20/level, max_res 4096, "
                               "sigma 2x64, colour 2x64, SH dirs), stratified renderer, train step incl. Adam",
                   "rays_per_step": a.batch, "samples": a.samples},
        "kernels_ms": {k: round(v, 4) for k, v in ms.items()},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None, "bytes_per_launch": by[dom],
                     "mean_launch_ms": round(ms[dom], 4)},
        "atomic_roofline": {"bound": "float-atomic requests", "kernel": bk, "requests_per_launch": nreq,
                            "achieved": round(req_s / 1e9, 2), "peak": round(ATOMIC_REQ_PEAK / 1e9, 2),
                            "unit": "G 64-B requests/s", "frac": round(req_s / ATOMIC_REQ_PEAK, 4)},
        "final_loss": round(float(loss.item()), 6),
    }
    out["cpu_baseline"] = None if a.no_cpu_baseline else cpu_baseline(a.cpu_seconds, a.samples)
    return out


def main():
    a = parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    print(json.dumps(run(a, dev)), flush=True)


if __name__ == "__main__":
    main()
