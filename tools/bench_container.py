#!/usr/bin/env python3
"""Bench of the reference's PRODUCTION train step (SURVEY.md §8f rows 1-3 together — not the headline metric
of bench.py): a MetaContainer of 4 Instant-NGP experts (nerf_runner.py:103-170 defaults: 16 levels x F=2,
2^20 entries/level, max_res 4096, sigma 2x64, colour 2x64, SH dirs; soft routing, boundary margin 1.05 on
(y,z); background MLP 32 wide) with occupancy-grid rendering (128^3 x 4 levels per expert, cone 0.004,
alpha_thre 1e-2, updates every 16 steps), through the reference's online train loop
(pipelines/online_stage/runtime_adapt.py:286-310): render_rays -> MSE (linear) -> backward ->
clip_grad_norm_(1.0) -> Adam with the encoding / sigma / color / background groups (common/args.py:115-119).
Every op is a HIP kernel reached through autograd; the optimiser is FlatAdam (nerf_adam on flat buffers).

Prints one JSON line: rays/s, ms/step, per-kernel-class times (HIP events), the dominant kernel's HBM
roofline and a CPU baseline (the oracle's stratified NGP container step on a bounded sample).

  python tools/bench_container.py [--steps 20] [--warmup 40] [--batch 4096]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/bench_container.py  (data parallel)
"""
import argparse
import json
import os
import sys
import time
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nerf-sys_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0
KW = dict(hidden=64, sigma_depth=2, color_hidden=64, color_depth=2, dir_encoding="spherical",
          hash_enc_conf=dict(levels=16, features_per_level=2, log2_hashmap_size=20, min_res=16, max_res=4096,
                             interpolation="Linear"))


def boxes_and_centroids():
    # 4 experts: the (y, z) quadrants of the [-1.5, 1.5]^3 scene box, overlapping by 0.1 (cluster_2d)
    b, c = [], []
    for sy in (-1, 1):
        for sz in (-1, 1):
            lo = torch.tensor([-1.5, -1.5 if sy < 0 else -0.1, -1.5 if sz < 0 else -0.1])
            hi = torch.tensor([1.5, 0.1 if sy < 0 else 1.5, 0.1 if sz < 0 else 1.5])
            b.append(torch.stack([lo, hi]))
            c.append([0.0, 0.75 * sy, 0.75 * sz])
    return b, torch.tensor(c)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=40, help="untimed steps; the occupancy warm-up is half of them")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--train-views", type=int, default=100)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend (gloo: a rehearsal of N ranks sharing one GPU; RCCL needs one GPU per rank)")
    ap.add_argument("--shard", action="store_true", help="shard FlatAdam over the ranks (reduce-scatter + all-gather)")
    ap.add_argument("--host-sized", action="store_true",
                    help="the host-sized render (two host reads of the packed sizes per step) instead of the "
                         "device-sized sync-free one (container.py, DESIGN.md §3.8)")
    ap.add_argument("--graph", dest="graph", action="store_true", default=None,
                    help="replay the train step as ONE captured hipGraph (nerf_amd/graph_step.py; world size 1, "
                         "device-sized render).  Off by default: measured no faster than eager on this ROCm "
                         "(DESIGN.md §3.8, profiles/r06/a5, a6)")
    ap.add_argument("--no-graph", dest="graph", action="store_false",
                    help="launch every kernel of the step from Python (eager; the default)")
    ap.add_argument("--no-bucket", action="store_true",
                    help="one all-reduce of the flat gradient in step() instead of per-table buckets started by the "
                         "hash-table backward")
    return ap.parse_args()


def cpu_baseline(seconds):
    """The oracle's container step (stratified, 96 samples; the occupancy marcher has no CPU reference) on
    16-ray batches: routing + 4 NGP experts + background MLP + volume render + MSE + clip + Adam."""
    from collections import OrderedDict
    from oracle import moe_oracle as MO
    from oracle import nerf_oracle as O
    from oracle import ngp_oracle as NO
    torch.manual_seed(0)
    hc = KW["hash_enc_conf"]
    L, F, log2T = hc["levels"], hc["features_per_level"], hc["log2_hashmap_size"]
    res, _ = NO.hash_resolutions(L, hc["min_res"], hc["max_res"])
    boxes, cents = boxes_and_centroids()
    experts, leaves = [], []
    for b in boxes:
        p = OrderedDict((k, (torch.randn(s) * 0.1).requires_grad_(True))
                        for k, s in NO.ngp_param_shapes(L * F, 64, 2, 15, 64, 2, 16).items())
        t = ((torch.rand(L * 2 ** log2T, F) * 2 - 1) * 1e-3).requires_grad_(True)
        experts.append(lambda x_d, p=p, t=t, b=b: NO.ngp_forward(p, t, x_d, b, res, log2T, F, sigma_depth=2,
                                                                 color_depth=2))
        leaves += [t] + list(p.values())
    bgw = [(torch.randn(32, 16) * 0.1).requires_grad_(True), torch.zeros(32, requires_grad=True),
           (torch.randn(3, 32) * 0.1).requires_grad_(True), torch.zeros(3, requires_grad=True)]
    opt = torch.optim.Adam(leaves + bgw, lr=2e-3)
    n = 16
    g = torch.Generator().manual_seed(0)
    o = torch.tensor([0.0, -4.0311, 0.5]).expand(n, 3)
    d = torch.nn.functional.normalize(torch.randn(n, 3, generator=g) * 0.15 + torch.tensor([0.0, 1.0, -0.12]), dim=-1)
    rays = torch.cat([o, d, torch.full((n, 1), 2.0), torch.full((n, 1), 6.0)], -1)
    gt = torch.rand(n, 3, generator=g)

    def step():
        bg = MO.background_color(d, *bgw)
        rgb = O.render_rays(lambda x_d: MO.container_forward(experts, x_d, cents, 1.05, True), rays, 96,
                            training=True, bg=bg)[0]
        loss = O.mse_loss(rgb, gt, "linear")
        opt.zero_grad()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(leaves + bgw, 1.0)
        opt.step()

    step()
    steps, t0 = 0, time.perf_counter()
    while True:
        step()
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds or (steps >= 2 and el / steps * (steps + 1) > seconds * 1.5):
            break
    return {"value": round(n * steps / el, 2), "unit": "rays/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"{steps} oracle container steps x {n} rays (stratified 96 samples, 4 NGP experts, fp32) "
                      f"in {el:.1f}s"}


def build_step(a, dev, rank=0, world=1):
    """The container, FlatAdam and one train step closure (step -> loss).  world > 1: data parallel — every rank
    draws its own ray batch (dp.shard_seed) and FlatAdam all-reduces the flat gradient."""
    from nerf_amd.dp import shard_seed
    from nerf_amd.container import MetaContainer
    from nerf_amd.losses import compute_mse_loss
    from nerf_amd.optim import FlatAdam
    from nerf_amd.ray_sampling import SceneBox
    from nerf_amd.scene import make_blender_scene
    from nerf_amd.trainer import RayBatcher
    torch.manual_seed(0)
    scene = make_blender_scene(n_train=a.train_views, n_test=1, H=800, W=800, seed=0, device=dev)
    boxes, cents = boxes_and_centroids()
    occ = {"use_occ": True, "resolution": 128, "levels": 4, "render_step_size": None, "occ_thre": 1e-2,
           "alpha_thre": 1e-2, "alpha_thre_start": 0.0, "alpha_thre_end": 1e-2, "cosine_anneal": True,
           "warmup_steps": a.warmup // 2, "update_interval": 16, "ema_decay": 0.95, "cone_angle": 0.004,
           "near_plane": 2.0, "far_plane": 6.0}
    model = MetaContainer(num_submodules=4, centroids=cents, aabb=torch.tensor([[-1.5] * 3, [1.5] * 3]),
                          nerf_variant="instant", boundary_margin=1.05, cluster_2d=True, use_bg_nerf=True,
                          bg_hidden=32, occ_conf=occ, expert_box_list=[SceneBox(aabb=b) for b in boxes], **KW)
    model = model.to(dev).train()
    # the sync-free step: every size after the march stays on the device (container.py "device-sized")
    model.device_sized = not getattr(a, "host_sized", False)
    lr = {"encoding": 1e-2, "sigma": 2e-3, "color": 2e-3, "background": 1e-3}
    groups = [{"params": g["params"], "lr": lr[k]} for k, g in model.get_param_groups().items()]
    opt = FlatAdam(groups, grad_clip=1.0, world_size=world, shard=a.shard, bucket_tables=not a.no_bucket)
    rb = RayBatcher(scene, dev)
    P = SimpleNamespace(ray_samples=96, chunk_points=262_144 * 17, color_space="linear")
    graph = use_graph(a, world)

    def one(step):
        model.maybe_update_expert_occupancies(step)
        rays, gt = rb.batch(a.batch, seed=shard_seed(step, rank, world))
        opt.zero_grad()
        loss = compute_mse_loss(P, model, {"rays": rays, "rgbs": gt})
        loss.backward()
        opt.step()
        return loss

    one.opt, one.graphed, one.eager = opt, None, one
    if not graph:
        return one, model
    # every step of a graph-mode run (eager or replayed) on one non-default stream, the one the graph is captured on
    # (graph_step.GraphedStep: the autograd AccumulateGrad nodes live on the stream of the eager steps)
    S = torch.cuda.Stream(device=dev)
    # graph mode (world 1): every step reads its seeds and its Adam step count from HBM, so eager steps and graph
    # replays run the same kernels; from capture_at on, the step is GraphedStep (warm-up, capture, replays)
    from nerf_amd.container import vis_thresholds
    from nerf_amd.graph_step import GraphedStep
    ctr = torch.zeros(1, dtype=torch.int64, device=dev)      # = the step index (batch seed = step * world + rank)
    model.step_seed = (ctr, 0x5EED0CC, 0x9E3779B97F4A7C15)     # marching jitter: its own counter stream
    opt.device_step()

    def body():
        rays, gt = rb.batch(a.batch, seed=rank, step_dev=ctr, seed_mul=world)
        opt.zero_grad()
        loss = compute_mse_loss(P, model, {"rays": rays, "rgbs": gt})
        loss.backward()
        opt.step()
        return loss

    def pre(step):
        ctr.fill_(step)
        model.maybe_update_expert_occupancies(step)
        if "_dev_sizes" in model.__dict__:
            vis_thresholds(model)   # in place: the captured visibility kernel reads the refreshed values

    def on_S(fn):
        # the step on S, ordered after the caller's stream work and before it (both ways: the caller reads the loss)
        cur = torch.cuda.current_stream()
        S.wait_stream(cur)
        with torch.cuda.stream(S):
            out = fn()
        cur.wait_stream(S)
        return out

    def eager(step):
        def run():
            pre(step)
            return body()
        return on_S(run)

    gs = GraphedStep(body, pre, warmup=2,
                     before_capture=lambda: model.__dict__["_dev_sizes"].freeze(device=dev))
    capture_at = max(a.warmup - 3, model.submodules[0].occ_warmup_steps + 2)

    def one_g(step):
        if step < capture_at:
            return eager(step)
        return on_S(lambda: gs(step))

    one_g.opt, one_g.graphed, one_g.eager, one_g.body, one_g.ctr, one_g.stream, one_g.on_S = opt, gs, eager, body, ctr, S, on_S
    return one_g, model


def use_graph(a, world):
    g = getattr(a, "graph", None)
    if g is None:
        g = False
    if g and (world > 1 or getattr(a, "host_sized", False)):
        raise ValueError("--graph: single rank, device-sized render only")
    return bool(g)


def run(a, dev, rank=0, world=1):
    """The container train-step bench on ``dev`` (process group already initialised when world > 1); returns the
    record (bench.py's ``container`` sub-record).  ``a`` carries steps, warmup, batch, train_views, cpu_seconds,
    no_cpu_baseline, shard, no_bucket."""
    import torch.distributed as dist
    from nerf_amd import ngp as G

    one, model = build_step(a, dev, rank, world)
    verbose = bool(os.environ.get("NERF_BENCH_VERBOSE"))
    for s in range(a.warmup):
        if verbose:
            print(f"[bench_container] warmup step {s}", file=sys.stderr, flush=True)
        loss = one(s)
    assert model.occ_ready, "occupancy warm-up did not finish"

    def fence():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    fence()
    t0 = time.perf_counter()
    host = 0.0  # host time inside the step calls: with no host sync in the step, ~ wall time means host-bound
    for s in range(a.warmup, a.warmup + a.steps):
        th = time.perf_counter()
        loss = one(s)
        host += time.perf_counter() - th
    if verbose:
        print("[bench_container] timed steps issued", file=sys.stderr, flush=True)
    fence()
    if verbose:
        print("[bench_container] timed steps done", file=sys.stderr, flush=True)
    el = time.perf_counter() - t0
    if world > 1:  # the job's time is the slowest rank's
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    # per-kernel-class times from HIP events in separate steps
    exch = None
    if world > 1:  # the exchange's exposed tail per step: HIP events around FlatAdam's wait + remaining all-reduce
        ms_ex = []
        for s in range(a.steps):
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            one.opt.exchange_events = ev
            one(a.warmup + a.steps + s)
            torch.cuda.synchronize()
            ms_ex.append(ev[0].elapsed_time(ev[1]))
        one.opt.exchange_events = None
        exch = {"exposed_exchange_ms": round(sum(ms_ex) / len(ms_ex), 4), "bucketed": one.opt.bucket_tables,
                "grad_bytes": int(one.opt.grad.numel() * 4),
                "note": "events on the compute stream around FlatAdam's wait for the table buckets (started by each "
                        "expert's hash backward) plus the all-reduce of the remaining ranges; mean over the steps"}
    G.TIMING.enabled = True
    for s in range(a.steps):   # (graph mode: the same step launched eagerly — a replay records no events)
        one.eager(a.warmup + a.steps + s)
    per = G.TIMING.collect()
    G.TIMING.enabled = False
    if verbose:
        print("[bench_container] timing pass done", file=sys.stderr, flush=True)
    ms = {k: sum(t for t, _ in v) / a.steps for k, v in per.items()}          # per step (all experts)
    launch = {k: sum(t for t, _ in v) / len(v) for k, v in per.items()}      # per launch
    n_launch = {k: len(v) / a.steps for k, v in per.items()}
    rows = {k: sum(r for _, r in v) for k, v in per.items()}
    dom = max(ms, key=ms.get)
    # algorithmic bytes of the hash-grid kernels per sample (L=16, F=2): fwd 12 + 8*L*F*4 + L*F*4;
    # bwd 12 + L*F*4 + 2*8*L*F*4 (atomic read-modify-write)
    L, F = 16, 2
    bps = {"hash_fwd": 12 + 8 * L * F * 4 + L * F * 4, "hash_bwd": 12 + L * F * 4 + 2 * 8 * L * F * 4}
    # the fused launches of the production shape: the forward's gathers as hash_fwd; the fused MLP backward + table
    # scatter (bwd_hash) has its own model — x_d row 24 B + the enc row its MLP recompute reads (L*F*4) + d_rgb_sigma
    # 16 B + the atomic read-modify-write of 8 corners x L x F floats; d_enc stays in LDS (no HBM traffic)
    bps.update(fwd_enc=bps["hash_fwd"], density_enc=bps["hash_fwd"],
               bwd_hash=24 + L * F * 4 + 16 + 2 * 8 * L * F * 4)
    labels = {"bwd_hash": "bwd_hash (fused MLP backward + table scatter)"}
    hk = max((k for k in bps if k in per), key=lambda k: ms.get(k, 0.0))
    tot_ms = sum(t for t, _ in per[hk])
    ach = bps[hk] * rows[hk] / (tot_ms * 1e-3) / 1e9
    roof = {"bound": "hbm", "kernel": labels.get(hk, hk), "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
            "bytes_per_launch": round(bps[hk] * rows[hk] / len(per[hk])), "mean_launch_ms": round(launch[hk], 4)}
    out = {
        "metric": "rays/sec (train step), production MoE container: 4 Instant-NGP experts + occupancy rendering "
                  "+ background MLP (SURVEY §8f rows 1-3), 800x800 Lego-style",
        "value": round(a.batch * world * a.steps / el, 1), "unit": "rays/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 3),
        "host_ms_per_step": round(host / a.steps * 1e3, 3), "higher_is_better": True, "dtype": "f32",
        "data": "synthetic",
        "config": {"workload": "MetaContainer(4 x MetaNGP 16x2^20, 2x64 / 2x64, SH), soft routing bm 1.05, "
                               "occupancy 128^3 x 4 levels, bg MLP 32, autograd train step + FlatAdam",
                   "rays_per_step": a.batch * world, "parallelism": f"dp{world}"},
        "kernels_ms_per_step": {k: round(v, 4) for k, v in ms.items()},
        "launches_per_step": {k: round(v, 2) for k, v in n_launch.items()},
        "mean_launch_ms": {k: round(v, 4) for k, v in launch.items()},
        "dominant": dom,
        "roofline": roof,
        "samples_per_step": round((rows.get("fwd_enc", 0) + rows.get("mlp_fwd", 0)) / a.steps),
        "final_loss": round(float(loss.item()), 6),
    }
    if exch:
        out["exchange"] = exch
    sz = model.__dict__.get("_dev_sizes")
    if one.graphed is not None:
        mx, over = sz.frozen_report()
        out["graph"] = {"captured": one.graphed.graph is not None, "replays": one.graphed.calls - one.graphed.warmup,
                        "capacity": sz.cap, "max_march_samples_frozen": mx, "overflow": over,
                        "note": "timed steps are replays of ONE hipGraph of the whole train step (nerf_amd/"
                                "graph_step.py): seeds and the Adam step count read from HBM, occupancy updates "
                                "eager between replays; kernels_ms_per_step from eager launches of the same step"}
    else:
        out["graph"] = None
    if model.device_sized and sz is not None:
        torch.cuda.synchronize()
        sz.poll()
        out["device_sized"] = {"capacity": sz.cap, "max_march_samples": sz.max_seen, "calls": sz.calls,
                               "overflows": sz.overflows,
                               "note": "every size after the march read on the device (no host sync in the step); "
                                       "buffers sized for `capacity` samples (>= 2x the largest march seen); the "
                                       "kernels' grids cover the capacity, their row counts (the roofline's bytes) "
                                       "are the real ones, read back after the timed steps"}
    else:
        out["device_sized"] = None
    if world > 1:   # the replicas after every step above: one gradient exchange per step keeps them bitwise equal
        from nerf_amd.dp import params_checksum
        out["dp"] = {"world_size": world, "backend": dist.get_backend(), "flat_adam": {
            "world_size": one.opt.world_size, "shard": one.opt.shard, "bucket_tables": one.opt.bucket_tables,
            "grad_bytes": int(one.opt.grad.numel() * 4)}, **params_checksum(one.opt.flat, world)}
    out["cpu_baseline"] = None if (a.no_cpu_baseline or world > 1) else cpu_baseline(a.cpu_seconds)
    return out


def main():
    import faulthandler
    faulthandler.enable()
    a = parse()
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local % torch.cuda.device_count())  # a gloo rehearsal may run more ranks than GPUs
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group(a.backend, device_id=dev if a.backend == "nccl" else None)
    out = run(a, dev, rank, world)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
