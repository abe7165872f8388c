#!/usr/bin/env python3
"""Benchmark: rays/sec of the full NeRF train step (BASELINE.json configs[1]: Lego-style 800x800,
64 coarse + 128 fine hierarchical, fp32, two networks), data parallel over N GPUs (one process per
GPU, the flat gradient buffer all-reduced over RCCL in two buckets per step: coarse net as soon as its backward
ends, fine net + loss after the fine backward).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--strong] [--path engine|dropin] [--precision fp32|bf16]

With --gpus N > 1 and no torchrun environment, bench.py starts `torch.distributed.run` with N ranks itself
(before any GPU call) and exits with its status; under the driver's own torchrun it runs as one rank.
Weak scaling (default): 4096 rays per GPU per step.  --strong: 4096 rays per step in total, each rank taking
the rank-strided slice of the same global draw (an/scripts/create_clusters.py:799).

Prints ONE JSON line on rank 0 (contract in the task statement), with
  roofline      — the dominant kernel class of the fine net's trunk GEMMs: the class (fwd / dgrad / wgrad)
                  with the largest mean launch time.  Durations are HIP events the library records on the
                  launch stream in --timing-steps (default 3) extra steps AFTER the timed region, run with
                  every launch alone on the device (the production step runs the coarse backward on a second
                  stream beside the fine backward, --overlap-with; a launch's wall time is shared there); achieved = algorithmic FLOP per launch / mean.
                  With --precision bf16 the MLP is one fused forward launch plus one fused backward launch
                  per trunk layer (HBM-bound): the kernel with the largest total time per step is reported
                  against the HBM peak, with algorithmic bytes per launch (roofline_bf16).
  bf16 / fp32   — the other MLP precision's engine step timed in the same run (BASELINE configs[2] beside
                  configs[1]), with its own roofline, step MFMA fraction and (N = 1) its drop-in loop body.
  psnr          — the metric's PSNR half: both precisions' engines, from the same seed-0 weights and
                  batches, continue to --psnr-steps total steps (outside the timed region), then render every
                  held-out 800x800 view; mean full-image PSNR per precision and the bf16 - fp32 gap.  At N > 1 every
                  rank trains the replica (data parallel, global batch N x 4096) and rank 0 renders it after an
                  all-gathered parameter checksum (params_equal_across_ranks per precision).
  dp            — (N > 1) per-rank step time (max / min), HIP-event time of each all-reduce bucket, and
                  params_equal_across_ranks: an all-gathered fp64 sum + bit hash of every rank's parameters.
  llff          — BASELINE configs[3] (C4): the Fern-style 1008x756 NDC scene, same fp32 engine, --llff-steps steps.
  sweep         — BASELINE configs[4] (C5): 8 seeded scenes x --sweep-steps bf16 4096-ray steps, rank r training
                  scenes r, r+N, ...; aggregate rays/s vs the bf16 MFMA roofline and mean held-out PSNR.
  ngp           — (N = 1) the reference's production expert (MetaNGP, 16 x 2^20 hash grid, 96 stratified samples) train
                  step: rays/s, per-kernel times, the table scatter against the float-atomic request rate, CPU oracle
                  beside it (tools/bench_ngp.py).
  container     — the production MoE container (4 NGP experts + occupancy marching + background MLP,
                  autograd + FlatAdam): rays/s, per-kernel-class times, the hash kernels' HBM roofline, CPU oracle
                  (tools/bench_container.py).  At N > 1: FlatAdam(world_size=N) with the bucketed gradient
                  all-reduce, and a `dp` block (params_equal_across_ranks).
  cpu_baseline  — the CPU oracle (a restatement of the reference's PyTorch path, pinned to its golden
                  vectors) running the same train step (4096 rays, 64+128, 2 nets), median of >= 5 steps
                  on this host's CPU share (rank 0, after every GPU leg; at N > 1 the other ranks wait in a
                  gloo barrier); `all_cores` beside it at os.cpu_count() threads.
  dropin        — (N=1) the reference's own loop body (an/pipelines/online_stage/runtime_adapt.py:286-310:
                  render_rays -> compute_mse_loss -> backward -> clip_grad_norm_ -> torch Adam; under
                  autocast + GradScaler for bf16) on this repo's drop-in render_rays + VanillaNeRF autograd
                  path, same workload, timed beside the fused engine.  --path dropin makes it the reported value.
"""
import argparse
import faulthandler
import json
import os
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "nerf-sys_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (importing torch initialises no GPU)
import torch.distributed as dist  # noqa: E402

# a native fault (HIP runtime, profiler, ctypes) prints every thread's Python stack instead of a bare address list
faulthandler.enable(all_threads=True)

METRIC = "rays/sec (train step) + full-image PSNR, 800×800 Lego, 64+128 samples"
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 / 16x16x4_f32, dense
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA (no sparsity)
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E peak
MAC_PER_EVAL = 500864
FLOP_PER_RAY = 769327104       # 6*MAC*(64 coarse + 192 fine evaluations), SURVEY.md §8(d)
K256 = [1, 2, 3, 5, 6, 7]      # trunk layers with a 256x256 weight (trunk.0: K=63, trunk.4: K=319)


_T0 = time.perf_counter()


def progress(msg):
    """A heartbeat on stderr (stdout carries only the one JSON line): the long legs (PSNR training, the CPU baseline)
    would otherwise print nothing for minutes."""
    print(f"[bench {time.perf_counter() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=4096,
                    help="rays per GPU per step (weak scaling) or per step in total (--strong)")
    ap.add_argument("--strong", action="store_true", help="strong scaling: --batch rays per step over all ranks")
    ap.add_argument("--samples", type=int, default=64)
    ap.add_argument("--importance", type=int, default=128)
    ap.add_argument("--train-views", type=int, default=100)
    ap.add_argument("--scene", default="blender", choices=["blender", "llff"],
                    help="blender = Lego-style 800x800 (configs[1]/[2]); llff = Fern-style 1008x756 NDC (configs[3])")
    ap.add_argument("--path", default="engine", choices=["engine", "dropin"],
                    help="engine = the fused train step (headline); dropin = the reference loop body on the "
                         "drop-in render_rays / VanillaNeRF autograd surface")
    ap.add_argument("--cpu-batch", type=int, default=4096)
    ap.add_argument("--cpu-steps", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-dropin", action="store_true", help="skip the drop-in path measurement beside the engine")
    ap.add_argument("--no-psnr", action="store_true",
                    help="skip the full-image PSNR record (training to --psnr-steps + held-out renders, N = 1 only)")
    ap.add_argument("--no-overlap", action="store_true", help="run the coarse-net backward on the main stream")
    ap.add_argument("--overlap-with", default="bwd", choices=["fwd", "bwd"],
                    help="what the side-stream coarse backward runs beside: the fine backward (default) or forward")
    ap.add_argument("--split-wgrad", action="store_true",
                    help="fp32: the fine net's weight-gradient GEMMs on a second stream (nerf_mlp_bwd_2s)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (the product); gloo = rehearsal of N ranks sharing the visible GPUs")
    ap.add_argument("--precision", default="fp32", choices=["fp32", "bf16"],
                    help="MLP GEMM precision: fp32 = BASELINE configs[1] (default, the headline), bf16 = configs[2]")
    ap.add_argument("--timing-steps", type=int, default=3,
                    help="timed steps (the last ones) whose fine-net launches are bracketed by HIP events")
    ap.add_argument("--bf16-flags", type=int, default=0,
                    help="A/B runs of the layered bf16 launches (1 = layered forward, 2 = layered backward)")
    ap.add_argument("--no-other-precision", action="store_true",
                    help="skip the sub-record of the other MLP precision (bf16 beside fp32, or fp32 beside bf16)")
    ap.add_argument("--psnr-steps", type=int, default=3000,
                    help="total train steps of each precision's engine before the held-out PSNR renders")
    ap.add_argument("--psnr-views", type=int, default=8, help="held-out 800x800 views rendered for the PSNR")
    ap.add_argument("--no-llff", action="store_true", help="skip the C4 (Fern-style NDC) sub-record")
    ap.add_argument("--llff-steps", type=int, default=20, help="timed steps of the C4 sub-record")
    ap.add_argument("--no-sweep", action="store_true", help="skip the C5 (8-scene sweep) sub-record")
    ap.add_argument("--sweep-scenes", type=int, default=8)
    ap.add_argument("--sweep-steps", type=int, default=500, help="bf16 train steps per scene of the C5 sub-record")
    ap.add_argument("--sweep-views", type=int, default=20, help="training views per C5 scene")
    ap.add_argument("--fp32-gemm", default="split", choices=["split", "native_dgrad", "native"],
                    help="fp32 trunk GEMMs: all as bf16 split products (gemm_x6.hpp, default), input gradients on the "
                         "fp32 MFMA (native_dgrad), or all on the fp32 MFMA kernels (native)")
    ap.add_argument("--no-ngp", action="store_true",
                    help="skip the Instant-NGP expert sub-record (SURVEY §8f row 1, tools/bench_ngp.py)")
    ap.add_argument("--no-container", action="store_true",
                    help="skip the production MoE-container sub-record (SURVEY §8f rows 1-3, tools/bench_container.py)")
    ap.add_argument("--container-steps", type=int, default=48, help="timed steps of the container sub-record")
    ap.add_argument("--container-warmup", type=int, default=40,
                    help="untimed container steps (the occupancy warm-up is half of them)")
    ap.add_argument("--prod-cpu-seconds", type=float, default=12.0,
                    help="CPU-oracle sample of the ngp / container sub-records (seconds)")
    ap.add_argument("--no-native-ref", action="store_true",
                    help="skip the fp32-MFMA (native) engine leg timed beside the split-GEMM engine")
    return ap.parse_args()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(a):
    """--gpus N > 1 outside torchrun: run N ranks under torch.distributed.run as a CHILD process (no exec, no
    GPU touched in this process) and return its exit status."""
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_share():
    """What this process may run on: the affinity mask and the cgroup v2 CPU quota (cpu.max), if readable."""
    info = {"host_cpus": os.cpu_count()}
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        pass
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        info["cgroup_cpu_quota"] = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return info


def _oracle_step_rate(S, NI, n, steps, threads, budget_s=None):
    from oracle import nerf_oracle as O
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    g = torch.Generator().manual_seed(0)
    o = torch.tensor([0.0, -4.0311, 0.5]).expand(n, 3)
    d = torch.nn.functional.normalize(torch.randn(n, 3, generator=g) * 0.15 + torch.tensor([0.0, 1.0, -0.12]), dim=-1)
    rays = torch.cat([o, d, torch.full((n, 1), 2.0), torch.full((n, 1), 6.0)], -1)
    gt = torch.rand(n, 3, generator=g)
    tr = O.OracleTrainer(O.init_vanilla_params(1), O.init_vanilla_params(2))
    tr.step(rays[:128], gt[:128], S, n_importance=NI)  # warm-up (allocator, thread pool)
    times = []
    for _ in range(steps):
        t0 = time.perf_counter()
        tr.step(rays, gt, S, n_importance=NI)
        times.append(time.perf_counter() - t0)
        progress(f"cpu baseline: {n} rays x {threads} threads: step {len(times)}/{steps} {times[-1]:.2f} s")
        if budget_s is not None and sum(times) > budget_s:
            break
    return statistics.median(times), times


def _baseline_threads(world):
    """OMP_NUM_THREADS (the box's CPU share: 16 on a one-GPU box).  Under torchrun at N > 1 an unset OMP_NUM_THREADS
    becomes 1 per rank; rank 0 then uses the share it may run on (affinity, bounded by the cgroup quota), since
    the other ranks sit blocked in a barrier while it runs."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and not (world > 1 and env == "1"):
        return int(env)
    sh = _cpu_share()
    n = sh.get("affinity_cpus") or os.cpu_count() or 1
    q = sh.get("cgroup_cpu_quota")
    return max(1, min(n, int(q))) if q else n


def cpu_baseline(S, NI, n, steps, world=1):
    """The CPU oracle's train step (same op graph: 2 nets, 64+128, MSE coarse+fine, clip, Adam) on an n-ray
    batch through a Blender-style camera: one warm-up step on 128 rays, then the median of `steps` steps.
    Threads = the host CPU share this process is given (OMP_NUM_THREADS on the GPU box: 16 of the machine's CPUs).
    BASELINE.md §3 asks for torch.set_num_threads(os.cpu_count()): that leg runs beside it as `all_cores` on a
    smaller sample (512 rays, median of <= 3 steps, ~30 s budget) — on the GPU box os.cpu_count() reports the whole
    machine, more threads than this process's share (affinity / cgroup quota are reported with it)."""
    threads = _baseline_threads(world)
    med, times = _oracle_step_rate(S, NI, n, steps, threads)
    rec = {"value": round(n / med, 2), "unit": "rays/s", "cores": threads, "kind": "port",
           "sample": f"median of {steps} oracle train steps x {n} rays (64+128, 2 nets, fp32, MSE coarse+fine, "
                     f"clip, Adam): {med:.2f} s/step (steps {', '.join(f'{t:.2f}' for t in times)} s)",
           "cpu_model": _cpu_model(), "torch_threads": torch.get_num_threads(), **_cpu_share()}
    if world > 1:
        rec["note"] = (f"rank 0 of {world}, after every GPU leg, with the other ranks blocked in a gloo barrier; the "
                       "same bounded sample as at N = 1")
    allc = os.cpu_count() or 1
    quota = rec.get("cgroup_cpu_quota")
    if allc != threads and quota is not None and quota < allc:
        # measured on the GPU box (round 3): 256 threads on a 16-CPU cgroup quota ran 512 rays in 68.7 s/step
        # (7.45 rays/s) — oversubscribing the share 16x measures the scheduler, not the reference path
        rec["all_cores"] = {"value": None, "cores": allc,
                            "skipped": f"this process's cgroup CPU quota is {quota} CPUs of os.cpu_count()={allc}: "
                                       f"torch.set_num_threads({allc}) would oversubscribe the share "
                                       f"{allc / max(quota, 1e-9):.0f}x (measured once, round 3: 7.45 rays/s on 512 "
                                       "rays, 68.7 s/step); the baseline above uses the whole quota"}
    elif allc != threads:
        n2 = min(n, 512)
        progress(f"cpu baseline: all-cores leg, {n2} rays at {allc} threads")
        med2, times2 = _oracle_step_rate(S, NI, n2, 3, allc, budget_s=30.0)
        rec["all_cores"] = {"value": round(n2 / med2, 2), "unit": "rays/s", "cores": allc,
                            "torch_threads": torch.get_num_threads(),
                            "sample": f"median of {len(times2)} oracle train steps x {n2} rays at "
                                      f"torch.set_num_threads(os.cpu_count()={allc}) (BASELINE.md §3): "
                                      f"{', '.join(f'{t:.2f}' for t in times2)} s"}
        torch.set_num_threads(threads)
    return rec


def dropin_run(rb, dev, a, world, rank, n_local, precision="fp32", amp_dtype=torch.float16):
    """The reference loop body (runtime_adapt.py:286-310) on the drop-in surface: HierarchicalNeRF (coarse +
    fine VanillaNeRF, autograd through the HIP MLP / compositing / sampling ops) -> compute_mse_loss (coarse +
    fine terms) -> backward -> clip_grad_norm_(1.0) -> torch.optim.Adam ('sigma' / 'color' groups).  precision
    "bf16" runs it as the reference's use_amp=True body (configs/train.json): autocast(fp16) around the loss ->
    GradScaler scale / unscale_ / step / update; the expert then dispatches to the fp16 build of the fused MLP kernels
    (vanilla.amp_precision), beside the bf16 C3 engine.  Adam is torch's fused implementation (no host sync inside GradScaler.step; foreach
    if this torch build lacks it).  The ray batch comes from images resident in HBM (the reference's DataLoader +
    .to(device) is not timed).  amp_dtype=torch.bfloat16 (tools/amp_kernels_ab.py only) runs the same body under
    autocast(bfloat16), i.e. on the bf16 build of the kernels."""
    from types import SimpleNamespace
    from nerf_amd.losses import compute_mse_loss
    from nerf_amd.vanilla import HierarchicalNeRF
    torch.manual_seed(0)
    model = HierarchicalNeRF().to(dev).train()
    grp = model.get_param_groups()
    groups = [{"params": grp["sigma"]["params"], "lr": 2e-3}, {"params": grp["color"]["params"], "lr": 2e-3}]
    try:
        opt, kind = torch.optim.Adam(groups, fused=True), "torch.optim.Adam(fused=True)"
    except (RuntimeError, ValueError):
        opt, kind = torch.optim.Adam(groups, foreach=True), "torch.optim.Adam(foreach=True)"
    use_amp = precision == "bf16"
    scaler = torch.amp.GradScaler("cuda", enabled=use_amp)
    P = SimpleNamespace(ray_samples=a.samples, n_importance=a.importance, chunk_points=1 << 22, color_space="linear")

    def one(step):
        rays, gt = _batch(rb, a, step, rank, world, n_local)
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=amp_dtype, enabled=use_amp):
            loss = compute_mse_loss(P, model, {"rays": rays, "rgbs": gt})
        scaler.scale(loss).backward()
        scaler.unscale_(opt)
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        scaler.step(opt)
        scaler.update()
        return loss

    for s in range(a.warmup):
        one(s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(a.warmup, a.warmup + a.steps):
        loss = one(s)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    rec = {"value": round(n_local * a.steps / el, 1), "unit": "rays/s", "ms_per_step": round(el / a.steps * 1e3, 3),
           "final_loss": round(float(loss.item()), 6), "optimizer": kind,
           "path": "render_rays + HierarchicalNeRF(VanillaNeRF x2) autograd + compute_mse_loss + "
                   "clip_grad_norm_ + " + kind + " (runtime_adapt.py:286-310)"}
    if use_amp:
        rec["amp"] = ("torch.autocast(fp16) -> the fp16 build of the fused MLP kernels (the reference's autocast "
                      "rounding points) + fp32 compositing; GradScaler scale "
                      f"{scaler.get_scale():.0f} after {a.warmup + a.steps} steps (halves on any inf)")
    return rec


def _batch(rb, a, step, rank, world, n_local):
    from nerf_amd.dp import shard_seed
    if a.strong:   # one global draw per step, rank-strided slice
        return rb.batch(a.batch, seed=step, shard=(rank, world))
    return rb.batch(n_local, seed=shard_seed(step, rank, world))  # disjoint per-rank streams


def _traffic(bf16, key, split=False):
    tpath = os.path.join(ROOT, "profiles", "traffic_bf16.json" if bf16 else
                         ("traffic_split.json" if split else "traffic.json"))
    if os.path.exists(tpath):
        try:
            return json.load(open(tpath)).get(key)
        except Exception:
            return None
    return None


def roofline_bf16(tm):
    """bf16 (configs[2]): the MLP runs as ONE fused forward launch (mlp_bf16_fused.hpp; events 0 -> 1 bracket it) and,
    per trunk layer, ONE fused backward launch (mlp_bf16_bwd.hpp: input + weight gradient; events 4i -> 4i+1).
    Both are HBM-bound; the reported kernel is the class with the largest TOTAL time per step (launch mean x
    launches per step), the other is listed beside it.
    Algorithmic bytes per sample row:
      fused_bwd_layer  G (dZ_i) 512 B read + X_i 512 B read + dZ_{i-1} 512 B written = 1,536 B
                       (+ the split-M weight-gradient slabs, S x 256 KiB per launch, listed as slab_bytes)
      fused_fwd        encoding + colour-input prefill 256 B read; saved activations 7 x 512 + trunk.3 512 B,
                       colour input 128 B, colour layer 0 256 B, sigma / colour-out pre-activations 20 B,
                       rgb_sigma 16 B written = 4,772 B (the fused backward takes its ReLU masks from the saved
                       activations: no bitmask words are written)"""
    M = tm["M"]
    mean = lambda xs: sum(xs) / len(xs)
    bwd_ms = mean([st[i] for st in tm["wgrad"] for i in K256])
    fwd_ms = mean([st[0] for st in tm["fwd"]])
    S = min(256, max(1, (M + 255) // 256 * 256 // 2048))
    cls = {
        "fused_bwd_layer": {"kernel": "bwd_layer_bf16 (fused input + weight gradient of one 256x256 trunk layer)",
                            "mean_launch_ms": bwd_ms, "launches": len(K256), "bytes": 1536.0 * M,
                            "slab_bytes": S * 256 * 256 * 4.0, "flop": 2 * 2.0 * M * 256 * 256},
        "fused_fwd": {"kernel": "mlp_fwd_fused_bf16 (whole MLP forward, one persistent launch)",
                      "mean_launch_ms": fwd_ms, "launches": 1, "bytes": 4772.0 * M, "flop": 2.0 * MAC_PER_EVAL * M},
    }
    for k, c in cls.items():
        ms = c["mean_launch_ms"]
        c["achieved_gbs"] = round(c["bytes"] / (ms * 1e-3) / 1e9, 1)
        c["hbm_frac"] = round(c["bytes"] / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        c["mfma_tflops"] = round(c["flop"] / (ms * 1e-3) / 1e12, 1)
        c["mfma_frac_bf16"] = round(c["flop"] / (ms * 1e-3) / 1e12 / BF16_MFMA_PEAK_TFLOPS, 4)
        c["ms_per_step"] = round(ms * c["launches"], 4)
        c["mean_launch_ms"] = round(ms, 4)
    dom = max(cls, key=lambda k: cls[k]["ms_per_step"])
    d = cls[dom]
    return {"bound": "hbm", "kernel": f"{d['kernel']}, fine net M={M}", "achieved": d["achieved_gbs"],
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": d["hbm_frac"], "bytes_per_launch": d["bytes"],
            "traffic": _traffic(True, dom), "class": dom, "mean_launch_ms": d["mean_launch_ms"],
            "classes": cls, "rule": "largest total time per step (mean launch x launches) among the fused MLP kernels"}


X6_PRODUCTS = 6  # bf16 piece products per fp32 product in the split GEMMs (nerf-sys_amd/csrc/gemm_x6.hpp)


def roofline(tm, bf16, overlap, bf16_flags=0, split=False):
    """fp32 native: the fine net's 256x256 trunk GEMMs on the fp32 MFMA (peak 157.3 TFLOP/s).  fp32 split (``split`` =
    the trainer's fp32_gemm, "split" by default): the forward and weight-gradient GEMMs run X6_PRODUCTS bf16 MFMA
    products per fp32 product, so their matrix-core work per launch is 6 x 2*M*256*256 bf16 FLOP against the dense
    bf16 peak (fp32-equivalent rate listed beside it); split == "native_dgrad" keeps the input gradients on the fp32
    MFMA."""
    if bf16 and not bf16_flags:
        return roofline_bf16(tm)
    M = tm["M"]
    mean = lambda xs: sum(xs) / len(xs)
    flop256 = 2.0 * M * 256 * 256
    cls = {
        "fwd": mean([st[i] for st in tm["fwd"] for i in K256]),
        "wgrad": mean([st[i] for st in tm["wgrad"] for i in K256]),
        "dgrad": mean([st[i - 1] for st in tm["dgrad"] for i in K256]),
    }
    eligible = [k for k in cls if not (overlap and k == "fwd")]
    dom = max(eligible, key=lambda k: cls[k])
    ms = cls[dom]
    ach = flop256 / (ms * 1e-3) / 1e12
    if bf16:  # the layered bf16 path (--bf16-flags A/B runs)
        names = {"fwd": "gemm_nt_bf16 fwd", "wgrad": "gemm_wgrad_bf16", "dgrad": "gemm_nt_bf16 dgrad"}
        kern = f"{names[dom]}, fine net M={M}: trunk 256x256 layers {K256}"
        # bf16 layers are HBM-bound: algorithmic bytes per launch per sample row = bf16 rows in (256 * 2 B) +
        # bf16 rows out (256 * 2 B) [+ the 32-B ReLU bitmask word row of dgrad]; wgrad reads two bf16 rows
        row = {"fwd": 256 * 2 + 256 * 2 + 32, "dgrad": 256 * 2 + 256 * 2 + 32, "wgrad": 256 * 2 + 256 * 2}[dom]
        by = M * float(row)
        ach_gbs = by / (ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "kernel": kern, "achieved": round(ach_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach_gbs / HBM_PEAK_GBS, 4), "bytes_per_launch": by, "mfma_tflops": round(ach, 1),
                "mfma_frac_bf16": round(ach / BF16_MFMA_PEAK_TFLOPS, 4)}
        peak_c = {k: BF16_MFMA_PEAK_TFLOPS for k in cls}
        split_cls = set()
    else:
        split_cls = set() if not split else ({"fwd", "wgrad"} if split == "native_dgrad" else {"fwd", "wgrad", "dgrad"})
        names = {"fwd": "gemm_nt16 fwd (fp32 16x16x4, bias+ReLU)", "wgrad": "gemm_wgrad (fp32 32x32x2, split-M)",
                 "dgrad": "gemm_nt16 dgrad (fp32 16x16x4, ReLU mask)"}
        nt_f, nt_d = "gemm_nt_x6w fwd (fp32 as 6 bf16 split products, 512x128 tiles, bias+ReLU)", \
            "gemm_nt_x6w<BIGSMALL, 32-row waves> dgrad (fp32 as 6 bf16 split products, small-term accumulators, 256x128 tiles)"
        if "fwd" in split_cls:
            names["fwd"] = nt_f
        if "wgrad" in split_cls:
            names["wgrad"] = "gemm_wgrad_x6w (fp32 as 6 bf16 split products, one 512-thread workgroup per split)"
        if "dgrad" in split_cls:
            names["dgrad"] = nt_d
        kern = f"{names[dom]}, fine net M={M}: trunk 256x256 layers {K256}"
        peak_c = {k: (BF16_MFMA_PEAK_TFLOPS / X6_PRODUCTS if k in split_cls else FP32_MFMA_PEAK_TFLOPS) for k in cls}
        if dom in split_cls:
            roof = {"bound": "mfma", "kernel": kern, "achieved": round(X6_PRODUCTS * ach, 1),
                    "peak": BF16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(X6_PRODUCTS * ach / BF16_MFMA_PEAK_TFLOPS, 4),
                    "flop_per_launch": X6_PRODUCTS * flop256, "fp32_flop_per_launch": flop256,
                    "fp32_equiv_tflops": round(ach, 2),
                    "fp32_equiv_frac_of_fp32_peak": round(ach / FP32_MFMA_PEAK_TFLOPS, 4),
                    # the split method's own ceiling: the dense bf16 peak over 6 products per fp32 product (= `frac`)
                    "split_ceiling_fp32_equiv_tflops": round(BF16_MFMA_PEAK_TFLOPS / X6_PRODUCTS, 1),
                    "fp32_equiv_frac_of_split_ceiling": round(ach / (BF16_MFMA_PEAK_TFLOPS / X6_PRODUCTS), 4)}
        else:
            roof = {"bound": "mfma", "kernel": kern, "achieved": round(ach, 2), "peak": FP32_MFMA_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 4), "flop_per_launch": flop256}
    roof.update({"traffic": _traffic(bf16, dom, dom in split_cls), "class": dom, "mean_launch_ms": round(ms, 4),
                 "classes_ms": {k: round(v, 4) for k, v in cls.items()},
                 "classes_frac": {k: round(flop256 / (v * 1e-3) / 1e12 / peak_c[k], 4) for k, v in cls.items()},
                 "classes_engine": {k: ("split x6" if k in split_cls else ("bf16" if bf16 else "fp32 MFMA"))
                                    for k in cls},
                 "rule": "largest mean launch time among classes that run alone" +
                         (" (fine fwd overlaps the coarse backward: excluded)" if overlap else "")})
    return roof


def engine_run(a, dev, rb, world, rank, n_local, precision, barrier, nccl, fp32_gemm=None):
    """The fused train step (NeRFTrainer) timed over a.steps after a.warmup: value, ms/step, the live-event roofline,
    and (N > 1) the per-rank exchange diagnostics.  Returns (record, trainer, (coarse, fine))."""
    from nerf_amd.trainer import NeRFTrainer
    from nerf_amd.vanilla import VanillaNeRF
    torch.manual_seed(0)   # the same initial weights for every precision (the PSNR comparison starts from them)
    coarse, fine = VanillaNeRF().to(dev), VanillaNeRF().to(dev)
    tr = NeRFTrainer(coarse, fine, n_samples=a.samples, n_importance=a.importance, world_size=world, device=dev,
                     overlap=not a.no_overlap, overlap_with=getattr(a, "overlap_with", "bwd"), precision=precision,
                     bf16_flags=a.bf16_flags if precision == "bf16" else 0, split_wgrad=a.split_wgrad,
                     fp32_gemm=fp32_gemm or a.fp32_gemm)

    def one(step):
        rays, gt = _batch(rb, a, step, rank, world, n_local)
        return tr.step(rays, gt, seed=step * world + rank)

    for s in range(a.warmup):
        loss = one(s)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(a.warmup, a.warmup + a.steps):
        loss = one(s)
    barrier()
    torch.cuda.synchronize()
    el_local = time.perf_counter() - t0
    # the roofline pass: timing_steps more steps (outside the timed region) with every launch alone on the device —
    # the coarse backward back on the main stream, the fine weight gradients back in line — and HIP events around the
    # fine net's trunk GEMMs, so each kernel class's mean launch time is its own (the production step runs them
    # concurrently on three streams, where a launch's wall time is shared)
    n_ev = max(1, a.timing_steps)
    conc = (tr.overlap, tr.split_wgrad)
    tr.overlap, tr.split_wgrad = False, False
    tr.enable_timing(n_ev, skip=0)
    for s in range(a.warmup + a.steps, a.warmup + a.steps + n_ev):
        one(s)
    torch.cuda.synchronize()
    tr.overlap, tr.split_wgrad = conc
    tm = tr.collect_timing()
    el = el_local
    dp = None
    if world > 1:
        # the exchange as it runs in production: a.timing_steps more steps with the side stream on and events around the
        # two buckets only (bucket 0 = coarse gradient on the side stream, bucket 1 = fine gradient + loss); the kernel
        # pass above ran without the side stream, i.e. with ONE all-reduce of the whole buffer (reported beside it)
        single = [x[0] for x in (tm.get("allreduce") or []) if x]
        saved = _snapshot(tr)   # a timing device: the trainer leaves it in the state it entered it
        tr.enable_exchange_timing(n_ev)
        for s in range(a.warmup + a.steps + n_ev, a.warmup + a.steps + 2 * n_ev):
            one(s)
        torch.cuda.synchronize()
        _restore(tr, saved)
        ex = tr.collect_exchange_timing()
        ar_mean = [sum(x[b] for x in ex if x[b] is not None) / max(1, sum(x[b] is not None for x in ex)) for b in range(2)]
        single_mean = sum(single) / len(single) if single else 0.0
        mine = torch.tensor([el_local] + ar_mean + [single_mean], dtype=torch.float64, device=dev)
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        rows = [x.tolist() for x in allr]
        el = max(r[0] for r in rows)
        dp = {"world_size": dist.get_world_size(), "backend": "nccl (RCCL)" if nccl else "gloo (rehearsal)",
              "step_ms_max": round(el / a.steps * 1e3, 3), "step_ms_min": round(min(r[0] for r in rows) / a.steps * 1e3, 3),
              "allreduce_ms_per_rank": [[round(r[1], 4), round(r[2], 4)] for r in rows],
              "allreduce_single_bucket_ms_per_rank": [round(r[3], 4) for r in rows],
              "allreduce_note": "HIP events on the consuming stream around each bucket's all_reduce (issued "
                                "async_op=True, end event after work.wait() on that stream), in timing_steps extra "
                                "production-form steps: [bucket 1 = coarse net gradient, issued on the side stream right "
                                "after the coarse backward; bucket 2 = fine gradient + loss, after the fine backward], "
                                "mean over the steps, including the wait for the slowest rank; "
                                "allreduce_single_bucket_ms_per_rank: the kernel-timing pass (no side stream), one "
                                "all-reduce of the whole buffer",
              "bytes_per_step": int(tr.gbuf.numel() * 4)}
        dp.update(params_checksum(tr.params, world))
        dp.update(exposed_exchange(a, tr, one, dev, world, barrier, el / a.steps * 1e3))
    rec = {"value": round(n_local * world * a.steps / el, 1), "ms_per_step": round(el / a.steps * 1e3, 3),
           "final_loss": round(float(loss.item()), 6),
           "roofline": dict(roofline(tm, precision == "bf16", False, tr.bf16_flags,
                                     split=(tr.fp32_gemm if precision == "fp32" and tr.fp32_gemm != "native"
                                            else False)), event_steps=n_ev,
                            event_pass="the timing_steps steps after the timed region, every launch alone (no "
                                       "side-stream coarse backward, fine weight gradients in line)"),
           "streams": {"coarse_bwd_beside_fine_fwd": tr.overlap and tr.overlap_with == "fwd",
                       "coarse_bwd_beside_fine_bwd": tr.overlap and tr.overlap_with == "bwd", "fine_wgrad_stream": tr.split_wgrad}}
    if precision == "fp32":
        rec["fp32_gemm"] = tr.fp32_gemm
    peak = BF16_MFMA_PEAK_TFLOPS if precision == "bf16" else FP32_MFMA_PEAK_TFLOPS
    rec["step_mfma_frac"] = round(rec["value"] * FLOP_PER_RAY / world / 1e12 / peak, 4)
    if precision == "fp32" and tr.fp32_gemm != "native":  # most of the trunk's fp32 FLOPs ran as 6 bf16 products
        rec["step_mfma_frac_note"] = ("fp32 FLOPs of the step / fp32 MFMA peak (157.3 TFLOP/s); the split GEMMs execute "
                                      "them on the bf16 matrix cores, so a value above 1 is possible")
    if dp:
        rec["dp"] = dp
    return rec, tr, (coarse, fine)


def _snapshot(tr):
    return [x.detach().clone() for x in (tr.params, tr.m, tr.v)], tr.step_count


def _restore(tr, saved):
    with torch.no_grad():
        for x, y in zip((tr.params, tr.m, tr.v), saved[0]):
            x.copy_(y)
    tr.step_count = saved[1]


def exposed_exchange(a, tr, one, dev, world, barrier, step_ms):
    """The exchange's exposed cost, measured rather than inferred from events: after the checksum, the same step runs
    a.steps more times with the all-reduces skipped (tr.exchange_enabled = False: every rank applies its own
    gradient), timed like the main region (barrier + synchronize, max over ranks); exposed = step time with the
    exchange - step time without it.  The trainer's parameters / moments are restored afterwards."""
    saved = _snapshot(tr)
    tr.exchange_enabled = False
    s0 = a.warmup + a.steps + 2 * max(1, a.timing_steps)   # seeds after the kernel- and exchange-timing passes
    try:
        one(s0)
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s in range(s0 + 1, s0 + 1 + a.steps):
            one(s)
        barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    finally:
        tr.exchange_enabled = True
        _restore(tr, saved)
    mine = torch.tensor([el], dtype=torch.float64, device=dev)
    allr = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allr, mine)
    no_x = max(float(r.item()) for r in allr) / a.steps * 1e3
    return {"step_ms_no_exchange": round(no_x, 3), "exposed_exchange_ms": round(step_ms - no_x, 3),
            "exposed_exchange_note": "step time (max over ranks) with the two all-reduce buckets minus the same "
                                     "steps with the all-reduces skipped, both timed over --steps steps"}


def params_checksum(params, world):
    from nerf_amd.dp import params_checksum as pc
    return pc(params, world)


def llff_run(a, dev, world, rank, barrier, nccl):
    """BASELINE configs[3] (C4): the Fern-style 1008x756 forward-facing scene with NDC rays (synthetic, 20 views), the
    same fp32 engine step (64 + 128, two nets) over a.llff_steps timed steps; data parallel at N > 1 as the headline."""
    from types import SimpleNamespace
    from nerf_amd.scene import make_llff_scene
    from nerf_amd.trainer import RayBatcher
    torch.manual_seed(0)
    scene = make_llff_scene(n_train=20, n_test=1, seed=0, device=dev)
    rb = RayBatcher(scene, dev)
    b = SimpleNamespace(**{**vars(a), "steps": a.llff_steps, "timing_steps": 1})
    n_local = a.batch // world if a.strong else a.batch
    rec, _, _ = engine_run(b, dev, rb, world, rank, n_local, "fp32", barrier, nccl)
    out = {"config": "configs[3]: Fern-style 1008x756 forward-facing, NDC rays (near plane 1, t in [0,1]), 64+128, "
                     "2 x (8x256 MLP), fp32 engine (synthetic analytic scene, 20 views; LLFF data is not in the image)",
           "value": rec["value"], "unit": "rays/s", "ms_per_step": rec["ms_per_step"], "steps": b.steps,
           "n_gpus": world, "step_mfma_frac": rec["step_mfma_frac"], "final_loss": rec["final_loss"],
           "roofline_class_ms": rec["roofline"].get("classes_ms")}
    if rec.get("dp"):
        out["dp"] = {k: rec["dp"][k] for k in ("world_size", "step_ms_max", "step_ms_min", "params_equal_across_ranks")}
    return out


def sweep_run(a, dev, world, rank):
    """BASELINE configs[4] (C5): a.sweep_scenes seeded Lego-style scenes (800x800, a.sweep_views training views, 2 held-out),
    each trained independently by the bf16 engine for a.sweep_steps 4096-ray steps (64 + 128, lr 2e-3); rank r trains
    scenes r, r+N, ... (no collective on the data path), results all-gathered once.  Aggregate rays/s = sum over GPUs
    of each GPU's rays / its training time, against the bf16 MFMA roofline; mean held-out PSNR after a.sweep_steps."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import sweep_scenes
    res = []
    for sid in range(rank, a.sweep_scenes, world):
        r = sweep_scenes.train_scene(sid, steps=a.sweep_steps, batch=a.batch, train_views=a.sweep_views, test_views=2,
                                     precision="bf16", lr=2e-3, dev=dev)
        r.pop("losses", None)
        r["rank"] = rank
        res.append(r)
        progress(f"sweep: scene {sid} psnr {r['psnr']} at {r['rays_per_s']} rays/s")
        torch.cuda.empty_cache()
    if world > 1:
        allr = [None] * world
        dist.all_gather_object(allr, res)
        res = [r for rr in allr for r in rr]
    summ = sweep_scenes.summarize(res, a.batch, "bf16", world)
    summ.update({"steps_per_scene": a.sweep_steps, "train_views": a.sweep_views, "test_views": 2,
                 "per_scene": [{k: r[k] for k in ("scene_seed", "psnr", "rays_per_s", "loss", "rank")} for r in res]})
    return summ


def production_runs(a, dev, rank=0, world=1):
    """the reference's production path — its default expert is Instant-NGP (common/args.py:56-58) with
    occupancy marching (models/inr/meta_ngp.py:389-443, nerfs/ray_rendering.py:494-558) inside the MoE container
    (models/inr/meta_container.py:275-343).  The ngp and container sub-records time their train steps (inputs resident
    in HBM), each with its dominant kernel against its own roofline and the CPU oracle beside it."""
    from types import SimpleNamespace
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    out = {}
    cpu = dict(cpu_seconds=a.prod_cpu_seconds, no_cpu_baseline=a.no_cpu_baseline)
    if not a.no_ngp and world == 1:   # the single-expert NGP step has no gradient exchange of its own
        import bench_ngp
        progress("ngp (Instant-NGP expert) leg")
        out["ngp"] = bench_ngp.run(SimpleNamespace(steps=20, warmup=5, batch=4096, samples=96, train_views=100, **cpu),
                                   dev)
        torch.cuda.empty_cache()
    if not a.no_container:
        import bench_container
        progress("container (MoE: 4 NGP experts + occupancy + bg MLP) leg")
        out["container"] = bench_container.run(
            SimpleNamespace(steps=a.container_steps, warmup=a.container_warmup, batch=4096, train_views=a.train_views,
                            shard=False, no_bucket=False, **cpu), dev, rank, world)
        torch.cuda.empty_cache()
    return out


def psnr_run(a, rb, scene, runs, rank, world, n_local):
    """The metric's PSNR half (runtime_adapt.py:150-157): every engine trainer in ``runs`` (precision -> (trainer,
    (coarse, fine)), all started from the same seed-0 weights and fed the same batches) continues to a.psnr_steps
    total steps, then renders every held-out 800x800 view (64 + 128, fp32 compositing) — outside the timed region."""
    from nerf_amd.losses import image_psnr
    from nerf_amd.ray_rendering import render_image
    fx, fy, cx, cy = scene.intrinsics
    out = {}
    replicas = {}
    for prec, (tr, (coarse, fine)) in runs.items():
        done = tr.step_count
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        progress(f"psnr: training the {prec} engine from step {done} to {a.psnr_steps}")
        for s in range(done, a.psnr_steps):
            rays, gt = _batch(rb, a, s, rank, world, n_local)
            tr.step(rays, gt, seed=s * world + rank)
            if (s + 1) % 250 == 0:
                torch.cuda.synchronize()
                progress(f"psnr: {prec} step {s + 1}/{a.psnr_steps}")
        torch.cuda.synchronize()
        train_s = time.perf_counter() - t0
        if world > 1:   # data parallel: every rank trained this replica; rank 0 renders it (the others are equal)
            chk = params_checksum(tr.params, world)
            replicas[prec] = chk["params_equal_across_ranks"]
            if rank != 0:
                continue
        tr.sync_to_modules()
        coarse.eval(), fine.eval()
        ps = []
        for v in range(scene.test_poses.shape[0]):
            img, _, _ = render_image(coarse, H=scene.H, W=scene.W, fx=fx, fy=fy, cx=cx, cy=cy, c2w=scene.test_poses[v],
                                     near=scene.near, far=scene.far, ray_samples=a.samples, n_importance=a.importance,
                                     fine_model=fine, ndc=(scene.focal, 1.0) if scene.ndc else None)
            ps.append(image_psnr(img, scene.test_images[v], "linear"))
        coarse.train(), fine.train()
        out[prec] = {"psnr": round(sum(ps) / len(ps), 3), "per_view": [round(p, 3) for p in ps],
                     "steps": tr.step_count, "train_s_after_timed": round(train_s, 2)}
    if rank != 0:
        return None
    rec = {"steps": a.psnr_steps, "views": int(scene.test_poses.shape[0]), "image": f"{scene.W}x{scene.H}",
           "samples": [a.samples, a.importance], "n_gpus": world, "global_batch": n_local * world, **out,
           "protocol": "engine trainers from the same seed-0 weights and the same 4096-ray batches / jitter seeds, "
                       "trained to `steps` total steps (the timed steps included), then full-image PSNR of each "
                       "held-out view in linear colour space (runtime_adapt.py:150-157), averaged"}
    if "fp32" in out and "bf16" in out:
        rec["bf16_minus_fp32_db"] = round(out["bf16"]["psnr"] - out["fp32"]["psnr"], 3)
    if world > 1:
        rec["params_equal_across_ranks"] = replicas
        rec["dp_note"] = (f"{world} ranks trained each replica data parallel (global batch {n_local * world} rays per "
                          "step, one gradient all-reduce per step); rank 0 rendered the held-out views after an "
                          "all-gathered checksum of every rank's parameters")
    return rec


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}")
    nccl = a.dist_backend == "nccl"
    dev = torch.device("cuda", local if nccl else local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    if world > 1:
        if nccl:
            dist.init_process_group("nccl", device_id=dev)  # RCCL on ROCm
        else:
            dist.init_process_group("gloo")

    cpu_group = None
    if world > 1:   # a host-side group for the final wait (rank 0's CPU baseline runs for ~1-2 minutes)
        import datetime
        cpu_group = dist.new_group(backend="gloo", timeout=datetime.timedelta(minutes=30)) if nccl else None

    def barrier():
        if world > 1:
            dist.barrier(device_ids=[dev.index]) if nccl else dist.barrier()

    if a.path == "dropin" and world > 1:
        raise SystemExit("--path dropin runs on one GPU (the reference loop body has no gradient exchange)")
    if a.strong and a.batch % world:
        raise SystemExit("--strong needs --batch divisible by the number of GPUs")
    n_local = a.batch // world if a.strong else a.batch

    from nerf_amd.scene import make_blender_scene, make_llff_scene
    from nerf_amd.trainer import RayBatcher

    torch.manual_seed(0)
    n_test = 1 if a.no_psnr else a.psnr_views
    if a.scene == "llff":
        scene = make_llff_scene(n_train=min(a.train_views, 20), n_test=n_test, seed=0, device=dev)
    else:
        scene = make_blender_scene(n_train=a.train_views, n_test=n_test, H=800, W=800, seed=0, device=dev)
    rb = RayBatcher(scene, dev)
    bf16 = a.precision == "bf16"
    other = "fp32" if bf16 else "bf16"

    runs = {}
    engine = None
    progress(f"rank {rank}/{world}: scene ready")
    if a.path == "engine" or world == 1:
        engine, tr, nets = engine_run(a, dev, rb, world, rank, n_local, a.precision, barrier, nccl)
        runs[a.precision] = (tr, nets)
    drop = None
    if world == 1 and (a.path == "dropin" or not a.no_dropin):
        drop = dropin_run(rb, dev, a, world, rank, n_local, a.precision)
    sub = None
    if not a.no_other_precision and a.path == "engine":
        sub, tr2, nets2 = engine_run(a, dev, rb, world, rank, n_local, other, barrier, nccl)
        runs[other] = (tr2, nets2)
        if world == 1 and not a.no_dropin:
            sub["dropin"] = dropin_run(rb, dev, a, world, rank, n_local, other)
            sub["dropin_vs_engine"] = round(sub["dropin"]["value"] / sub["value"], 4)

    native = None
    if (world == 1 and a.path == "engine" and not bf16 and a.fp32_gemm != "native" and not a.no_native_ref):
        native, _, _ = engine_run(a, dev, rb, world, rank, n_local, "fp32", barrier, nccl, fp32_gemm="native")
    main_res = drop if a.path == "dropin" else engine
    value = main_res["value"]
    out = {
        "metric": METRIC, "value": value, "unit": "rays/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": main_res["ms_per_step"], "higher_is_better": True,
        "scaling": "strong" if a.strong else "weak", "vs_baseline": None, "dtype": "bf16" if bf16 else "f32",
        "data": "synthetic",
        "config": {"workload": ("Fern-style 1008x756 forward-facing NDC (synthetic analytic scene, 20 views)"
                                if a.scene == "llff" else "Lego-style 800x800 (synthetic analytic scene, 100 views)") +
                               ", 64 coarse + 128 fine hierarchical, 2 x (8x256 MLP), " +
                               ("bf16 MLP + fp32 compositing" if bf16 else "fp32") +
                               ", train step incl. ray gen + Adam" +
                               (" [drop-in render_rays/autograd path]" if a.path == "dropin" else " [fused engine]"),
                   "global_batch": a.batch if a.strong else a.batch * world, "rays_per_gpu": n_local,
                   "samples": [a.samples, a.importance], "parallelism": f"dp{world}", "precision": a.precision,
                   "path": a.path, "fp32_gemm": None if bf16 else a.fp32_gemm},
        "rccl_ranks": world, "backend": ("nccl (RCCL)" if nccl else "gloo (rehearsal)") if world > 1 else None,
        "roofline": engine["roofline"] if engine else None,
        "step_mfma_frac": round(value * FLOP_PER_RAY / world / 1e12 /
                                (BF16_MFMA_PEAK_TFLOPS if bf16 else FP32_MFMA_PEAK_TFLOPS), 4),
        "final_loss": main_res["final_loss"],
    }
    if engine and engine.get("dp"):
        out["dp"] = engine["dp"]
    if a.path == "dropin" and engine:
        out["engine"] = {k: engine[k] for k in ("value", "ms_per_step")}
    elif drop:
        out["dropin"] = drop
    if drop and engine:
        out["dropin_vs_engine"] = round(drop["value"] / engine["value"], 4)
    if sub:
        out[other] = sub
    if native:
        out["fp32_native_gemm"] = {k: native[k] for k in ("value", "ms_per_step", "final_loss", "step_mfma_frac")}
        out["fp32_native_gemm"]["roofline_classes_ms"] = native["roofline"].get("classes_ms")
    if not a.no_llff and a.scene == "blender" and a.path == "engine":
        progress("C4 (llff) leg")
        out["llff"] = llff_run(a, dev, world, rank, barrier, nccl)
    progress("timed legs done")
    if not a.no_psnr and runs:
        ps = psnr_run(a, rb, scene, runs, rank, world, n_local)
        if rank == 0:
            out["psnr"] = ps
    if not a.no_sweep and a.scene == "blender" and a.path == "engine":
        progress("C5 (8-scene sweep) leg")
        sw = sweep_run(a, dev, world, rank)
        if rank == 0:
            out["sweep"] = sw
    if a.path == "engine" and a.scene == "blender":
        prod = production_runs(a, dev, rank, world)
        if rank == 0:
            out.update(prod)
    # the CPU baseline on rank 0 after every GPU leg; at N > 1 the other ranks wait in a gloo barrier (blocked in a
    # socket read, not spinning on a core beside the baseline's threads)
    if rank == 0 and not a.no_cpu_baseline:
        progress("cpu baseline leg")
        out["cpu_baseline"] = cpu_baseline(a.samples, a.importance, a.cpu_batch, a.cpu_steps, world)
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        cpu_group.barrier() if cpu_group is not None else barrier()  # everyone waits for rank 0's report
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
