#!/usr/bin/env python3
"""Bench of the data path (SURVEY.md §8f row 4 — not the headline metric of bench.py): RamRaysDataset's ray
build (data/ram_rays_dataset.py:46-121) for a Blender-style scene, 100 posed 800x800 views (hemisphere poses,
radius 4.0311, focal 1111.1), scene box [-1.5, 1.5]^3 (AABB near/far), near/far override (2, 6), a random
keep mask on every second view.

value = rays/s of the whole GPU dataset build with the decoded uint8 images already resident in HBM (count
pass + scan + write pass, timed with HIP events on the launch stream); the end-to-end constructor time
(host stacking + H2D upload included) is reported beside it. Roofline of the dominant kernel against HBM.
cpu_baseline: the oracle's _process_single_image restatement on a bounded sample of views.

  python tools/bench_data.py [--views 100] [--reps 5]
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nerf-sys_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0
BOX = torch.tensor([[-1.5, -1.5, -1.5], [1.5, 1.5, 1.5]])


class MD:
    """ImageMetadata surface over in-memory arrays (image_metadata.py:41-121)."""

    def __init__(self, i, c2w, K, img, mask):
        self.H, self.W = img.shape[:2]
        self.c2w, self.intrinsics, self.image_index, self.is_val = c2w, K, i, False
        self._img, self._mask = img, mask

    def load_image(self):
        return self._img

    def load_mask(self):
        return self._mask


def scene(views, H=800, W=800):
    from nerf_amd.scene import hemisphere_poses
    focal = 0.5 * W / math.tan(0.5 * 0.6911112)
    poses = hemisphere_poses(views, seed=0)
    g = torch.Generator().manual_seed(0)
    mds = []
    for i in range(views):
        img = torch.randint(0, 256, (H, W, 3), generator=g, dtype=torch.uint8)
        mask = (torch.rand(H, W, generator=g) > 0.25) if i % 2 else None
        mds.append(MD(i, poses[i][:3, :4].float(), torch.tensor([focal, focal, W / 2, H / 2]), img, mask))
    return mds


def cpu_baseline(mds, seconds):
    from oracle import meta_oracle as MO
    torch.set_num_threads(min(16, os.cpu_count() or 1))  # the box's CPU share
    MO.process_single_image(mds[0]._img, mds[0]._mask, mds[0].H, mds[0].W, mds[0].intrinsics, mds[0].c2w, BOX,
                            near_far_override=(2.0, 6.0))
    n, views, t0 = 0, 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds and views < len(mds):
        m = mds[views]
        r = MO.process_single_image(m._img, m._mask, m.H, m.W, m.intrinsics, m.c2w, BOX, near_far_override=(2.0, 6.0),
                                    image_index=m.image_index)
        n += 0 if r is None else r[0].shape[0]
        views += 1
    el = time.perf_counter() - t0
    return {"value": round(n / el, 1), "unit": "rays/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"{views} views x 800x800 through the oracle's _process_single_image in {el:.1f}s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--views", type=int, default=100)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from nerf_amd import data as D
    from nerf_amd._lib import check, lib, ptr, stream
    from nerf_amd.occupancy import exclusive_scan
    from nerf_amd.ray_sampling import SceneBox

    mds = scene(a.views)
    kw = {"scene_box": SceneBox(aabb=BOX), "near_far_override": (2.0, 6.0)}
    ds = D.RamRaysDataset(mds, center_pixels=True, ray_gen_kwargs=kw, device=dev)   # warm-up + result size
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        ds = D.RamRaysDataset(mds, center_pixels=True, ray_gen_kwargs=kw, device=dev)
    torch.cuda.synchronize()
    e2e = (time.perf_counter() - t0) / a.reps
    n_rays = len(ds)

    # device-resident inputs: the same kernels as build_run, timed per stage with HIP events
    H, W, n_img = 800, 800, len(mds)
    imgs = torch.stack([m._img for m in mds]).to(dev)
    masks = torch.stack([torch.ones(H * W, dtype=torch.bool) if m._mask is None else m._mask.reshape(-1)
                         for m in mds]).to(torch.uint8).to(dev)
    c2w = torch.stack([m.c2w.reshape(12) for m in mds]).to(dev)
    intr = torch.stack([m.intrinsics for m in mds]).float().to(dev)
    ids = torch.arange(n_img, dtype=torch.int32, device=dev)
    aabb = BOX.reshape(6).to(dev)
    n = n_img * H * W
    flags = torch.empty(n, dtype=torch.int32, device=dev)
    rays = torch.empty((n_rays, 8), dtype=torch.float32, device=dev)
    rgbs = torch.empty((n_rays, 3), dtype=torch.float32, device=dev)
    idx = torch.empty((n_rays,), dtype=torch.int32, device=dev)
    L = lib()
    args = (ptr(c2w), ptr(intr), ptr(ids), n_img, H, W, 1, ptr(aabb), 1, 2.0, 1, 6.0, ptr(imgs), ptr(masks))
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    t = {"count": 0.0, "scan": 0.0, "write": 0.0}
    for rep in range(a.reps + 1):
        ev[0].record()
        check(L.nerf_dataset_rays(*args, ptr(flags), None, None, None, None, stream()), "count")
        ev[1].record()
        pos = exclusive_scan(flags)
        ev[2].record()
        check(L.nerf_dataset_rays(*args, None, ptr(pos), ptr(rays), ptr(rgbs), ptr(idx), stream()), "write")
        ev[3].record()
        torch.cuda.synchronize()
        if rep:  # first rep is warm-up
            t["count"] += ev[0].elapsed_time(ev[1]) / a.reps
            t["scan"] += ev[1].elapsed_time(ev[2]) / a.reps
            t["write"] += ev[2].elapsed_time(ev[3]) / a.reps
    assert int(pos[-1].item()) == n_rays
    assert torch.equal(rays, ds._rays) and torch.equal(rgbs, ds._rgbs)
    dev_ms = sum(t.values())
    # algorithmic bytes: count = mask 1 B/px (read) + flag 4 B/px (write); scan = 4 B/px in + 4 B/px out;
    # write = pos 4 B/px + per kept row 3 B pixel + 48 B out (rays 32, rgb 12, index 4)
    n_masked = sum(1 for m in mds if m._mask is not None)
    algo = {"count": n * 4 + n_masked * H * W, "scan": 8 * n, "write": 4 * n + n_rays * 51}
    dom = max(t, key=t.get)
    ach = algo[dom] / (t[dom] * 1e-3) / 1e9
    out = {
        "metric": "rays/s (RamRaysDataset GPU build, SURVEY §8f row 4), 100 x 800x800 Blender-style views",
        "value": round(n_rays / (dev_ms * 1e-3), 1), "unit": "rays/s", "n_gpus": 1, "steps": a.reps, "warmup": 1,
        "ms_per_step": round(dev_ms, 4), "higher_is_better": True, "dtype": "f32", "data": "synthetic",
        "config": {"workload": f"{n_img} views 800x800, AABB [-1.5,1.5]^3, override (2,6), mask on every 2nd view",
                   "pixels": n, "rays_kept": n_rays},
        "stage_ms": {k: round(v, 4) for k, v in t.items()},
        "end_to_end_ms": round(e2e * 1e3, 2),
        "end_to_end_rays_per_s": round(n_rays / e2e, 1),
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None, "bytes_per_launch": algo[dom],
                     "all_stages_GBs": round(sum(algo.values()) / (dev_ms * 1e-3) / 1e9, 1)},
    }
    out["cpu_baseline"] = None if a.no_cpu_baseline else cpu_baseline(mds, a.cpu_seconds)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
