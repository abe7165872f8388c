#!/usr/bin/env python3
"""The engine train step repeated under a profiler with a flushed progress line every --every steps (and the dispatch
count so far from the step's kernel count), to find where a rocprofv3 --pmc pass fails on this image (DESIGN.md §4,
"rocprofv3 PMC").  Same step as bench.py's engine leg (4096 rays, 64 + 128, two nets).

  python3 tools/pmc_engine_probe.py [--precision bf16|fp32] [--steps 4000] [--every 100] [--no-overlap]"""
import argparse
import faulthandler
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "nerf-sys_amd")]
import torch  # noqa: E402

faulthandler.enable(all_threads=True)
ap = argparse.ArgumentParser()
ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
ap.add_argument("--steps", type=int, default=4000)
ap.add_argument("--every", type=int, default=100)
ap.add_argument("--no-overlap", action="store_true", help="one stream: no side-stream coarse backward")
a = ap.parse_args()
from nerf_amd.scene import make_blender_scene  # noqa: E402
from nerf_amd.trainer import NeRFTrainer, RayBatcher  # noqa: E402
from nerf_amd.vanilla import VanillaNeRF  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
scene = make_blender_scene(n_train=4, n_test=1, H=800, W=800, seed=0, device=dev)
rb = RayBatcher(scene, dev)
tr = NeRFTrainer(VanillaNeRF().to(dev), VanillaNeRF().to(dev), n_samples=64, n_importance=128, device=dev,
                 precision=a.precision, overlap=not a.no_overlap)


def library_bases():
    """dladdr() of one exported symbol per runtime library in this process: the base each library is mapped at, so
    the raw PCs of a crash report name a library and an offset."""
    import ctypes

    class DlInfo(ctypes.Structure):
        _fields_ = [("fname", ctypes.c_char_p), ("fbase", ctypes.c_void_p), ("sname", ctypes.c_char_p),
                    ("saddr", ctypes.c_void_p)]
    libdl = ctypes.CDLL("libc.so.6")
    libdl.dladdr.argtypes = [ctypes.c_void_p, ctypes.POINTER(DlInfo)]
    for lib, sym in (("libc.so.6", "raise"), ("libamdhip64.so.7", "hipLaunchKernel"), ("libamdhip64.so", "hipLaunchKernel"),
                     ("libhsa-runtime64.so.1", "hsa_init"), ("librocprofiler-sdk.so.1", "rocprofiler_get_version"),
                     ("librocprofiler-sdk.so", "rocprofiler_get_version"),
                     ("librocprofiler-sdk-tool.so.1", "rocprofiler_configure"),
                     ("libnerf_amd.so", "nerf_mlp_layout")):
        try:
            h = ctypes.CDLL(lib, mode=getattr(ctypes, "RTLD_NOLOAD", 4) | ctypes.RTLD_GLOBAL)
            addr = ctypes.cast(getattr(h, sym), ctypes.c_void_p).value
        except (OSError, AttributeError):
            continue
        info = DlInfo()
        if libdl.dladdr(addr, ctypes.byref(info)):
            print(f"[engine probe] {sym} at {addr:#x}: {info.fname.decode()} mapped at {info.fbase:#x}", flush=True)


t0 = time.perf_counter()
for s in range(1, a.steps + 1):
    rays, gt = rb.batch(4096, seed=s)
    loss = tr.step(rays, gt, seed=s)
    if s == 1:
        library_bases()
    if s % a.every == 0:
        torch.cuda.synchronize()
        print(f"[engine probe {time.perf_counter() - t0:7.1f}s] {a.precision} step {s}, loss {float(loss.item()):.5f}",
              flush=True)
print("engine probe done", flush=True)
