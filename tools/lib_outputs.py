#!/usr/bin/env python3
"""Bitwise A/B of two library builds (tools/build_exp.sh): run the fused MLP forward / backward of one precision on
fixed seeded inputs with the library NERF_AMD_LIB names and save the outputs; --compare A B checks two saved files
bit for bit (no GPU).

  NERF_AMD_LIB=exp/x.so python tools/lib_outputs.py --precision fp16 --out gpurun_out/x.pt
  python tools/lib_outputs.py --compare gpurun_out/x.pt gpurun_out/y.pt"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "nerf-sys_amd")]
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--precision", default="fp16")
ap.add_argument("--out")
ap.add_argument("--compare", nargs=2)
a = ap.parse_args()
if a.compare:
    x, y = (torch.load(f, weights_only=True) for f in a.compare)
    bad = [k for k in x if not torch.equal(x[k], y[k])]
    print("bitwise equal" if not bad else f"DIFFER: {bad}", {k: tuple(v.shape) for k, v in x.items()})
    for k in bad:  # largest difference relative to the array's scale, and the count of differing elements
        d = (x[k].double() - y[k].double()).abs()
        print(f"  {k}: {int((d > 0).sum())} differ, max |d| {d.max().item():.3e}, "
              f"max |d| / max |y| {(d.max() / y[k].double().abs().max()).item():.3e}")
    sys.exit(1 if bad else 0)
from nerf_amd import kernels as K  # noqa: E402
from nerf_amd.vanilla import VanillaNeRF  # noqa: E402

dev = "cuda"
torch.manual_seed(0)
w = VanillaNeRF().to(dev).packed().detach().contiguous()
out = {}
for M in (4096, 40001):
    g = torch.Generator().manual_seed(M)
    x = torch.cat([torch.rand(M, 3, generator=g) * 3 - 1.5,
                   torch.nn.functional.normalize(torch.randn(M, 3, generator=g), dim=-1)], -1).to(dev)
    ws = K.mlp_workspace(M, True, dev, a.precision)
    out[f"fwd{M}"] = K.mlp_fwd(w, x, ws, True, precision=a.precision).cpu()
    gup = (torch.randn(M, 4, generator=g) * 64).to(dev)
    out[f"bwd{M}"] = K.mlp_bwd(w, M, gup, ws, precision=a.precision).cpu()
torch.save(out, a.out)
print("saved", a.out)
