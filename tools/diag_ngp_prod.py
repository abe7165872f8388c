"""Diagnostic: production-shape NGP backward, prod kernel vs generic kernel vs the oracle in fp32 and fp64."""
import os
import sys
from collections import OrderedDict
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nerf-sys_amd"))
sys.path.insert(0, ROOT)
import torch
from oracle import ngp_oracle as NO
from nerf_amd.ngp import InstantNGP

M = int(sys.argv[1]) if len(sys.argv) > 1 else 40001
levels = 8
torch.manual_seed(5)
box = torch.tensor([[-1.5] * 3, [1.5] * 3])
net = InstantNGP(scene_box=box, hidden=64, sigma_depth=2, color_hidden=64, color_depth=2, dir_encoding="spherical",
                 hash_enc_conf=dict(levels=levels, features_per_level=2, log2_hashmap_size=12, min_res=8, max_res=128,
                                    interpolation="Linear")).to("cuda")
with torch.no_grad():
    net.xyz_encoder.hash_table.uniform_(-0.1, 0.1)
g = torch.Generator().manual_seed(M)
x_d = torch.cat([torch.rand(M, 3, generator=g) * 3 - 1.5,
                 torch.nn.functional.normalize(torch.randn(M, 3, generator=g), dim=-1)], -1)
gup = torch.randn(M, 4, generator=g)


def grads(prod):
    net.net_struct.generic_kernels = 0 if prod else 1
    net.zero_grad(set_to_none=True)
    out = net(x_d.cuda())
    (out * gup.cuda()).sum().backward()
    torch.cuda.synchronize()
    return {n: p.grad.detach().cpu().double() for n, p in net.named_parameters()}


gp, gg = grads(True), grads(False)
res, _ = NO.hash_resolutions(levels, 8, 128)


def oracle(dt):
    w = OrderedDict((n, p.detach().cpu().to(dt).clone().requires_grad_(True)) for n, p in net.named_parameters())
    table = w.pop("xyz_encoder.hash_table")
    ref = NO.ngp_forward(w, table, x_d.to(dt), box.to(dt), res, 12, 2, sigma_depth=2, color_depth=2)
    rg = torch.autograd.grad((ref * gup.to(dt)).sum(), list(w.values()) + [table])
    return {n: r.detach().double() for (n, _), r in zip(list(w.items()) + [("xyz_encoder.hash_table", table)], rg)}


r32 = oracle(torch.float32)
try:
    r64 = oracle(torch.float64)
except Exception as e:  # the oracle may be fp32-only
    print("fp64 oracle failed:", e)
    r64 = None
for n in gp:
    e = lambda a, b: float((a - b).abs().max())
    line = f"{n:40s} max|r|={float(r32[n].abs().max()):9.4f} prod-r32={e(gp[n], r32[n]):.3e} gen-r32={e(gg[n], r32[n]):.3e} prod-gen={e(gp[n], gg[n]):.3e}"
    if r64 is not None:
        line += f" prod-r64={e(gp[n], r64[n]):.3e} gen-r64={e(gg[n], r64[n]):.3e} r32-r64={e(r32[n], r64[n]):.3e}"
    print(line)
