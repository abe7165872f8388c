"""Which half of the fp32 MLP backward carries the split GEMMs' extra gradient error: forward / backward engines
combined (native = fp32 MFMA, split = bf16 x6), weight-gradient error norms against an fp64 autograd reference (the
oracle on the GPU, test infrastructure), M = 40,001, kink rows excluded as in tests/test_gpu_split_gemm.py."""
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "nerf-sys_amd")
from oracle import nerf_oracle as O  # noqa: E402
from nerf_amd import kernels as K  # noqa: E402
from nerf_amd.vanilla import PackedLayout, VanillaNeRF  # noqa: E402

DEV = "cuda"
M = int(sys.argv[1]) if len(sys.argv) > 1 else 40001
net = VanillaNeRF().load_reference_state(O.init_vanilla_params(6)).to(DEV)
p = {k: v.detach() for k, v in net.named_parameters()}
w = net.packed().detach().contiguous()
g = torch.Generator().manual_seed(M + 1)
x = torch.cat([torch.rand(M, 3, generator=g) * 3 - 1.5,
               torch.nn.functional.normalize(torch.randn(M, 3, generator=g), dim=-1)], -1).to(DEV)
gup = torch.randn(M, 4, generator=g).to(DEV) * 1e-3
p64 = {k: v.double().requires_grad_(True) for k, v in p.items()}
seen = []
relu = torch.relu
torch.relu = lambda t: (seen.append(t.detach().abs().amin(-1)), relu(t))[1]
O.vanilla_forward({k: v.detach() for k, v in p64.items()}, x.double())
torch.relu = relu
gup[torch.stack(seen, 0).amin(0) < 2e-6] = 0.0
ref = O.vanilla_forward(p64, x.double())
gr = torch.autograd.grad((ref * gup.double()).sum(), list(p64.values()))
L = PackedLayout.get()
rp = torch.zeros(L.total, dtype=torch.float64, device=DEV)
for name, gk in zip(p64.keys(), gr):
    rp[L.index[name].to(DEV)] = gk.reshape(-1)
N = K.MLP_NATIVE_FP32
print("combo (fwd/bwd)   " + " ".join(f"t{t:<8d}" for t in range(0, 16)))
for fname, ff in (("native", N), ("split", 0)):
    for bname, bf in (("native", N), ("split", 0)):
        ws = K.mlp_workspace(M, True, DEV)
        K.mlp_fwd(w, x, ws, True, fp32_flags=ff)
        dw = K.mlp_bwd(w, M, gup, ws, fp32_flags=bf)
        row = []
        for t, (off, rows, cols, _) in enumerate(L.table[:16]):
            r = rp[off:off + rows * cols]
            row.append((dw[off:off + rows * cols].double() - r).norm().item() / max(r.norm().item(), 1e-300))
        print(f"{fname:>6s}/{bname:<9s} " + " ".join(f"{e:.2e}" for e in row))
