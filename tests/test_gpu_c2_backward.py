"""C2-size backward parity (-m gpu): one engine train step at the headline shape — 4096 rays x (64 + 128), two 8x256
nets, the default fp32 engine (every trunk GEMM as split bf16 products, gemm_x6.hpp) — so every split kernel runs on
its C2 grids (fine M = 786,432, coarse M = 262,144), checked against an fp64 autograd evaluation of the oracle's
render_rays (oracle/nerf_oracle.py, run on the GPU in float64 as the checker) on the same rays, the same stratified /
inverse-CDF jitter and the same initial weights (runtime_adapt.py:286-306: render -> MSE coarse + fine -> backward).

Bounds: the step's loss within 1e-5 relative; every parameter tensor of both nets within 1e-4 relative error norm and
its largest element error within 1e-4 of the tensor's scale (the north-star tolerance).  The fine samples are
resampled from each side's own coarse weights (fp32 vs fp64); the inverse CDF is continuous in the weights, so that
difference is of the fp32 rounding size.  ReLU pre-activations within rounding of 0 may flip between the two sides;
each such row moves one sample's term of a 786,432-row sum, far below the bound (measured errors are printed)."""
import math

import pytest
import torch

from oracle import nerf_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def K():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from nerf_amd import kernels
    return kernels


def _rays(n, seed):
    """Rays of a Lego-style capture: origins on a radius-4 sphere around the object, aimed at it with a jitter that
    covers an 800x800 view's field, near 2 / far 6 (the blender defaults)."""
    g = torch.Generator().manual_seed(seed)
    th = torch.rand(n, generator=g) * 2 * math.pi
    ph = torch.rand(n, generator=g) * 0.5 * math.pi
    o = 4.0 * torch.stack([ph.cos() * th.cos(), ph.cos() * th.sin(), ph.sin()], -1)
    d = torch.nn.functional.normalize(-o / 4.0 + 0.35 * (torch.rand(n, 3, generator=g) - 0.5), dim=-1)
    rays = torch.cat([o, d, torch.full((n, 1), 2.0), torch.full((n, 1), 6.0)], -1)
    gt = torch.rand(n, 3, generator=g)
    return rays, gt


def test_c2_engine_step_gradients_vs_fp64(K):
    from nerf_amd.trainer import NeRFTrainer
    from nerf_amd.vanilla import PackedLayout, VanillaNeRF
    n, S, NI = 4096, 64, 128
    rays, gt = _rays(n, 11)
    g = torch.Generator().manual_seed(12)
    us, up = torch.rand(n, S, generator=g), torch.rand(n, NI, generator=g)
    pc, pf = O.init_vanilla_params(21), O.init_vanilla_params(22)
    tr = NeRFTrainer(VanillaNeRF().load_reference_state(pc).to(DEV), VanillaNeRF().load_reference_state(pf).to(DEV),
                     n_samples=S, n_importance=NI)
    assert tr.fp32_gemm == "split"
    loss = tr.step(rays.to(DEV), gt.to(DEV), seed=0, u_strat=us.to(DEV), u_pdf=up.to(DEV)).item()
    torch.cuda.synchronize()

    p64 = [{k: v.to(DEV, torch.float64).requires_grad_(True) for k, v in p.items()} for p in (pc, pf)]
    rgb, _, _, _, ex = O.render_rays(p64[0], rays.to(DEV, torch.float64), S, training=True,
                                     u_strat=us.to(DEV, torch.float64), bg="white", p_fine=p64[1], n_importance=NI,
                                     u_pdf=up.to(DEV, torch.float64))
    gt64 = gt.to(DEV, torch.float64)
    lref = O.mse_loss(rgb, gt64) + O.mse_loss(ex["rgb_coarse"], gt64)
    grads = torch.autograd.grad(lref, [v for p in p64 for v in p.values()])
    lref = lref.item()
    assert abs(loss - lref) <= 1e-5 * lref, (loss, lref)

    L = PackedLayout.get()
    names = list(p64[0].keys())
    worst = (0.0, None)
    for k in range(2):
        gk = L.unpack(tr.g(k).detach().cpu())
        for j, nme in enumerate(names):
            ref = grads[k * len(names) + j].detach().cpu()
            got = gk[nme].double()
            rn = ref.norm().item()
            rel = (got - ref).norm().item() / rn if rn > 0 else (got - ref).norm().item()
            mx = (got - ref).abs().max().item() / max(ref.abs().max().item(), 1e-30)
            worst = max(worst, (rel, f"net{k} {nme}"))
            assert rel <= 1e-4, f"net{k} {nme}: relative error norm {rel:.3e}"
            assert mx <= 1e-4, f"net{k} {nme}: max element error {mx:.3e} of the tensor scale"
    print(f"C2 step: loss {loss:.7f} vs fp64 {lref:.7f}; worst tensor relative error {worst[0]:.3e} ({worst[1]})")
