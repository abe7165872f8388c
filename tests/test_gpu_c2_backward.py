"""C2-size backward parity (-m gpu): one engine train step at the headline shape — 4096 rays x (64 + 128), two 8x256
nets, the default fp32 engine (every trunk GEMM as split bf16 products, gemm_x6.hpp) — so every split kernel runs on
its C2 grids (fine M = 786,432, coarse M = 262,144), checked against an fp64 autograd evaluation of the oracle
network + compositing (oracle/nerf_oracle.py, run on the GPU in float64 as the checker) at the engine's own fp32
sample positions, with the same initial weights and the loss of runtime_adapt.py:286-306 (MSE coarse + fine).

Why the engine's positions: the positional encoding's top band is sin(512 x); one fp32 ulp of a point (~2.4e-7 at
|x| ~ 2) moves its phase by ~1e-4 rad, so an fp64 re-derivation of the points (o + t d in fp64) alone moves the
trunk.0 weight gradient by ~4e-4 relative (measured on MI355X) — input rounding, not arithmetic.  The positions are
recomputed by the same deterministic kernels the step ran (stratified t from the injected jitter, the coarse forward +
compositing weights -> inverse-CDF t from the injected jitter, then the points), so they are the step's bitwise.

Bounds: the step's loss within 1e-5 relative of the fp64 loss; every parameter tensor of both nets within 1e-4
relative error norm and its largest element error within 1e-4 of the tensor's scale (the north-star tolerance), and
within 2x the relative error of the same step on the fp32-MFMA engine (fp32_gemm="native") — the split products are
as accurate as fp32 arithmetic at this size too.
ReLU pre-activations within rounding of 0 may flip between the two sides; each such row moves one sample's term of a
786,432-row sum, far below the bound (the measured worst tensor is printed)."""
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
    rd, usd, upd = rays.to(DEV), us.to(DEV), up.to(DEV)
    trs, losses = {}, {}
    for eng in ("split", "native"):  # the default engine, and every GEMM on the fp32 MFMA (the error yardstick)
        trs[eng] = NeRFTrainer(VanillaNeRF().load_reference_state(pc).to(DEV),
                               VanillaNeRF().load_reference_state(pf).to(DEV), n_samples=S, n_importance=NI,
                               fp32_gemm=eng)
        losses[eng] = trs[eng].step(rd, gt.to(DEV), seed=0, u_strat=usd, u_pdf=upd).item()
    torch.cuda.synchronize()
    loss = losses["split"]

    # the step's sample positions, from the same kernels on the same inputs (initial coarse weights)
    w0 = VanillaNeRF().load_reference_state(pc).to(DEV).packed().detach().contiguous()
    t_c = K.sample_stratified(rd, S, True, usd, 0)
    xd_c = K.build_xd(rd, t_c)
    rs_c = K.mlp_fwd(w0, xd_c, K.mlp_workspace(n * S, False, DEV), False)
    w_c = K.composite_fwd(rs_c, t_c, torch.ones(n, 3, device=DEV))[2]
    t_f = K.sample_pdf(t_c, w_c, NI, u=upd, det=False, seed=0)
    xd_f = K.build_xd(rd, t_f)

    p64 = [{k: v.to(DEV, torch.float64).requires_grad_(True) for k, v in p.items()} for p in (pc, pf)]
    gt64 = gt.to(DEV, torch.float64)
    bg64 = torch.ones(n, 3, dtype=torch.float64, device=DEV)
    lref = 0.0
    for p, xd, t, k in ((p64[0], xd_c, t_c, S), (p64[1], xd_f, t_f, S + NI)):
        rs = O.vanilla_forward(p, xd.double()).view(n, k, 4)
        rgb = O.volume_render(rs, t.double(), bg64)[0]
        lref = lref + O.mse_loss(rgb, gt64)
    grads = torch.autograd.grad(lref, [v for p in p64 for v in p.values()])
    lref = lref.item()
    assert abs(loss - lref) <= 1e-5 * lref, (loss, lref)

    L = PackedLayout.get()
    names = list(p64[0].keys())
    worst = (0.0, None, 0.0)
    for k in range(2):
        gk = {eng: L.unpack(t.g(k).detach().cpu()) for eng, t in trs.items()}
        for j, nme in enumerate(names):
            ref = grads[k * len(names) + j].detach().cpu()
            rn = max(ref.norm().item(), 1e-300)
            rel = {eng: (g[nme].double() - ref).norm().item() / rn for eng, g in gk.items()}
            mx = (gk["split"][nme].double() - ref).abs().max().item() / max(ref.abs().max().item(), 1e-30)
            worst = max(worst, (rel["split"], f"net{k} {nme}", rel["native"]))
            assert rel["split"] <= 1e-4, f"net{k} {nme}: relative error norm {rel['split']:.3e}"
            assert mx <= 1e-4, f"net{k} {nme}: max element error {mx:.3e} of the tensor scale"
            # the split engine as accurate as the fp32 MFMA engine on the same positions (2x, as test_gpu_split_gemm)
            assert rel["split"] <= 2.0 * rel["native"] + 1e-7, (k, nme, rel)
    print(f"C2 step: loss {loss:.7f} (native engine {losses['native']:.7f}) vs fp64 {lref:.7f}; worst tensor "
          f"relative error {worst[0]:.3e} ({worst[1]}; native engine {worst[2]:.3e})")
