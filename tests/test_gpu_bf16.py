"""bf16 MLP path (BASELINE.json configs[2], "bf16 MLP with fp32 compositing") on an MI355X (-m gpu).

There is no bf16 reference in psklavos1/NeRF-Sys (its low-precision mode is fp16 autocast), so the bf16
path is checked against the fp32 oracle / the fp32 HIP path with tolerances that bf16 rounding of every
layer's inputs implies (8-bit mantissa: ~4e-3 relative per rounding, accumulated over 8+3 layers):
  forward   rgb within 2e-2 absolute, raw sigma (log sigma) within 0.1 absolute;
  gradients per parameter tensor: relative L2 error <= 0.15 and cosine >= 0.99 against the fp32 path
            (random upstream gradients cancel in the deep-layer sums, measured worst: trunk.0 0.11 / 0.994);
  training  the bf16 engine's loss trajectory tracks the fp32 engine's (same seeds) within 15 %.
The GEMM kernels themselves are exact up to fp32 accumulation order on bf16-rounded operands
(tools/gemm_bf16_test.hip checks them against an fp64 host product: <= 1e-7 of sum|a b|)."""
import pytest
import torch

from golden_io import mlp_params
from oracle import nerf_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def K():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from nerf_amd import kernels
    return kernels


@pytest.fixture(scope="module")
def wpk(K):
    from nerf_amd.vanilla import VanillaNeRF
    net = VanillaNeRF().load_reference_state(mlp_params("w/")).to(DEV)
    return net.packed().detach().contiguous()


def _xd(M, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.cat([torch.rand(M, 3, generator=g) * 3 - 1.5,
                      torch.nn.functional.normalize(torch.randn(M, 3, generator=g), dim=-1)], -1)


@pytest.mark.parametrize("M", [1, 255, 1000, 4096])
def test_mlp_bf16_forward_vs_oracle(K, wpk, M):
    x = _xd(M, 3)
    out = K.mlp_fwd(wpk, x.to(DEV), K.mlp_workspace(M, True, DEV, "bf16"), True, precision="bf16").cpu()
    ref = O.vanilla_forward(mlp_params("w/"), x).detach()
    assert torch.isfinite(out).all()
    assert (out[:, :3] - ref[:, :3]).abs().max().item() <= 2e-2
    raw = torch.log(out[:, 3].clamp_min(1e-30))
    raw_ref = torch.log(ref[:, 3].clamp_min(1e-30))
    assert (raw - raw_ref).abs().max().item() <= 0.1


def test_mlp_bf16_inference_equals_training(K, wpk):
    x = _xd(3000, 5).to(DEV)
    a = K.mlp_fwd(wpk, x, K.mlp_workspace(3000, True, DEV, "bf16"), True, precision="bf16")
    b = K.mlp_fwd(wpk, x, K.mlp_workspace(3000, False, DEV, "bf16"), False, precision="bf16")
    assert torch.equal(a, b)


def test_mlp_bf16_gradients_vs_fp32(K, wpk):
    from nerf_amd.vanilla import PackedLayout
    M = 8192
    x = _xd(M, 7).to(DEV)
    g = torch.Generator().manual_seed(11)
    gup = (torch.randn(M, 4, generator=g) * 1e-3).to(DEV)
    grads = {}
    for prec in ("fp32", "bf16"):
        ws = K.mlp_workspace(M, True, DEV, prec)
        K.mlp_fwd(wpk, x, ws, True, precision=prec)
        grads[prec] = K.mlp_bwd(wpk, M, gup, ws, precision=prec)
    L = PackedLayout.get()
    a, b = L.unpack(grads["bf16"]), L.unpack(grads["fp32"])
    for name in b:
        ref, got = b[name].double(), a[name].double()
        if ref.norm() == 0:
            continue
        rel = ((got - ref).norm() / ref.norm()).item()
        cos = (torch.dot(got.flatten(), ref.flatten()) / (got.norm() * ref.norm())).item()
        assert rel <= 0.15 and cos >= 0.99, f"{name}: rel {rel:.3e} cos {cos:.5f}"


def test_bf16_engine_tracks_fp32_loss(K):
    from nerf_amd.scene import make_blender_scene
    from nerf_amd.trainer import NeRFTrainer, RayBatcher
    from nerf_amd.vanilla import VanillaNeRF
    scene = make_blender_scene(n_train=4, n_test=1, H=100, W=100, seed=0, device=DEV)
    rb = RayBatcher(scene, DEV)
    curves = {}
    for prec in ("fp32", "bf16"):
        torch.manual_seed(0)
        c, f = VanillaNeRF().to(DEV), VanillaNeRF().to(DEV)
        tr = NeRFTrainer(c, f, n_samples=32, n_importance=32, device=DEV, precision=prec)
        ls = []
        for s in range(40):
            rays, gt = rb.batch(1024, seed=s)
            ls.append(float(tr.step(rays, gt, seed=s).item()))
        curves[prec] = ls
    a, b = torch.tensor(curves["bf16"]), torch.tensor(curves["fp32"])
    assert torch.isfinite(a).all()
    assert a[-10:].mean() < a[:5].mean()  # it learns
    assert (a[-10:].mean() - b[-10:].mean()).abs() <= 0.15 * b[-10:].mean()


def test_fused_forward_matches_layered(K, wpk):
    """The single-launch fused bf16 forward (mlp_bf16_fused.hpp) against the layer-by-layer bf16 GEMM path
    (bf16_flags=BF16_LAYERED_FWD): the same bf16 rounding points and k order, only the bias enters the fp32 accumulator
    first instead of last — outputs agree to bf16 rounding flips, the saved activations feed the same backward."""
    M = 5000  # two row tiles short of a multiple of 256: pad rows in the last tile
    x = _xd(M, 9).to(DEV)
    g = torch.Generator().manual_seed(13)
    gup = (torch.randn(M, 4, generator=g) * 1e-3).to(DEV)
    res = {}
    for mode in ("0", "1"):
        fl = K.BF16_LAYERED_FWD if mode == "0" else 0
        ws = K.mlp_workspace(M, True, DEV, "bf16")
        out = K.mlp_fwd(wpk, x, ws, True, precision="bf16", bf16_flags=fl)
        d_w = K.mlp_bwd(wpk, M, gup, ws, precision="bf16", bf16_flags=fl)
        inf = K.mlp_fwd(wpk, x, K.mlp_workspace(M, False, DEV, "bf16"), False, precision="bf16", bf16_flags=fl)
        assert torch.equal(out, inf), f"mode {mode}: inference != training forward"
        res[mode] = (out.cpu(), d_w.cpu())
    (o0, g0), (o1, g1) = res["0"], res["1"]
    assert (o1[:, :3] - o0[:, :3]).abs().max().item() <= 5e-3
    assert ((o1[:, 3] - o0[:, 3]).abs() <= 2e-2 * o0[:, 3].abs() + 1e-6).all()
    from nerf_amd.vanilla import PackedLayout
    a, b = PackedLayout.get().unpack(g1), PackedLayout.get().unpack(g0)
    for name in b:
        ref, got = b[name].double(), a[name].double()
        if ref.norm() == 0:
            continue
        rel = ((got - ref).norm() / ref.norm()).item()
        assert rel <= 2e-2, f"{name}: fused vs layered gradient rel {rel:.3e}"


@pytest.mark.parametrize("M", [1, 5000, 40001, 786432])
def test_fused_backward_matches_layered(K, wpk, M):
    """The fused per-layer bf16 backward (mlp_bf16_bwd.hpp: input + weight gradient of a trunk layer in one launch,
    ReLU mask from the saved input; the head / colour "tail" in one launch, mlp_bf16_tail.hpp) against the layered
    launches (bf16_flags=BF16_LAYERED_BWD): the same bf16 operands, rounding points and MFMA k order, so dZ7 and the
    256-wide trunk weight gradients are BITWISE equal; the trunk biases (column sums by the io waves that stage the
    rows), the head / colour sums (each split in two row halves) and the narrow trunk.0 / trunk.4-encoding sums (4x
    finer sub-splits) are the same fp32 terms in another fixed order: within 1e-5 of their scale, and bitwise
    reproducible run to run.
    Sizes: one row; a ragged tile; 19 splits (not a multiple of the 8-split block pairing: idle pairs exit); the
    C2 fine-net size (256 splits of 3,072 rows, 512 workgroups)."""
    from nerf_amd.vanilla import PackedLayout
    x = _xd(M, 21).to(DEV)
    g = torch.Generator().manual_seed(23)
    gup = (torch.randn(M, 4, generator=g) * 1e-3).to(DEV)
    ws = K.mlp_workspace(M, True, DEV, "bf16")
    # a forward for the layered backward also writes its ReLU bitmasks (the fused backward ignores them)
    K.mlp_fwd(wpk, x, ws, True, precision="bf16", bf16_flags=K.BF16_LAYERED_BWD)
    res = {}
    for mode in ("0", "1", "1b"):
        fl = K.BF16_LAYERED_BWD if mode == "0" else 0
        res[mode] = K.mlp_bwd(wpk, M, gup, ws, precision="bf16", bf16_flags=fl).cpu()
        torch.cuda.synchronize()
    assert torch.isfinite(res["1"]).all()
    assert torch.equal(res["1"], res["1b"]), "fused backward not reproducible"
    a, b = PackedLayout.get().unpack(res["1"]), PackedLayout.get().unpack(res["0"])
    exact = {f"trunk.{i}.linear.weight" for i in (1, 2, 3, 5, 6, 7)}
    for n in b:
        got, ref = a[n], b[n]
        if n == "trunk.4.linear.weight":  # the trunk.3 columns: fused; the encoding columns: narrow sub-split wgrad
            assert torch.equal(got[:, :256], ref[:, :256]), f"{n}[:, :256]: fused != layered at M={M}"
            got, ref = got[:, 256:], ref[:, 256:]
        if n in exact:
            assert torch.equal(got, ref), f"{n}: fused != layered at M={M}, max {float((got - ref).abs().max()):.3e}"
        else:  # same fp32 terms, another fixed summation order (io-wave column sums, split halves, sub-splits)
            scale = max(float(ref.abs().max()), 1e-30)
            err = float((got - ref).abs().max())
            assert err <= 1e-5 * scale, f"{n}: fused vs layered {err:.3e} (scale {scale:.3e}) at M={M}"
