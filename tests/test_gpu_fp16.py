"""fp16 build of the fused MLP kernels (include/nerf_amd.h nerf_mlp_*_f16) against the reference's autocast(float16)
numerics (-m gpu).

The reference trains with use_amp (configs/train.json:37; pipelines/online_stage/runtime_adapt.py:291-310): under
``torch.autocast(float16)`` every ``inputs.matmul(weight.t())`` of MetaLinear (models/metamodule/metamodule.py:150-156)
takes fp16 operands and returns fp16, the fp32 bias is added after it (so the layer outputs, ReLU and trunc_exp's input
are fp32), the matmul backward returns fp16 input / weight gradients and the bias gradients are fp32 sums.  The oracle
restates exactly that (oracle/nerf_oracle.py ``_MatmulF16`` / ``_lin(amp="fp16")``, pinned to the imported reference's
vectors in tests/golden/amp.npz by tests/test_oracle_golden.py), and the kernels keep the same rounding points.  What
still differs is the fp32 summation order inside each product (MFMA k order vs the CPU's), which moves an fp16 rounding
now and then; the bounds below are set for that:
  forward   rgb within 2e-3 absolute, raw sigma within 2e-3 of its scale (one fp16 ulp at the pre-activation's size
            is ~5e-4 relative; a flipped rounding deep in the trunk moves the outputs by a few of those);
  backward  every parameter tensor's relative error norm <= 1e-2, flat cosine >= 0.9999, bias of the sigma head and
            the colour-out layer (fp32 sums of fp32 gradients) <= 1e-3;
  format    the weight entries of d_w are fp16 values (the reference's weight gradient is an fp16 matmul output), the
            bias entries are not rounded; accumulate adds in fp32 after the rounding; bitwise run to run."""
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


def _oracle_amp(x, gup=None):
    p = {k: v.clone().requires_grad_(gup is not None) for k, v in mlp_params("w/").items()}
    out = O.vanilla_forward(p, x, amp="fp16")
    if gup is None:
        return out.detach(), None
    out.backward(gup)
    return out.detach(), {k: v.grad for k, v in p.items()}


@pytest.mark.parametrize("M", [1, 255, 1000, 4096])
def test_mlp_fp16_forward_vs_oracle_amp(K, wpk, M):
    x = _xd(M, 3)
    out = K.mlp_fwd(wpk, x.to(DEV), K.mlp_workspace(M, True, DEV, "fp16"), True, precision="fp16").cpu()
    ref, _ = _oracle_amp(x)
    assert torch.isfinite(out).all()
    e_rgb = (out[:, :3] - ref[:, :3]).abs().max().item()
    e_sig = ((out[:, 3] - ref[:, 3]).abs() / ref[:, 3].abs().clamp_min(1e-3)).max().item()
    print(f"M={M}: max |rgb - oracle amp| {e_rgb:.2e}, max sigma rel {e_sig:.2e}")
    assert e_rgb <= 2e-3 and e_sig <= 2e-3, (e_rgb, e_sig)
    # the fp16 build is closer to the reference's AMP arithmetic than the bf16 build is
    b16 = K.mlp_fwd(wpk, x.to(DEV), K.mlp_workspace(M, False, DEV, "bf16"), False, precision="bf16").cpu()
    if M >= 1000:
        assert e_rgb < (b16[:, :3] - ref[:, :3]).abs().max().item()


def test_mlp_fp16_inference_equals_training(K, wpk):
    x = _xd(3000, 5).to(DEV)
    a = K.mlp_fwd(wpk, x, K.mlp_workspace(3000, True, DEV, "fp16"), True, precision="fp16")
    b = K.mlp_fwd(wpk, x, K.mlp_workspace(3000, False, DEV, "fp16"), False, precision="fp16")
    assert torch.equal(a, b)


@pytest.mark.parametrize("M", [5000, 40001])
def test_mlp_fp16_gradients_vs_oracle_amp(K, wpk, M):
    from nerf_amd.vanilla import PackedLayout
    x = _xd(M, 7)
    g = torch.Generator().manual_seed(11)
    gup = torch.randn(M, 4, generator=g) * 64.0    # a GradScaler-style scaled upstream gradient
    ws = K.mlp_workspace(M, True, DEV, "fp16")
    K.mlp_fwd(wpk, x.to(DEV), ws, True, precision="fp16")
    d_w = K.mlp_bwd(wpk, M, gup.to(DEV), ws, precision="fp16")
    _, ref = _oracle_amp(x, gup)
    got = PackedLayout.get().unpack(d_w.cpu())
    a = torch.cat([got[n].double().flatten() for n in ref])
    b = torch.cat([ref[n].double().flatten() for n in ref])
    cos = float(a @ b / (a.norm() * b.norm()))
    worst = (0.0, "")
    for n, r in ref.items():
        r = r.double()
        if r.norm() == 0:
            continue
        err = float((got[n].double() - r).norm() / r.norm())
        worst = max(worst, (err, n))
        bound = 1e-3 if n in ("sigma_head.bias", "color_mlp.color_out.bias") else 1e-2
        assert err <= bound, f"{n}: relative error norm {err:.3e} > {bound}"
    print(f"M={M}: cosine {cos:.7f}, worst tensor {worst[1]} {worst[0]:.3e}")
    assert cos >= 0.9999, cos


def test_mlp_fp16_weight_gradient_format(K, wpk):
    """Weight entries of d_w are fp16-representable (an fp16 matmul output cast to fp32), bias entries are fp32 sums;
    accumulate=1 adds the rounded values in fp32; the result is bitwise reproducible."""
    from nerf_amd.vanilla import PackedLayout
    M = 9000
    x = _xd(M, 9).to(DEV)
    g = torch.Generator().manual_seed(5)
    gup = (torch.randn(M, 4, generator=g) * 1e3).to(DEV)
    ws = K.mlp_workspace(M, True, DEV, "fp16")
    K.mlp_fwd(wpk, x, ws, True, precision="fp16")
    d1 = K.mlp_bwd(wpk, M, gup, ws, precision="fp16")
    d2 = K.mlp_bwd(wpk, M, gup, ws, precision="fp16")
    assert torch.equal(d1, d2)
    parts = PackedLayout.get().unpack(d1.cpu())
    n_bias_off = 0
    for n, v in parts.items():
        if n.endswith(".weight"):
            assert torch.equal(v, v.half().float()), f"{n} is not fp16-valued"
        elif not torch.equal(v, v.half().float()):
            n_bias_off += 1
    assert n_bias_off > 0  # the bias sums are fp32, not rounded
    base = torch.randn_like(d1) * 1e-3
    acc = base.clone()
    K.mlp_bwd(wpk, M, gup, ws, d_w=acc, accumulate=True, precision="fp16")
    assert torch.equal(acc, base + d1)


def test_mlp_fp16_refuses_layered_flags(K, wpk):
    import ctypes  # noqa: F401
    from nerf_amd._lib import lib
    from nerf_amd.kernels import ptr
    M = 256
    x = _xd(M, 1).to(DEV)
    ws = K.mlp_workspace(M, True, DEV, "fp16")
    out = torch.empty(M, 4, device=DEV)
    rc = lib().nerf_mlp_fwd_f16(ptr(wpk), ptr(x), M, ptr(out), ptr(ws), ws.numel(), 1, K.BF16_LAYERED_FWD, None,
                                None)
    assert rc == -3  # NERF_E_ENUM: the fp16 build has only the fused kernels
    assert K.mlp_workspace_bytes(M, True, "fp16") == K.mlp_workspace_bytes(M, True, "bf16")


def test_mlp_fp16_empty_and_accumulate_zero_rows(K, wpk):
    """M = 0: the forward is a no-op and the backward zero-fills d_w (or leaves an accumulated d_w untouched)."""
    x = torch.empty(0, 6, device=DEV)
    ws = K.mlp_workspace(0, True, DEV, "fp16")
    out = K.mlp_fwd(wpk, x, ws, True, precision="fp16")
    assert out.shape == (0, 4)
    d_w = K.mlp_bwd(wpk, 0, torch.empty(0, 4, device=DEV), ws, precision="fp16")
    assert torch.count_nonzero(d_w) == 0
    base = torch.randn_like(wpk)
    acc = base.clone()
    K.mlp_bwd(wpk, 0, torch.empty(0, 4, device=DEV), ws, d_w=acc, accumulate=True, precision="fp16")
    assert torch.equal(acc, base)
