"""The multi-stream schedule of the fp32 train step (-m gpu): nerf_mlp_bwd_2s runs the weight-gradient GEMMs on a
second stream beside the input-gradient chain.  It launches the same kernels on the same grids into the same split
slabs, so the packed gradient must be BITWISE the one-stream nerf_mlp_bwd's — at a ragged size, at the C2 fine-net
size, accumulating into a non-zero target — and a NeRFTrainer step with the fine weight gradients on their own
stream must equal the in-line step over three steps: gradient buffer and post-Adam parameters bitwise, the loss scalar
(summed by per-ray atomics in the compositing kernel) to rounding."""
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


@pytest.mark.parametrize("M", [1, 40001, 786432])
def test_two_stream_backward_bitwise(K, M):
    from nerf_amd.vanilla import VanillaNeRF
    w = VanillaNeRF().load_reference_state(O.init_vanilla_params(4)).to(DEV).packed().detach().contiguous()
    g = torch.Generator().manual_seed(M)
    x = torch.cat([torch.rand(M, 3, generator=g) * 3 - 1.5,
                   torch.nn.functional.normalize(torch.randn(M, 3, generator=g), dim=-1)], -1).to(DEV)
    gup = (torch.randn(M, 4, generator=g) * 1e-3).to(DEV)
    ws1 = K.mlp_workspace(M, True, DEV)
    ws2 = torch.empty(K.mlp_workspace_bytes_2s(M), dtype=torch.uint8, device=DEV)
    o1 = K.mlp_fwd(w, x, ws1, True)
    o2 = K.mlp_fwd(w, x, ws2, True)
    assert torch.equal(o1, o2)
    base = (torch.randn(w.shape, generator=g) * 1e-2).to(DEV)
    d1 = K.mlp_bwd(w, M, gup, ws1, d_w=base.clone(), accumulate=True)
    side = torch.cuda.Stream()
    sync = [torch.cuda.Event() for _ in range(10)]
    d2 = K.mlp_bwd(w, M, gup, ws2, d_w=base.clone(), accumulate=True, wgrad_stream=side, sync=sync)
    torch.cuda.synchronize()
    assert torch.isfinite(d1).all()
    assert torch.equal(d1, d2), f"max diff {float((d1 - d2).abs().max()):.3e}"


def test_trainer_split_wgrad_equals_inline(K):
    from nerf_amd.trainer import NeRFTrainer
    from nerf_amd.vanilla import VanillaNeRF
    g = torch.Generator().manual_seed(31)
    n = 512
    o = torch.tensor([0.0, -4.0311, 0.5]).expand(n, 3)
    d = torch.nn.functional.normalize(torch.randn(n, 3, generator=g) * 0.2 + torch.tensor([0.0, 1.0, -0.12]), dim=-1)
    rays = torch.cat([o, d, torch.full((n, 1), 2.0), torch.full((n, 1), 6.0)], -1).to(DEV)
    gt = torch.rand(n, 3, generator=g).to(DEV)
    us = [torch.rand(n, 64, generator=g).to(DEV) for _ in range(3)]
    up = [torch.rand(n, 128, generator=g).to(DEV) for _ in range(3)]
    res = {}
    for split in (False, True):
        tr = NeRFTrainer(VanillaNeRF().load_reference_state(O.init_vanilla_params(1)).to(DEV),
                         VanillaNeRF().load_reference_state(O.init_vanilla_params(2)).to(DEV),
                         n_samples=64, n_importance=128, split_wgrad=split)
        assert tr.split_wgrad == split
        out = []
        for s in range(3):
            loss = tr.step(rays, gt, seed=s, u_strat=us[s], u_pdf=up[s])
            torch.cuda.synchronize()
            out.append((float(loss.item()), tr.grads.clone(), tr.params.clone()))
        res[split] = out
    for s in range(3):
        a, b = res[False][s], res[True][s]
        # the loss scalar is summed by per-ray float atomics (order not fixed run to run: 512 rays of ~5e-4 each, so
        # a few fp32 ulps of the sum apart, 2.7e-7 relative seen on MI355X); the gradients do not depend on it
        assert abs(a[0] - b[0]) <= 1e-5 * abs(a[0]), (s, a[0], b[0])
        assert torch.equal(a[1], b[1]), f"step {s}: gradient buffers differ"
        assert torch.equal(a[2], b[2]), f"step {s}: parameters differ"


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_trainer_stream_schedules_equal(K, precision):
    """Where the coarse backward runs — beside the fine backward (the default since round 6), beside the fine forward,
    or in line on the main stream (overlap=False) — is scheduling only: the two nets' gradients land in disjoint
    segments of the flat buffer, so the gradients and post-Adam parameters are bitwise equal over three steps."""
    from nerf_amd.trainer import NeRFTrainer
    from nerf_amd.vanilla import VanillaNeRF
    g = torch.Generator().manual_seed(37)
    n = 1024
    o = torch.tensor([0.0, -4.0311, 0.5]).expand(n, 3)
    d = torch.nn.functional.normalize(torch.randn(n, 3, generator=g) * 0.2 + torch.tensor([0.0, 1.0, -0.12]), dim=-1)
    rays = torch.cat([o, d, torch.full((n, 1), 2.0), torch.full((n, 1), 6.0)], -1).to(DEV)
    gt = torch.rand(n, 3, generator=g).to(DEV)
    us = [torch.rand(n, 64, generator=g).to(DEV) for _ in range(3)]
    up = [torch.rand(n, 128, generator=g).to(DEV) for _ in range(3)]
    res = {}
    for name, kw in (("bwd", {}), ("fwd", {"overlap_with": "fwd"}), ("inline", {"overlap": False})):
        tr = NeRFTrainer(VanillaNeRF().load_reference_state(O.init_vanilla_params(1)).to(DEV),
                         VanillaNeRF().load_reference_state(O.init_vanilla_params(2)).to(DEV),
                         n_samples=64, n_importance=128, precision=precision, **kw)
        assert tr.overlap == (name != "inline") and (name == "inline" or tr.overlap_with == name)
        out = []
        for s in range(3):
            loss = tr.step(rays, gt, seed=s, u_strat=us[s], u_pdf=up[s])
            torch.cuda.synchronize()
            out.append((float(loss.item()), tr.grads.clone(), tr.params.clone()))
        res[name] = out
    for name in ("fwd", "inline"):
        for s in range(3):
            a, b = res["bwd"][s], res[name][s]
            assert abs(a[0] - b[0]) <= 1e-5 * abs(a[0]), (name, s, a[0], b[0])  # per-ray atomics in the loss sum
            assert torch.equal(a[1], b[1]), f"{name} step {s}: gradient buffers differ"
            assert torch.equal(a[2], b[2]), f"{name} step {s}: parameters differ"
