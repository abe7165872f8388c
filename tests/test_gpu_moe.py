"""MoE container on the HIP path vs the reference's golden vectors
(tests/golden/moe.npz) and the CPU oracle (oracle/moe_oracle.py).  Run on an MI355X: -m gpu.

Tolerances: routing weights 1e-6 (direct distances vs torch.cdist's matrix form: fp32 rounding); the
mix outputs 1e-5 (north-star bar 1e-4); gradients 1e-4 of their scale."""
from collections import OrderedDict

import pytest
import torch

from golden_io import load
from oracle import moe_oracle as MO
from oracle import nerf_oracle as O
from oracle import ngp_oracle as NO

pytestmark = pytest.mark.gpu
DEV = "cuda"
K = 3
CASES = {"soft": (1.05, True), "hard": (1.0, False)}
KW = dict(hidden=32, sigma_depth=1, color_hidden=32, color_depth=1, dir_encoding="spherical",
          hash_enc_conf=dict(levels=4, features_per_level=2, log2_hashmap_size=10, min_res=8, max_res=128,
                             interpolation="Linear"))


def _err(a, b):
    return (a.detach().float().cpu() - b.detach().float().cpu()).abs().max().item() if a.numel() else 0.0


@pytest.fixture(scope="module")
def z():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return load("moe")


def _container(z, tag):
    from nerf_amd.container import MetaContainer
    from nerf_amd.ray_sampling import SceneBox
    bm, c2d = CASES[tag]
    mc = MetaContainer(num_submodules=K, centroids=z["centroids"], aabb=torch.tensor([[-1.5] * 3, [1.5] * 3]),
                       nerf_variant="instant", boundary_margin=bm, cluster_2d=c2d, use_bg_nerf=True, bg_hidden=32,
                       occ_conf={}, expert_box_list=[SceneBox(aabb=z[f"box{k}"]) for k in range(K)], **KW)
    state = {k[len(tag) + 3:]: v for k, v in z.items() if k.startswith(f"{tag}_w/")}
    assert set(state) == {n for n, _ in mc.named_parameters()}
    return mc.load_reference_state(state).to(DEV)


@pytest.mark.parametrize("tag", list(CASES))
def test_routing_and_dispatch(z, tag):
    from nerf_amd.container import moe_route, moe_dispatch
    bm, c2d = CASES[tag]
    x = z["x_d"].to(DEV)
    W = moe_route(x, z["centroids"].reshape(-1).tolist(), bm, c2d)
    assert _err(W, z[f"{tag}_route"]) <= 1e-6
    offs, idx = moe_dispatch(W)
    ref = z[f"{tag}_route"]
    for k in range(K):
        sel = idx[offs[k]:offs[k + 1]].cpu().long()
        assert torch.equal(sel, (ref[:, k] > 0).nonzero().squeeze(1)), k   # torch.nonzero order


@pytest.mark.parametrize("tag", list(CASES))
def test_container_golden(z, tag):
    mc = _container(z, tag)
    out = mc(z["x_d"].to(DEV))
    assert _err(out, z[f"{tag}_out"]) <= 1e-5
    (out * z[f"{tag}_gup"].to(DEV)).sum().backward()
    for n, p in mc.named_parameters():
        key = f"{tag}_g/{n}"
        if key not in z:
            assert p.grad is None or float(p.grad.abs().max()) == 0.0, n
            continue
        ref = z[key]
        assert _err(p.grad, ref) <= 1e-4 * max(1.0, ref.abs().max().item()), n
    g = mc.get_param_groups()
    assert [len(g[k]["params"]) for k in ("encoding", "sigma", "color", "background")] == z[f"{tag}_groups"].tolist()


def test_background_color_golden(z):
    mc = _container(z, "soft")
    out = mc.background_color(z["bg_d"].to(DEV))
    assert _err(out, z["bg_out"]) <= 1e-6
    (out * z["bg_gup"].to(DEV)).sum().backward()
    for n, p in mc.named_parameters():
        if n.startswith("bg_mlp"):
            ref = z[f"bg_g/{n}"]
            assert _err(p.grad, ref) <= 1e-5 * max(1.0, ref.abs().max().item()), n
    b3 = mc.background_color(z["bg_d"].to(DEV).view(3, 100, 3))
    assert b3.shape == (3, 100, 3) and torch.equal(b3.reshape(-1, 3), out.detach())


def test_container_fast_weights_and_active_module(z):
    mc = _container(z, "soft")
    x = z["x_d"].to(DEV)
    fast = OrderedDict((n, p * 1.0) for n, p in mc.meta_named_parameters())
    assert not any("hash_table" in n or "bg_mlp" in n for n in fast)
    assert torch.equal(mc(x, params=fast), mc(x))
    y1 = mc(x, active_module=1)
    assert torch.equal(y1, mc.submodules[1](x))


def test_container_render_rays(z):
    """The reference's production model on the stratified path: container of NGP experts + background MLP
    (use_bg_nerf) inside render_rays, vs the oracle composition."""
    from nerf_amd.ray_rendering import render_rays
    mc = _container(z, "soft").eval()
    g = torch.Generator().manual_seed(9)
    n = 64
    o = torch.tensor([0.1, -3.0, 0.3]).expand(n, 3)
    d = torch.nn.functional.normalize(torch.randn(n, 3, generator=g) * 0.3 + torch.tensor([0.0, 1.0, 0.0]), dim=-1)
    rays = torch.cat([o, d, torch.full((n, 1), 1.5), torch.full((n, 1), 4.5)], -1)
    rgb, depth, w, acc = render_rays(mc, rays.to(DEV), ray_samples=48)
    p = {k[len("soft_w/"):]: v for k, v in z.items() if k.startswith("soft_w/")}
    res, _ = NO.hash_resolutions(4, 8, 128)
    exps = []
    for k in range(K):
        pre = f"submodules.{k}."
        pk = OrderedDict((nm[len(pre):], v) for nm, v in p.items() if nm.startswith(pre))
        tb = pk.pop("xyz_encoder.hash_table")
        exps.append(lambda x_d, pk=pk, tb=tb, box=z[f"box{k}"]: NO.ngp_forward(pk, tb, x_d, box, res, 10, 2,
                                                                               sigma_depth=1, color_depth=1))
    bg = MO.background_color(d, p["bg_mlp.0.weight"], p["bg_mlp.0.bias"], p["bg_mlp.2.weight"], p["bg_mlp.2.bias"])
    ref = O.render_rays(lambda x_d: MO.container_forward(exps, x_d, z["centroids"], 1.05, True), rays, 48,
                        training=False, bg=bg)
    for a, b, what in ((rgb, ref[0], "rgb"), (depth, ref[1], "depth"), (w, ref[2], "weights"), (acc, ref[3], "acc")):
        assert _err(a, b) <= 1e-4 * max(1.0, b.abs().max().item()), what
