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


def _occ_container(z, seed=0):
    from nerf_amd.container import MetaContainer
    from nerf_amd.ray_sampling import SceneBox
    torch.manual_seed(seed)
    occ = {"use_occ": True, "resolution": 16, "levels": 2, "occ_ready": True, "near_plane": 0.05}
    mc = MetaContainer(num_submodules=K, centroids=z["centroids"], aabb=torch.tensor([[-1.5] * 3, [1.5] * 3]),
                       nerf_variant="instant", boundary_margin=1.05, cluster_2d=True, use_bg_nerf=True, bg_hidden=32,
                       occ_conf=occ, expert_box_list=[SceneBox(aabb=z[f"box{k}"]) for k in range(K)], **KW)
    state = {k[len("soft_w/"):]: v for k, v in z.items() if k.startswith("soft_w/")}
    mc.load_reference_state(state).to(DEV).eval()
    g = torch.Generator().manual_seed(seed + 1)
    for sub in mc.submodules:
        sub.occ_grid.binaries.copy_((torch.rand(sub.occ_grid.binaries.shape, generator=g) < 0.5).to(torch.uint8).to(DEV))
    return mc


def _capture_packed(fn):
    """Run fn() capturing the inputs of occupancy.render_packed (the merged packed segments)."""
    import nerf_amd.occupancy as occmod
    cap = {}
    orig = occmod.render_packed

    def spy(rs, t0, t1, offs, bg=None):
        cap.update(rs=rs.detach().cpu(), t0=t0.cpu(), t1=t1.cpu(), offs=offs.cpu(), bg=bg.detach().cpu())
        return orig(rs, t0, t1, offs, bg)

    occmod.render_packed = spy
    try:
        out = fn()
    finally:
        occmod.render_packed = orig
    return out, cap


def _occ_rays(n, seed):
    g = torch.Generator().manual_seed(seed)
    o = torch.tensor([0.1, -3.0, 0.3]).expand(n, 3)
    d = torch.nn.functional.normalize(torch.randn(n, 3, generator=g) * 0.4 + torch.tensor([0.0, 1.0, 0.0]), dim=-1)
    return torch.cat([o, d, torch.full((n, 1), 0.5), torch.full((n, 1), 6.0)], -1).to(DEV)


def test_segments_union_vs_torch_unique(z):
    """The GPU per-ray union of the experts' segments equals _merge_segments_union (torch.unique per ray,
    nerfs/ray_rendering.py:193-258) applied to the same per-expert segments — exactly."""
    from nerf_amd import container as C
    mc = _occ_container(z)
    n = 96
    rays = _occ_rays(n, 3)
    (rgb, depth, w, acc), cap = _capture_packed(lambda: C.render_container_occ(mc, rays))
    per_ri, per_t0, per_t1 = [], [], []
    r = rays.cpu()
    for ex in mc.submodules:
        lo, hi = torch.tensor(ex._aabb_host[:3]), torch.tensor(ex._aabb_host[3:])
        inv = torch.where(r[:, 3:6].abs() > 1e-9, 1.0 / r[:, 3:6], torch.full_like(r[:, 3:6], 1e9))
        ta, tb = (lo - r[:, :3]) * inv, (hi - r[:, :3]) * inv
        hit = torch.minimum(torch.maximum(ta, tb).amin(-1), r[:, 7]) > torch.maximum(torch.minimum(ta, tb).amax(-1),
                                                                                     r[:, 6])
        hidx = hit.nonzero().squeeze(1)
        if hidx.numel() == 0:
            continue
        ri, t0, t1, _ = ex.occupancy_marching_packed(rays[hidx.to(DEV)])
        per_ri.append(hidx[ri.cpu().long()])
        per_t0.append(t0.cpu())
        per_t1.append(t1.cpu())
    ri, t0, t1 = torch.cat(per_ri), torch.cat(per_t0), torch.cat(per_t1)
    ref0, ref1 = [], []
    for ray in range(n):
        sel = ri == ray
        if sel.any():
            b = torch.unique(torch.cat([t0[sel], t1[sel]]), sorted=True)
            ref0.append(b[:-1])
            ref1.append(b[1:])
    assert torch.equal(cap["t0"], torch.cat(ref0)) and torch.equal(cap["t1"], torch.cat(ref1))
    assert torch.isfinite(rgb).all() and float(acc.max()) <= 1.0 + 1e-5


def test_container_occ_render_vs_oracle(z):
    """Full-container occupancy rendering (eval: no jitter / filtering) vs the oracle chain on the SAME merged
    segments: route at midpoints, evaluate the routed experts, blend sigma/rgb before the packed integration
    (ray_rendering.py:441-481)."""
    from nerf_amd.ray_rendering import render_rays
    from oracle import occ_oracle as OO
    mc = _occ_container(z, 5)
    n = 64
    rays = _occ_rays(n, 6)
    (rgb, depth, w, acc), cap = _capture_packed(lambda: render_rays(mc, rays, ray_samples=64))
    p = {k[len("soft_w/"):]: v for k, v in z.items() if k.startswith("soft_w/")}
    res, _ = NO.hash_resolutions(4, 8, 128)
    exps = []
    for k in range(K):
        pre = f"submodules.{k}."
        pk = OrderedDict((nm[len(pre):], v) for nm, v in p.items() if nm.startswith(pre))
        tb = pk.pop("xyz_encoder.hash_table")
        exps.append(lambda x_d, pk=pk, tb=tb, box=z[f"box{k}"]: NO.ngp_forward(pk, tb, x_d, box, res, 10, 2,
                                                                               sigma_depth=1, color_depth=1))
    offs = cap["offs"].long()
    ri = torch.repeat_interleave(torch.arange(n), offs[1:] - offs[:-1])
    t0, t1 = cap["t0"], cap["t1"]
    r = rays.cpu()
    tm = 0.5 * (t0 + t1)
    xm = torch.cat([r[ri, :3] + r[ri, 3:6] * tm[:, None], r[ri, 3:6]], -1)
    Wt, _ = MO.routing(xm[:, :3], z["centroids"], 1.05, True)
    SIG = torch.zeros(xm.shape[0], K)
    RGB = torch.zeros(xm.shape[0], K, 3)
    for k in range(K):
        sel = (Wt[:, k] > 1e-8).nonzero().squeeze(1)
        if sel.numel():
            y = exps[k](xm[sel])
            SIG[sel, k] = y[:, 3]
            RGB[sel, k] = y[:, :3]
    s_num = (Wt * SIG).sum(1, keepdim=True).clamp_min(1e-12)
    rgb_mix = (Wt[..., None] * SIG[..., None] * RGB).sum(1) / s_num
    rs_ref = torch.cat([rgb_mix, s_num], -1)
    assert _err(cap["rs"], rs_ref) <= 1e-4 * max(1.0, rs_ref.abs().max().item())
    ref = OO.render_packed(rs_ref, t0, t1, ri, n, cap["bg"])
    for a, b, what in ((rgb, ref[0], "rgb"), (depth, ref[1], "depth"), (acc, ref[3], "acc")):
        assert _err(a, b) <= 1e-4 * max(1.0, b.abs().max().item()), what


def test_container_occ_training_gradients(z):
    """Training-mode container occupancy rendering: finite, non-zero gradients for every expert's MLP and
    hash table and the background MLP."""
    mc = _occ_container(z, 7).train()
    from nerf_amd.ray_rendering import render_rays
    rays = _occ_rays(128, 8)
    rgb, depth, w, acc = render_rays(mc, rays, ray_samples=64)
    ((rgb - 0.3) ** 2).mean().backward()
    for n_, p in mc.named_parameters():
        if p.grad is None:
            continue
        assert torch.isfinite(p.grad).all(), n_
    assert float(mc.bg_mlp[0].weight.grad.abs().sum()) > 0
    assert sum(float(s.xyz_encoder.hash_table.grad.abs().sum()) > 0 for s in mc.submodules
               if s.xyz_encoder.hash_table.grad is not None) >= 1


@pytest.mark.parametrize("train", [False, True])
def test_staged_march_equals_two_pass_march(z, train):
    """nerf_occ_march_multi_staged (count pass keeps the first cap segments, emit pass copies them, longer pairs are
    marched again) produces exactly the two-pass march's packed segments — with no overflow (cap 512) and with
    nearly every pair overflowing (cap 1, 3)."""
    import ctypes
    from nerf_amd import container as C
    from nerf_amd._lib import lib, ptr, stream
    from nerf_amd.occupancy import exclusive_scan
    mc = _occ_container(z, 2)
    subs = list(mc.submodules)
    n = 80
    rays = _occ_rays(n, 9)
    Kx = len(subs)
    grids = (type(subs[0].occ_grid.grid) * Kx)(*[ex.occ_grid.grid for ex in subs])
    bins = (ctypes.c_void_p * Kx)(*[ex.occ_grid.binaries.data_ptr() for ex in subs])
    boxes = (ctypes.c_float * (6 * Kx))(*[float(v) for ex in subs for v in ex._aabb_host])
    steps = (ctypes.c_float * Kx)(*[float(ex.render_step_size) for ex in subs])
    args = (grids, bins, boxes, steps, Kx, ptr(rays), n, float(subs[0].near_plane), float(subs[0].far_plane), 0.004,
            int(train), ctypes.c_uint64(1234), 8192)
    L = lib()
    counts = torch.empty(Kx * n, dtype=torch.int32, device=DEV)
    assert L.nerf_occ_march_multi(*args, ptr(counts), None, None, None, None, stream()) == 0
    offs = exclusive_scan(counts)
    M = int(offs[-1])
    assert M > 0 and int(counts.max()) > 3
    ref = [torch.empty(M, dtype=dt, device=DEV) for dt in (torch.int32, torch.float32, torch.float32)]
    assert L.nerf_occ_march_multi(*args, None, ptr(offs), *[ptr(t) for t in ref], stream()) == 0
    for cap in (512, 3, 1):
        c2 = torch.full_like(counts, -7)
        stage = torch.empty(Kx * n * cap * 2, dtype=torch.float32, device=DEV)
        assert L.nerf_occ_march_multi_staged(*args, ptr(c2), ptr(stage), cap, None, None, None, None, stream()) == 0
        assert torch.equal(c2, counts), cap
        out = [torch.full((M,), -5, dtype=dt, device=DEV) for dt in (torch.int32, torch.float32, torch.float32)]
        assert L.nerf_occ_march_multi_staged(*args, ptr(c2), ptr(stage), cap, ptr(offs), *[ptr(t) for t in out],
                                             stream()) == 0
        for a, b in zip(out, ref):
            assert torch.equal(a, b), cap
    assert L.nerf_occ_march_multi_staged(*args, ptr(counts), ptr(stage), 0, None, None, None, None, stream()) < 0


# ------------------------------------------------------------------ device-sized (sync-free) container step

PROD_KW = dict(hidden=64, sigma_depth=2, color_hidden=64, color_depth=2, dir_encoding="spherical",
               hash_enc_conf=dict(levels=16, features_per_level=2, log2_hashmap_size=14, min_res=16, max_res=512,
                                  interpolation="Linear"))


def _prod_container(seed=0):
    """A production-shape container (the fused NGP kernels' shape: 16 x 2 hash features, 2 x 64 trunk, 2 x 64 colour,
    SH directions; smaller tables and grids) with random occupancy — the shape the device-sized path runs on."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from nerf_amd.container import MetaContainer
    from nerf_amd.ray_sampling import SceneBox
    torch.manual_seed(seed)
    boxes, cents = [], []
    for sy in (-1, 1):
        for sz in (-1, 1):
            lo = torch.tensor([-1.5, -1.5 if sy < 0 else -0.1, -1.5 if sz < 0 else -0.1])
            hi = torch.tensor([1.5, 0.1 if sy < 0 else 1.5, 0.1 if sz < 0 else 1.5])
            boxes.append(SceneBox(aabb=torch.stack([lo, hi])))
            cents.append([0.0, 0.75 * sy, 0.75 * sz])
    occ = {"use_occ": True, "resolution": 16, "levels": 2, "occ_ready": True, "near_plane": 0.05,
           "alpha_thre": 1e-3, "cone_angle": 0.004}
    mc = MetaContainer(num_submodules=4, centroids=torch.tensor(cents), aabb=torch.tensor([[-1.5] * 3, [1.5] * 3]),
                       nerf_variant="instant", boundary_margin=1.05, cluster_2d=True, use_bg_nerf=True, bg_hidden=32,
                       occ_conf=occ, expert_box_list=boxes, **PROD_KW).to(DEV)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for sub in mc.submodules:
            sub.occ_grid.binaries.copy_((torch.rand(sub.occ_grid.binaries.shape, generator=g) < 0.6).to(torch.uint8))
            sub.xyz_encoder.hash_table.mul_(100.0)   # densities well away from zero: the visibility filter bites
    return mc


def _render_loss(mc, rays, seed, gt):
    from nerf_amd.ray_rendering import render_rays
    mc.zero_grad(set_to_none=True)
    torch.manual_seed(seed)                      # the march jitter seed is drawn from torch's CPU generator
    rgb, depth, w, acc = render_rays(mc, rays, ray_samples=64)
    loss = ((rgb - gt) ** 2).mean()
    loss.backward()
    grads = {n: p.grad.detach().clone() for n, p in mc.named_parameters() if p.grad is not None}
    return rgb.detach(), depth.detach(), w.detach(), acc.detach(), loss.detach(), grads


@pytest.mark.parametrize("train", [True, False])
def test_container_device_sized_equals_host_sized(train):
    """The sync-free container step (every size after the march read on the device, capacity-sized buffers) against
    the host-sized step on the same rays and jitter seed: rgb / depth / acc and the packed weights bitwise equal;
    parameter gradients equal up to the MLP weight-gradient slab partition (the persistent grid follows the
    capacity) and the hash scatter's atomic order — 1e-5 of each tensor's scale."""
    from nerf_amd import container as C
    mc = _prod_container(3).train(train)
    mc.device_sized = True
    rays = _occ_rays(1024, 12)
    gt = torch.rand(1024, 3, generator=torch.Generator().manual_seed(4)).to(DEV)
    _render_loss(mc, rays, 1, gt)                # first call: host-sized, seeds the capacity
    sizes = mc.__dict__["_dev_sizes"]
    assert sizes.calls == 0 and sizes.max_seen > 0
    calls = []
    orig = C._render_container_occ_dev
    C._render_container_occ_dev = lambda *a, **k: calls.append(1) or orig(*a, **k)
    try:
        dev_out = _render_loss(mc, rays, 7, gt)
    finally:
        C._render_container_occ_dev = orig
    assert calls, "the device-sized path did not run"
    mc.device_sized = False
    host_out = _render_loss(mc, rays, 7, gt)
    torch.cuda.synchronize()
    sizes.poll()
    assert sizes.overflows == 0 and sizes.calls == 1
    for a, b, what in zip(dev_out[:4], host_out[:4], ("rgb", "depth", "weights", "acc")):
        if what == "weights":
            a = a[:b.shape[0]]                   # capacity rows: the first M are the packed samples
        assert torch.equal(a, b), (what, (a - b).abs().max().item())
    assert torch.equal(dev_out[4], host_out[4])
    gd, gh = dev_out[5], host_out[5]
    assert set(gd) == set(gh) and len(gh) > 0
    for n_ in gh:
        scale = max(gh[n_].abs().max().item(), 1e-30)
        err = (gd[n_] - gh[n_]).abs().max().item()
        assert err <= 1e-5 * scale, (n_, err, scale)
    assert any(float(gh[n_].abs().sum()) > 0 for n_ in gh if "hash_table" in n_)


def test_container_device_sized_overflow_is_counted():
    """A capacity below the step's march count keeps the first CAP samples (finite outputs, no fault) and is counted
    once its count reaches the host; the next call's capacity covers the count."""
    from nerf_amd.ray_rendering import render_rays
    mc = _prod_container(5).train()
    mc.device_sized = True
    rays = _occ_rays(512, 13)
    torch.manual_seed(0)
    render_rays(mc, rays, ray_samples=64)         # seeds _dev_sizes
    sizes = mc.__dict__["_dev_sizes"]
    total = sizes.max_seen
    sizes.min_cap, sizes.cap, sizes.max_seen = 1, 256, 0
    assert total > 256
    torch.manual_seed(1)
    rgb, depth, w, acc = render_rays(mc, rays, ray_samples=64)
    ((rgb - 0.5) ** 2).mean().backward()
    torch.cuda.synchronize()
    assert torch.isfinite(rgb).all() and torch.isfinite(depth).all()
    cap = sizes.poll()
    assert sizes.overflows == 1 and cap >= 2 * (total // 2)
