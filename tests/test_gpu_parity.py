"""HIP path vs the reference golden vectors and the CPU oracle (run on an MI355X: -m gpu).

Tolerance contract (BASELINE.json north_star): outputs within 1e-4 (fp32) of the reference CPU path.
Gradients are compared with a tolerance relative to their scale (atol = 1e-4 * max|ref|)."""
import math

import pytest
import torch

from golden_io import load, mlp_params
from oracle import nerf_oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda"
TOL = 1e-4


def _close(a, b, atol=TOL, rel_scale=False, what=""):
    a = a.detach().float().cpu()
    b = b.detach().float().cpu()
    assert a.shape == b.shape, (what, a.shape, b.shape)
    tol = atol * max(1.0, b.abs().max().item()) if rel_scale else atol
    same = (a == b) | (torch.isnan(a) & torch.isnan(b))
    err = torch.where(same, torch.zeros_like(a), (a - b).abs()).max().item() if a.numel() else 0.0
    assert err <= tol, f"{what}: max err {err:.3e} > {tol:.3e}"
    return err


@pytest.fixture(scope="module")
def K():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from nerf_amd import kernels
    return kernels


# ------------------------------------------------------------------ encoding / rays / sampling


def test_freq_encode(K):
    z = load("freq")
    _close(K.freq_encode(z["x"].to(DEV), 10), z["enc_x"], 1e-5, what="xyz PE")
    _close(K.freq_encode(z["d"].to(DEV), 4), z["enc_d"], 1e-5, what="dir PE")
    _close(K.freq_encode(z["small_in"].to(DEV), 2), z["small_out"], 1e-6, what="PE known answer")


def test_rays(K):
    from nerf_amd.ray_sampling import get_ray_directions, rays_for_camera, SceneBox, clamp_rays_near_far
    z = load("rays")
    f = float(z["focal"])
    dirs = get_ray_directions(800, 800, f, f, 400.0, 400.0, True, DEV)
    _close(dirs[350:450, 350:450], z["dirs_crop"], 1e-6, what="directions")
    rays = rays_for_camera(800, 800, f, f, 400.0, 400.0, z["c2w"].to(DEV), near=2.0, far=6.0).view(800, 800, 8)
    _close(rays[350:450, 350:450].reshape(-1, 8), z["rays_const"], 2e-6, what="rays const near/far")
    box = SceneBox(aabb=torch.tensor([[-1.5, -1.5, -1.5], [1.5, 1.5, 1.5]], device=DEV))
    ra = rays_for_camera(24, 40, 30.0, 28.0, 19.3, 12.1, z["c2w_b"].to(DEV), scene_box=box)
    _close(ra, z["rays_aabb"], 1e-5, rel_scale=False, what="rays aabb")
    cl, valid = clamp_rays_near_far(ra, (0.5, 4.0))
    _close(cl, z["clamped"], 1e-5, what="clamp")
    assert torch.equal(valid.cpu(), z["valid"])
    dn = get_ray_directions(7, 9, 5.0, 6.0, 4.0, 3.5, False, DEV)
    _close(dn, z["dirs_nc"], 1e-6, what="directions (no centring)")


def test_rays_batch_gather(K):
    g = torch.Generator().manual_seed(3)
    imgs = torch.randint(0, 256, (3, 10, 12, 3), dtype=torch.uint8, generator=g)
    poses = torch.stack([torch.eye(4)[:3] for _ in range(3)])
    poses[:, :, 3] = torch.randn(3, 3, generator=g)
    pix = K.pick_pixels(4096, 3, 10, 12, 123, DEV)
    assert pix[:, 0].min() >= 0 and pix[:, 0].max() < 3 and pix[:, 1].max() < 10 and pix[:, 2].max() < 12
    rays, rgb = K.rays_gen(poses.to(DEV), 10, 12, 9.0, 9.0, 6.0, 5.0, pix=pix, near=2.0, far=6.0,
                           images_u8=imgs.to(DEV))
    p = pix.long().cpu()
    _close(rgb, imgs[p[:, 0], p[:, 1], p[:, 2]].float() / 255.0, 1e-7, what="gt gather")
    dirs = O.get_ray_directions(10, 12, 9.0, 9.0, 6.0, 5.0, True)
    ref_d = torch.einsum("nij,nj->ni", poses[p[:, 0], :, :3], dirs[p[:, 1], p[:, 2]])
    _close(rays[:, 3:6], ref_d, 2e-6, what="batch directions")
    _close(rays[:, :3], poses[p[:, 0], :, 3], 0, what="batch origins")


def test_stratified(K):
    z = load("render")
    rays = z["rays"].to(DEV)
    t = K.sample_stratified(rays, 64, True, z["u"].to(DEV))
    _close(t, z["t_train"], 2e-6, what="stratified t")
    t_eval = K.sample_stratified(rays, 64, False)
    _close(t_eval, O.stratified_t_vals(z["rays"][:, 6], z["rays"][:, 7], 64, False), 1e-6, what="linspace t")
    tr = K.sample_stratified(rays, 64, True, None, seed=5)
    assert (tr[:, 1:] >= tr[:, :-1]).all() and (tr >= 2.0).all() and (tr <= 6.0).all()


def test_ndc(K):
    g = torch.Generator().manual_seed(1)
    rays = torch.cat([torch.randn(256, 2, generator=g) * 0.3, torch.full((256, 1), 4.0),
                      torch.nn.functional.normalize(torch.randn(256, 3, generator=g) * 0.2 + torch.tensor([0, 0, -1.0]), dim=-1),
                      torch.zeros(256, 2)], -1)
    _close(K.rays_ndc(rays.to(DEV), 756, 1008, 815.0, 1.0), O.ndc_rays(756, 1008, 815.0, 1.0, rays), 1e-5, what="ndc")


# ------------------------------------------------------------------ compositing


@pytest.mark.parametrize("tag", ["s64", "s192"])
def test_volume_render(K, tag):
    from nerf_amd.ray_rendering import volume_render
    z = load("volume_render")
    rs = z[f"{tag}/rgbs"].to(DEV).requires_grad_(True)
    t = z[f"{tag}/t"].to(DEV)
    bg = torch.ones(t.shape[0], 3, device=DEV)
    rgb, d, w, a = volume_render(rs, t, bg)
    _close(rgb, z[f"{tag}/rgb"], what="rgb")
    _close(d, z[f"{tag}/depth"], what="depth")
    _close(w, z[f"{tag}/w"], what="weights")
    _close(a, z[f"{tag}/acc"], what="acc")
    L = ((rgb * z[f"{tag}/g_rgb"].to(DEV)).sum() + (d * z[f"{tag}/g_d"].to(DEV)).sum()
         + (a * z[f"{tag}/g_a"].to(DEV)).sum() + (w * z[f"{tag}/g_w"].to(DEV)).sum())
    g, = torch.autograd.grad(L, rs)
    _close(g, z[f"{tag}/grad_all"], rel_scale=True, what="d rgb_sigma")


def test_composite_fused_loss(K):
    z = load("volume_render")
    rs, t = z["s64/rgbs"], z["s64/t"]
    gt = torch.rand(t.shape[0], 3, generator=torch.Generator().manual_seed(2))
    for cs in ("linear", "srgb", "identity"):
        rsr = rs.clone().requires_grad_(True)
        rgb = O.volume_render(rsr, t, torch.ones(t.shape[0], 3))[0]
        loss = O.mse_loss(rgb, gt, cs)
        g_ref, = torch.autograd.grad(loss, rgb)
        out = K.composite_fwd(rs.to(DEV), t.to(DEV), torch.ones(t.shape[0], 3, device=DEV), gt=gt.to(DEV),
                              color_space=cs)
        assert abs(out[4].item() - loss.item()) < 1e-6 + 1e-5 * loss.item(), cs
        _close(out[5], g_ref, 1e-6, what=f"d loss/d rgb ({cs})")


def test_composite_edges(K):
    # S = 2, single ray, empty batch, ragged S, all-transparent and all-opaque rays
    for S in (2, 3, 65, 129, 200):
        n = 5
        g = torch.Generator().manual_seed(S)
        t = torch.sort(torch.rand(n, S, generator=g) * 4 + 2, -1)[0]
        rs = torch.rand(n, S, 4, generator=g)
        rs[0, :, 3] = 0.0
        rs[1, :, 3] = 1e5
        rsr = rs.clone().requires_grad_(True)
        ref = O.volume_render(rsr, t, None)
        gr = torch.randn(n, 3, generator=g)
        gref, = torch.autograd.grad((ref[0] * gr).sum() + ref[1].sum(), rsr)
        out = K.composite_fwd(rs.to(DEV), t.to(DEV), None)
        for a, b in zip(out, ref):
            _close(a, b, what=f"S={S} fwd")
        d = K.composite_bwd(rs.to(DEV), t.to(DEV), None, gr.to(DEV), torch.ones(n, device=DEV))
        _close(d, gref, rel_scale=True, what=f"S={S} bwd")
    e = K.composite_fwd(torch.zeros(0, 4, 4, device=DEV), torch.zeros(0, 4, device=DEV), None)
    assert e[0].shape == (0, 3)


# ------------------------------------------------------------------ MLP


@pytest.fixture(scope="module")
def net(K):
    from nerf_amd.vanilla import VanillaNeRF
    return VanillaNeRF().load_reference_state(mlp_params("w/")).to(DEV)


def test_mlp_forward_backward_golden(net):
    z = load("mlp")
    out = net(z["x_d"].to(DEV))
    _close(out, z["out"], what="mlp forward")
    net.zero_grad()
    (out * z["gup"].to(DEV)).sum().backward()
    ref = mlp_params("g/")
    for n, p in net.named_parameters():
        _close(p.grad, ref[n], rel_scale=True, what=f"grad {n}")


def test_mlp_ragged_and_fast_weights(net):
    # M not a multiple of the 256-row tile, fast-weights dict replacing a subset of tensors
    p = mlp_params("w/")
    g = torch.Generator().manual_seed(9)
    for M in (1, 7, 255, 257, 1000):
        x_d = torch.cat([torch.rand(M, 3, generator=g) * 4 - 2,
                         torch.nn.functional.normalize(torch.randn(M, 3, generator=g), dim=-1)], -1)
        _close(net(x_d.to(DEV)), O.vanilla_forward(p, x_d), what=f"mlp M={M}")
    fast = {k: (v * 1.01).to(DEV).requires_grad_(True) for k, v in p.items() if k.startswith("trunk.3")}
    x_d = torch.cat([torch.rand(300, 3, generator=g), torch.nn.functional.normalize(torch.randn(300, 3, generator=g), dim=-1)], -1)
    out = net(x_d.to(DEV), params=fast)
    pf = dict(p)
    pf.update({k: v.detach().cpu().requires_grad_(True) for k, v in fast.items()})
    ref = O.vanilla_forward(pf, x_d)
    _close(out, ref, what="fast-weights forward")
    gs = torch.autograd.grad(out.sum(), list(fast.values()))
    gr = torch.autograd.grad(ref.sum(), [pf[k] for k in fast])
    for a, b in zip(gs, gr):
        _close(a, b, rel_scale=True, what="fast-weights grad")


def _kink_rows(p64, x_d64, eps):
    """Rows with any ReLU pre-activation within eps of 0 in the fp64 oracle forward (test infrastructure: records
    the inputs of the oracle's torch.relu calls)."""
    seen = []
    relu = torch.relu

    def rec(x):
        seen.append(x.detach().abs().amin(dim=-1))
        return relu(x)

    torch.relu = rec
    try:
        O.vanilla_forward(p64, x_d64)
    finally:
        torch.relu = relu
    return torch.stack(seen, 1).amin(1) < eps


def test_mlp_backward_multi_split_ragged(net):
    """Weight gradients at sizes with several split-M slabs (S = Mp / 2048): M = 9000 (S = 4) and M = 40001
    (S = 19, rows per split 2176 -> the last split is short and the second half of its colour-backward pair is
    empty).  Exercises the narrow wgrad tiles (32 / 64-row slabs), the two-workgroup colour backward with its
    side buffer and the folded split reduce against the oracle's autograd in fp64; a second run must be
    bitwise identical (fixed reduction order, no atomics).

    ReLU boundary flips: a pre-activation within rounding of 0 passes the gradient in one evaluation and
    blocks it in another (the fp32 GPU forward vs the fp64 oracle), so that row's term enters one gradient and
    not the other.  Rows with any pre-activation within 2e-6 of 0 in the fp64 forward (~4 % of the rows; fp32
    pre-activations sit within 1.1e-6 of the fp64 ones) get a zero output gradient in BOTH evaluations; every
    other row is compared at the north-star 1e-4 of scale (a dropped split or 16-row sub-slab moves the
    gradient far beyond that)."""
    p = mlp_params("w/")
    g = torch.Generator().manual_seed(21)
    for M in (9000, 40001):
        x_d = torch.cat([torch.rand(M, 3, generator=g) * 4 - 2,
                         torch.nn.functional.normalize(torch.randn(M, 3, generator=g), dim=-1)], -1)
        gout = torch.randn(M, 4, generator=g)
        p64 = {k: v.double().requires_grad_(True) for k, v in p.items()}
        kink = _kink_rows({k: v.detach() for k, v in p64.items()}, x_d.double(), 2e-6)
        assert kink.float().mean().item() < 0.1, "too many rows near a ReLU kink"
        gout[kink] = 0.0
        fast = {k: v.to(DEV).requires_grad_(True) for k, v in p.items()}
        runs = []
        for _ in range(2):
            out = net(x_d.to(DEV), params=fast)
            runs.append(torch.autograd.grad((out * gout.to(DEV)).sum(), list(fast.values())))
        ref = O.vanilla_forward(p64, x_d.double())
        gr = torch.autograd.grad((ref * gout.double()).sum(), [p64[k] for k in fast])
        for k, a, a2, b in zip(fast, runs[0], runs[1], gr):
            assert torch.equal(a, a2), f"M={M} {k}: backward not bitwise reproducible"
            _close(a, b, rel_scale=True, what=f"M={M} grad {k} ({int(kink.sum())} kink rows excluded)")


def test_mlp_inference_equals_training_forward(net, K):
    g = torch.Generator().manual_seed(4)
    x_d = torch.cat([torch.rand(5000, 3, generator=g) * 4 - 2,
                     torch.nn.functional.normalize(torch.randn(5000, 3, generator=g), dim=-1)], -1).to(DEV)
    w = net.packed().detach()
    a = K.mlp_fwd(w, x_d, K.mlp_workspace(5000, True, DEV), True)
    b = K.mlp_fwd(w, x_d, K.mlp_workspace(5000, False, DEV), False)
    assert torch.equal(a, b)


# ------------------------------------------------------------------ render_rays end to end


def test_render_rays_golden(net):
    from nerf_amd.ray_rendering import render_rays
    z = load("render")
    rays = z["rays"].to(DEV)
    net.eval()
    with torch.no_grad():
        rgb, d, w, a = render_rays(net, rays, ray_samples=64)
    _close(rgb, z["e_rgb"], what="eval rgb")
    _close(d, z["e_depth"], what="eval depth", rel_scale=True)
    _close(w, z["e_w"], what="eval weights")
    _close(a, z["e_acc"], what="eval acc")
    net.train()
    with torch.no_grad():
        rgb, d, w, a = render_rays(net, rays, ray_samples=64, u_strat=z["u"].to(DEV))
    _close(rgb, z["t_rgb"], what="train rgb")
    _close(w, z["t_w"], what="train weights")
    net.eval()


def test_c1_crop_render_full_size(net):
    """BASELINE configs[0] (C1) at its stated size: the 100x100 centre crop of an 800x800 Lego-style camera (10,000
    rays, the golden `rays_const` crop), 64 coarse samples, coarse-only MLP, through render_rays on the GPU against
    the pinned oracle (an/nerfs/ray_rendering.py:290-345) at the north-star 1e-4: eval mode (linspace t) and train
    mode with an injected stratified draw, plus the train-mode MSE gradients of every parameter (1e-4 of scale)."""
    from nerf_amd.ray_rendering import render_rays
    from nerf_amd.ray_sampling import rays_for_camera
    z = load("rays")
    f = float(z["focal"])
    rays = rays_for_camera(800, 800, f, f, 400.0, 400.0, z["c2w"].to(DEV), near=2.0, far=6.0).view(800, 800, 8)
    rays = rays[350:450, 350:450].reshape(-1, 8).contiguous()
    assert rays.shape == (10000, 8)
    _close(rays, z["rays_const"], 2e-6, what="C1 crop rays")
    p = mlp_params("w/")
    rays_c = rays.cpu()
    net.eval()
    with torch.no_grad():
        rgb, d, w, a = render_rays(net, rays, ray_samples=64)
    ref = O.render_rays(p, rays_c, 64, training=False)
    _close(rgb, ref[0], what="C1 eval rgb")
    _close(d, ref[1], what="C1 eval depth", rel_scale=True)
    _close(w, ref[2], what="C1 eval weights")
    _close(a, ref[3], what="C1 eval acc")
    net.train()
    u = torch.rand(10000, 64, generator=torch.Generator().manual_seed(100))
    gt = torch.rand(10000, 3, generator=torch.Generator().manual_seed(101))
    net.zero_grad()
    rgb, d, w, a = render_rays(net, rays, ray_samples=64, u_strat=u.to(DEV))
    torch.nn.functional.mse_loss(rgb, gt.to(DEV)).backward()
    pr = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    ref = O.render_rays(pr, rays_c, 64, training=True, u_strat=u)
    torch.nn.functional.mse_loss(ref[0], gt).backward()
    _close(rgb, ref[0], what="C1 train rgb")
    _close(d, ref[1], what="C1 train depth", rel_scale=True)
    _close(w, ref[2], what="C1 train weights")
    for n, q in net.named_parameters():
        _close(q.grad, pr[n].grad, rel_scale=True, what=f"C1 train grad {n}")
    net.eval()


def test_sample_pdf_vs_oracle(K):
    g = torch.Generator().manual_seed(11)
    N, S, NI = 300, 64, 128
    t = torch.sort(torch.rand(N, S, generator=g) * 4 + 2, -1)[0]
    w = torch.rand(N, S, generator=g) ** 4
    w[0] = 0.0          # all-zero weights -> uniform pdf
    w[1] = 0.0
    w[1, 30] = 1.0      # one-hot
    u = torch.rand(N, NI, generator=g)
    out = K.sample_pdf(t.to(DEV), w.to(DEV), NI, u=u.to(DEV))
    ref = O.hierarchical_t_vals(t, w, NI, u=u)
    _close(out, ref, 1e-5, what="merged t (random u)")
    out = K.sample_pdf(t.to(DEV), w.to(DEV), NI, det=True)
    ref = O.hierarchical_t_vals(t, w, NI, det=True)
    _close(out, ref, 1e-5, what="merged t (det)")
    r = K.sample_pdf(t.to(DEV), w.to(DEV), NI, seed=1)
    assert (r[:, 1:] >= r[:, :-1]).all()
    for S2, NI2 in ((3, 1), (64, 64), (100, 156), (128, 384)):
        t2 = torch.sort(torch.rand(7, S2, generator=g) * 4 + 2, -1)[0]
        w2 = torch.rand(7, S2, generator=g)
        u2 = torch.rand(7, NI2, generator=g)
        _close(K.sample_pdf(t2.to(DEV), w2.to(DEV), NI2, u=u2.to(DEV)), O.hierarchical_t_vals(t2, w2, NI2, u=u2),
               1e-5, what=f"merged S={S2} NI={NI2}")


def test_hierarchical_render_vs_oracle(K):
    from nerf_amd.vanilla import VanillaNeRF
    from nerf_amd.ray_rendering import render_rays
    pc = O.init_vanilla_params(1)
    pf = O.init_vanilla_params(2)
    coarse = VanillaNeRF().load_reference_state(pc).to(DEV).eval()
    fine = VanillaNeRF().load_reference_state(pf).to(DEV).eval()
    z = load("render")
    rays = z["rays"]
    with torch.no_grad():
        rgb, d, w, a, ex = render_rays(coarse, rays.to(DEV), ray_samples=64, n_importance=128, fine_model=fine,
                                       return_extras=True)
    ref = O.render_rays(pc, rays, 64, training=False, p_fine=pf, n_importance=128)
    _close(ex["t_fine"], ref[4]["t_fine"], 1e-5, what="t_fine")
    _close(rgb, ref[0], what="fine rgb")
    _close(w, ref[2], what="fine weights")
    _close(d, ref[1], what="fine depth", rel_scale=True)


# ------------------------------------------------------------------ train steps


def _adam_step1_close(p, ref, g, g_ref, lr, what, eps=1e-8):
    """Post-Adam parameters after ONE step from the same start point.  Adam's first update is
    -lr * g/(|g|+eps) per element, so two gradients that agree to rounding level can still move an
    element whose gradient is at the noise floor by up to 2 lr.  The allowed deviation per element is
    exactly the update difference the two measured gradients imply, plus fp32 rounding."""
    p, ref = p.detach().double().cpu(), ref.detach().double().cpu()
    g, g_ref = g.detach().double().cpu(), g_ref.detach().double().cpu()
    phi = lambda x: x / (x.abs() + eps)
    bound = lr * (phi(g) - phi(g_ref)).abs() * 1.02 + 1e-6 * lr + 2.5e-7 * (1 + ref.abs())
    err = (p - ref).abs()
    bad = err > bound
    assert not bad.any(), f"{what}: {int(bad.sum())} elements beyond the implied bound, max err {err.max():.3e}"


def test_train_step_golden(net):
    """Reference runtime_adapt train step (runtime_adapt.py:286-310): autograd through the HIP ops,
    MSE in linear colour space, clip_grad_norm_(1.0), torch Adam — vs the reference's golden step."""
    from nerf_amd import ray_rendering as rr
    from nerf_amd.losses import color_space_transformer
    from nerf_amd.vanilla import VanillaNeRF
    z, zr = load("train_step"), load("render")
    m = VanillaNeRF().load_reference_state(mlp_params("w/")).to(DEV).train()
    grp = m.get_param_groups()
    opt = torch.optim.Adam([{"params": grp["sigma"]["params"], "lr": 2e-3}, {"params": grp["color"]["params"], "lr": 2e-3}])
    opt.zero_grad()
    out = rr.render_rays(m, zr["rays"].to(DEV), ray_samples=64, chunk=4096, u_strat=zr["u"].to(DEV))
    a, b = color_space_transformer(out[0], z["gt"].to(DEV), "linear")
    loss = torch.nn.functional.mse_loss(a, b)
    assert abs(loss.item() - float(z["loss"])) < 1e-5
    loss.backward()
    gn = torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0)
    assert abs(gn.item() - float(z["gnorm"])) < 1e-4 * float(z["gnorm"])
    # the same step through the CPU oracle (itself pinned to this golden step in test_oracle_golden.py)
    ot = O.OracleTrainer(mlp_params("w/"), lr_sigma=2e-3, lr_color=2e-3)
    lref = ot.step(zr["rays"], z["gt"], 64, training=True, u_strat=zr["u"])
    assert abs(lref - float(z["loss"])) < 1e-6
    named = dict(m.named_parameters())
    for n, p in named.items():
        _close(p.grad, ot.nets[0][n].grad, rel_scale=True, what=f"clipped grad {n}")
    opt.step()
    for n, p in named.items():
        _adam_step1_close(p, ot.nets[0][n], p.grad, ot.nets[0][n].grad, 2e-3, what=f"post-Adam {n}")
    for k, v in z.items():   # golden parameters: loose absolute bound (2 lr) + mean at rounding level
        if k.startswith("p/"):
            err = (named[k[2:]].detach().cpu() - v).abs()
            assert err.max() <= 4e-3 and err.mean() <= 5e-6, (k, err.max().item(), err.mean().item())


def test_engine_step_vs_oracle(K):
    """Fused engine (two nets, 64+128, fused loss, clip, HIP Adam) vs the oracle trainer on identical u:
    per-step loss over 3 steps, first-step clipped gradients and post-Adam parameters of both nets."""
    from nerf_amd.vanilla import VanillaNeRF, PackedLayout
    from nerf_amd.trainer import NeRFTrainer
    pc, pf = O.init_vanilla_params(1), O.init_vanilla_params(2)
    coarse = VanillaNeRF().load_reference_state(pc).to(DEV)
    fine = VanillaNeRF().load_reference_state(pf).to(DEV)
    tr = NeRFTrainer(coarse, fine, n_samples=64, n_importance=128, lr_sigma=2e-3, lr_color=1e-3)
    ot = O.OracleTrainer(pc, pf, lr_sigma=2e-3, lr_color=1e-3)
    L = PackedLayout.get()
    zr = load("render")
    rays = zr["rays"]
    g = torch.Generator().manual_seed(5)
    gt = torch.rand(rays.shape[0], 3, generator=g)
    for step in range(3):
        us = torch.rand(rays.shape[0], 64, generator=g)
        up = torch.rand(rays.shape[0], 128, generator=g)
        loss = tr.step(rays.to(DEV), gt.to(DEV), seed=step, u_strat=us.to(DEV), u_pdf=up.to(DEV)).item()
        lref = ot.step(rays, gt, 64, n_importance=128, training=True, u_strat=us, u_pdf=up)
        assert abs(loss - lref) < 1e-5 + 1e-4 * lref, (step, loss, lref)
        if step == 0:
            norm = tr.grads.double().norm().item()
            coef = min(1.0, 1.0 / (norm + 1e-6))
            for k in range(2):
                gk = L.unpack(tr.g(k).detach().cpu() * coef)
                pk = L.unpack(tr.w(k).detach().cpu())
                for n, v in gk.items():
                    _close(v, ot.nets[k][n].grad, rel_scale=True, what=f"net{k} grad {n}")
                    lr = 1e-3 if n.startswith("color_mlp") else 2e-3
                    _adam_step1_close(pk[n], ot.nets[k][n], v, ot.nets[k][n].grad, lr, what=f"net{k} {n} step 1")


def test_adam_kernel_matches_torch(K):
    g = torch.Generator().manual_seed(0)
    n = 10007
    p0 = torch.randn(n, generator=g)
    grads = [torch.randn(n, generator=g) * 3 for _ in range(4)]
    pt = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([{"params": [pt], "lr": 1e-3}], betas=(0.9, 0.999), eps=1e-8)
    p, m, v = p0.to(DEV), torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    for s, gr in enumerate(grads, 1):
        pt.grad = gr.clone()
        torch.nn.utils.clip_grad_norm_([pt], 1.0)
        opt.step()
        gd = gr.to(DEV)
        parts = K.grad_sqnorm(gd)
        K.adam(p, gd, m, v, [0, n], [1e-3], s, partials=parts, max_norm=1.0)
    _close(p, pt.detach(), 1e-6, what="adam")


# ------------------------------------------------------------------ full-size properties (C2 shapes)


def test_c2_scale_properties(K):
    """C2 sizes (4096 rays x 64+128): size-independent invariants of the full step."""
    from nerf_amd.vanilla import VanillaNeRF
    from nerf_amd.trainer import NeRFTrainer, RayBatcher
    from nerf_amd.scene import make_blender_scene
    scene = make_blender_scene(n_train=4, n_test=1, H=200, W=200, device=DEV)
    torch.manual_seed(0)
    tr = NeRFTrainer(VanillaNeRF().to(DEV), VanillaNeRF().to(DEV))
    rb = RayBatcher(scene, DEV)
    losses = []
    for s in range(6):
        rays, gt = rb.batch(4096, seed=s)
        losses.append(tr.step(rays, gt, seed=s).item())
    assert all(math.isfinite(l) for l in losses)
    assert torch.isfinite(tr.params).all()
    rays, gt = rb.batch(4096, seed=99)
    t = K.sample_stratified(rays, 64, True, None, 3)
    xd = K.build_xd(rays, t)
    rs = K.mlp_fwd(tr.w(0), xd, K.mlp_workspace(xd.shape[0], False, DEV), False)
    rgb, d, w, a = K.composite_fwd(rs, t, torch.ones(4096, 3, device=DEV))
    assert (a >= -1e-6).all() and (a <= 1 + 1e-5).all()
    torch.testing.assert_close(w.sum(1), a, rtol=1e-5, atol=1e-5)
    tf = K.sample_pdf(t, w, 128, seed=4)
    assert (tf[:, 1:] >= tf[:, :-1]).all()
    # every coarse t survives the merge (multiset union)
    assert torch.isin(t, tf).all()
