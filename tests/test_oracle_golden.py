"""Pin the CPU oracle (oracle/nerf_oracle.py) against golden vectors produced by importing the
reference itself (tools/gen_golden.py).  CPU only."""
import torch

from oracle import nerf_oracle as O
from golden_io import load, mlp_params

TOL = dict(rtol=0, atol=1e-6)


def test_freq_encoder_golden():
    z = load("freq")
    torch.testing.assert_close(O.freq_encode(z["x"], 10), z["enc_x"], **TOL)
    torch.testing.assert_close(O.freq_encode(z["d"], 4), z["enc_d"], **TOL)
    # SURVEY §8 a8 known answer: [x, cos f0..f1, sin f0..f1] per dim, dim-major
    torch.testing.assert_close(O.freq_encode(z["small_in"], 2), z["small_out"], **TOL)
    x = z["small_in"][0]
    ref = torch.cat([x, torch.stack([torch.cos(x[0]), torch.cos(2 * x[0]), torch.sin(x[0]), torch.sin(2 * x[0])])])
    torch.testing.assert_close(z["small_out"][0, :7], ref, **TOL)


def test_rays_golden():
    z = load("rays")
    f = float(z["focal"])
    dirs = O.get_ray_directions(800, 800, f, f, 400.0, 400.0, True)
    torch.testing.assert_close(dirs[350:450, 350:450], z["dirs_crop"], **TOL)
    rays = O.get_rays(z["dirs_crop"], z["c2w"], near=2.0, far=6.0).reshape(-1, 8)
    torch.testing.assert_close(rays, z["rays_const"], **TOL)
    ds = O.get_ray_directions(24, 40, 30.0, 28.0, 19.3, 12.1, True)
    torch.testing.assert_close(ds, z["dirs_small"], **TOL)
    aabb = torch.tensor([[-1.5, -1.5, -1.5], [1.5, 1.5, 1.5]])
    ra = O.get_rays(ds, z["c2w_b"], aabb=aabb).reshape(-1, 8)
    torch.testing.assert_close(ra, z["rays_aabb"], rtol=1e-6, atol=1e-5)
    assert (ra[:, 6] == 1e10).any() and (ra[:, 6] < 1e10).any()  # both hit and miss rays present
    cl, valid = O.clamp_rays_near_far(ra, (0.5, 4.0))
    torch.testing.assert_close(cl, z["clamped"], rtol=1e-6, atol=1e-5)
    assert torch.equal(valid, z["valid"])
    torch.testing.assert_close(O.get_ray_directions(7, 9, 5.0, 6.0, 4.0, 3.5, False), z["dirs_nc"], **TOL)


def test_mlp_forward_backward_golden():
    z = load("mlp")
    p = mlp_params("w/")
    assert sum(v.numel() for v in p.values()) == 503059
    for k, v in p.items():
        assert tuple(v.shape) == O.VANILLA_SHAPES[k], k
    pg = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    out = O.vanilla_forward(pg, z["x_d"])
    torch.testing.assert_close(out, z["out"], rtol=0, atol=2e-6)
    grads = torch.autograd.grad((out * z["gup"]).sum(), list(pg.values()))
    ref = mlp_params("g/")
    for (k, g), (k2, r) in zip(zip(pg.keys(), grads), ref.items()):
        assert k == k2
        torch.testing.assert_close(g, r, rtol=1e-4, atol=2e-5 * max(1.0, r.abs().max().item()))


def test_trunc_exp_golden():
    z = load("mlp")
    x = z["te_x"].clone().requires_grad_(True)
    y = O.trunc_exp(x)
    g, = torch.autograd.grad(y.sum(), x)
    torch.testing.assert_close(y, z["te_y"], **TOL)
    torch.testing.assert_close(g, z["te_g"], **TOL)
    assert g[-1] > 0  # gradient does not vanish beyond the clamp


def test_volume_render_golden():
    z = load("volume_render")
    for tag in ("s64", "s192"):
        rs = z[f"{tag}/rgbs"].clone().requires_grad_(True)
        t = z[f"{tag}/t"]
        bg = torch.ones(t.shape[0], 3)
        rgb, d, w, a = O.volume_render(rs, t, bg)
        for got, key in ((rgb, "rgb"), (d, "depth"), (w, "w"), (a, "acc")):
            torch.testing.assert_close(got, z[f"{tag}/{key}"], rtol=0, atol=2e-6)
        L = ((rgb * z[f"{tag}/g_rgb"]).sum() + (d * z[f"{tag}/g_d"]).sum() + (a * z[f"{tag}/g_a"]).sum()
             + (w * z[f"{tag}/g_w"]).sum())
        g, = torch.autograd.grad(L, rs)
        torch.testing.assert_close(g, z[f"{tag}/grad_all"], rtol=1e-5, atol=1e-5)


def test_render_rays_golden():
    z = load("render")
    p = mlp_params("w/")
    rgb, d, w, a, _ = O.render_rays(p, z["rays"], 64, training=False)
    torch.testing.assert_close(rgb, z["e_rgb"], rtol=0, atol=2e-6)
    torch.testing.assert_close(d, z["e_depth"], rtol=0, atol=1e-5)
    torch.testing.assert_close(w, z["e_w"], rtol=0, atol=2e-6)
    torch.testing.assert_close(a, z["e_acc"], rtol=0, atol=2e-6)
    # training mode: the reference's rand_like jitter is reproduced by the stored u
    t = O.stratified_t_vals(z["rays"][:, 6], z["rays"][:, 7], 64, True, z["u"])
    torch.testing.assert_close(t, z["t_train"], rtol=0, atol=1e-6)
    rgb, d, w, a, _ = O.render_rays(p, z["rays"], 64, training=True, u_strat=z["u"])
    torch.testing.assert_close(rgb, z["t_rgb"], rtol=0, atol=2e-6)
    torch.testing.assert_close(w, z["t_w"], rtol=0, atol=2e-6)


def test_train_step_golden():
    z = load("train_step")
    zr = load("render")
    tr = O.OracleTrainer(mlp_params("w/"), lr_sigma=2e-3, lr_color=2e-3)
    loss = tr.step(zr["rays"], z["gt"], 64, training=True, u_strat=zr["u"])
    assert abs(loss - float(z["loss"])) < 1e-6
    for k, v in z.items():
        if k.startswith("p/"):
            torch.testing.assert_close(tr.nets[0][k[2:]].detach(), v, rtol=0, atol=2e-6)


def test_sample_pdf_known_answers():
    """sample_pdf has no reference (PARITY UNPINNED): known-answer properties."""
    N, B = 4, 8
    bins = torch.linspace(2, 6, B + 1).expand(N, B + 1).contiguous()
    # uniform weights -> samples at the u quantiles of [2,6]
    u = torch.rand(N, 32)
    s = O.sample_pdf(bins, torch.ones(N, B), 32, u=u)
    torch.testing.assert_close(s, 2 + 4 * u, rtol=0, atol=1e-5)
    # one-hot weight -> (almost) all samples inside that bin
    w = torch.zeros(N, B); w[:, 3] = 1.0
    s = O.sample_pdf(bins, w, 256, det=True)
    inside = ((s >= bins[:, 3:4]) & (s <= bins[:, 4:5])).float().mean()
    assert inside > 0.98
    # monotone in u
    uu, _ = torch.sort(torch.rand(N, 64), -1)
    s = O.sample_pdf(bins, torch.rand(N, B), 64, u=uu)
    assert (s[:, 1:] >= s[:, :-1] - 1e-6).all()
