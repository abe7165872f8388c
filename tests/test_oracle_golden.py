"""Pin the CPU oracle (oracle/nerf_oracle.py) against golden vectors produced by importing the
reference itself (tools/gen_golden.py).  CPU only."""
from collections import OrderedDict

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


# ------------------------------------------------------------------ the reference's AMP numerics (tests/golden/amp.npz)


def _cos(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return float(a @ b / (a.norm() * b.norm() + 1e-300))


def test_amp_trunc_exp_input_is_fp32_golden():
    """Under autocast(float16) the imported reference's MetaNeRF hands trunc_exp an fp32 tensor (MetaLinear adds
    its fp32 bias to the fp16 matmul output, metamodule.py:153-156), so the clamp is fp32's 88.72
    (trunc_exp.py:30-35), not fp16's 11.09: sigma(15) = exp(15) = 3.27e6 > 65504.  The oracle's AMP restatement
    gives the same sigma and d sigma / d bias at every pre-activation of the known-answer set."""
    z = load("amp")
    assert int(z["sigma_in_bits"]) == 32 and int(z["out_bits"]) == 32
    x = z["te16_x"]
    y, g = z["te16_y"], z["te16_g"]
    assert float(y[x == 15.0]) > 65504.0 * 40 and float(y[x == 30.0]) > 1e12
    xr = x.clone().requires_grad_(True)
    h = O.trunc_exp(xr.view(-1, 1))
    gx, = torch.autograd.grad(h.sum(), xr)
    torch.testing.assert_close(h.detach().view(-1), y, rtol=1e-6, atol=0)
    torch.testing.assert_close(gx, g, rtol=1e-6, atol=0)


def test_amp_mlp_forward_backward_golden():
    """oracle.vanilla_forward(amp="fp16") (fp16 matmul operands / outputs, fp32 bias, ReLU and trunc_exp) against
    the reference's MetaNeRF run under autocast(float16): forward bitwise, every parameter gradient within 1e-3 of
    its norm (the fp16 rounding of the backward GEMM outputs happens inside the host's matmul differently)."""
    z = load("amp")
    m = load("mlp")
    p = OrderedDict((k, v.clone().requires_grad_(True)) for k, v in mlp_params("w/").items())
    x, gup = m["x_d"][:256], m["gup"][:256]
    out = O.vanilla_forward(p, x, amp="fp16")
    torch.testing.assert_close(out.detach(), z["out"], rtol=0, atol=1e-6)
    grads = torch.autograd.grad((out * gup).sum(), list(p.values()))
    for (n, _), gr in zip(p.items(), grads):
        ref = z[f"g/{n}"].double()
        rel = float((gr.double() - ref).norm() / (ref.norm() + 1e-30))
        assert rel <= 1e-3, f"{n}: AMP gradient rel err {rel:.2e}"
    # the fp32 oracle is NOT the reference's AMP result (fp16 rounding moves the early-layer gradients by ~8 %)
    out32 = O.vanilla_forward(mlp_params("w/"), x)
    assert (out32 - z["out"]).abs().max() > 1e-5


def test_amp_train_loss_and_scaled_gradients_golden():
    """The reference's use_amp loop body (runtime_adapt.py:291-305) on 64 rays x 32 coarse samples, jitter as
    recorded: autocast(float16) loss, backward of loss x 2^16, gradients unscaled.  OracleTrainer(amp="fp16")'s
    render + loss + scaled backward gives the same loss (to fp32 rounding) and gradients within 1e-3 of their norm."""
    z = load("amp")
    ot = O.OracleTrainer(mlp_params("w/"), amp="fp16", grad_clip=None)
    ot.opt.step = lambda: None  # compare the unscaled gradients, before any update
    loss = ot.step(z["step_rays"], z["step_gt"], 32, training=True, u_strat=z["step_u"])
    assert abs(loss - float(z["step_loss"])) <= 1e-6 * float(z["step_loss"]) + 1e-9, (loss, float(z["step_loss"]))
    for n, q in ot.nets[0].items():
        ref = z[f"sg/{n}"].double()
        rel = float((q.grad.double() - ref).norm() / (ref.norm() + 1e-30))
        assert rel <= 1e-3 and _cos(q.grad, ref) >= 0.99999, f"{n}: rel {rel:.2e}"


def test_amp_oracle_gradscaler_update():
    """OracleTrainer(amp="fp16") follows GradScaler.update: a step whose scaled gradients overflow is skipped (the
    parameters stay put) and halves the scale; 2000 clean steps in a row double it (torch.amp.GradScaler defaults)."""
    z = load("amp")
    ot = O.OracleTrainer(mlp_params("w/"), amp="fp16", grad_clip=None, loss_scale=3.0e38)  # x 3e38 overflows
    before = {n: q.detach().clone() for n, q in ot.nets[0].items()}
    ot.step(z["step_rays"][:8], z["step_gt"][:8], 32, training=True, u_strat=z["step_u"][:8])
    assert ot.loss_scale == 1.5e38
    assert all(torch.equal(q.detach(), before[n]) for n, q in ot.nets[0].items())
    ot2 = O.OracleTrainer(mlp_params("w/"), amp="fp16", grad_clip=None)
    ot2._growth_tracker = 1999
    ot2.opt.step = lambda: None
    ot2.step(z["step_rays"][:8], z["step_gt"][:8], 32, training=True, u_strat=z["step_u"][:8])
    assert ot2.loss_scale == 131072.0 and ot2._growth_tracker == 0
