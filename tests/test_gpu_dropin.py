"""The drop-in surface under the reference's own training-loop body (-m gpu).

The north star's contract is that this repo's ``render_rays`` + expert "drop into the existing training loop":
an/pipelines/online_stage/runtime_adapt.py:286-310 —

    optimizer.zero_grad()
    with torch.cuda.amp.autocast(enabled=use_amp, dtype=torch.float16):
        loss = compute_mse_loss(P, model=base, data={"rays": rays, "rgbs": rgbs}, ...)
    scaler.scale(loss).backward()
    scaler.unscale_(optimizer); torch.nn.utils.clip_grad_norm_(base.parameters(), grad_clip)
    scaler.step(optimizer); scaler.update()

* fp32 (use_amp False): the hierarchical step — ``HierarchicalNeRF`` (coarse + fine VanillaNeRF) through
  ``compute_mse_loss`` (MSE(fine) + MSE(coarse), nerf_amd/losses.py) with the jitter injected, autograd backward,
  ``clip_grad_norm_(1.0)`` and ``torch.optim.Adam`` — against ``OracleTrainer`` (the CPU restatement pinned to the
  reference's golden train step): loss to 1e-5, both nets' clipped gradients to 1e-4 of their scale, post-Adam
  parameters within the update difference the two measured gradients imply (test_gpu_parity._adam_step1_close);
  then two more steps' losses.
* AMP (configs/train.json "use_amp": true): inside ``autocast(fp16)`` the expert runs the fp16 build of the fused MLP
  kernels (bitwise ``nerf_mlp_fwd_f16``; ``autocast(bfloat16)`` the bf16 build), compositing stays fp32; the loop body
  as written with ``GradScaler`` trains and its loss tracks the fp32 loop's from the same seed.
* AMP parity: the reference under autocast(float16) keeps trunc_exp's input fp32 (MetaLinear's fp32 bias promotes
  the fp16 matmul output; tests/golden/amp.npz from the imported reference), so sigma is NOT clamped at fp16's 11.09
  — known answers beyond +-11.09 through the drop-in expert under autocast; and the drop-in AMP hierarchical step's
  first unscaled gradients against OracleTrainer(amp="fp16"), the CPU restatement of the reference's autocast
  numerics pinned to that fixture (tests/test_oracle_golden.py::test_amp_*): per tensor within 1e-2 relative error
  norm and flat cosine >= 0.9999 (the kernels keep the reference's fp16 rounding points; what differs is the fp32
  summation order inside each product, which moves an fp16 rounding now and then)."""
import types

import pytest
import torch

from golden_io import load
from oracle import nerf_oracle as O
from test_gpu_parity import _adam_step1_close, _close

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def K():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from nerf_amd import kernels
    return kernels


def _model(pc, pf):
    from nerf_amd.vanilla import HierarchicalNeRF, VanillaNeRF
    return HierarchicalNeRF(VanillaNeRF().load_reference_state(pc), VanillaNeRF().load_reference_state(pf)).to(DEV)


def _adam(model, lr_sigma, lr_color, **kw):
    grp = model.get_param_groups()
    return torch.optim.Adam([{"params": grp["sigma"]["params"], "lr": lr_sigma},
                             {"params": grp["color"]["params"], "lr": lr_color}], **kw)


def test_dropin_hierarchical_step_vs_oracle(K):
    from nerf_amd.losses import compute_mse_loss
    pc, pf = O.init_vanilla_params(1), O.init_vanilla_params(2)
    model = _model(pc, pf).train()
    opt = _adam(model, 2e-3, 1e-3)
    ot = O.OracleTrainer(pc, pf, lr_sigma=2e-3, lr_color=1e-3)
    P = types.SimpleNamespace(ray_samples=64, n_importance=128, chunk_points=1 << 22, color_space="linear")
    rays = load("render")["rays"]
    g = torch.Generator().manual_seed(17)
    gt = torch.rand(rays.shape[0], 3, generator=g)
    nets = {0: model.coarse, 1: model.fine}
    for step in range(3):
        us, up = torch.rand(rays.shape[0], 64, generator=g), torch.rand(rays.shape[0], 128, generator=g)
        opt.zero_grad()
        loss = compute_mse_loss(P, model, {"rays": rays.to(DEV), "rgbs": gt.to(DEV)}, u_strat=us.to(DEV),
                                u_pdf=up.to(DEV))
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        lref = ot.step(rays, gt, 64, n_importance=128, training=True, u_strat=us, u_pdf=up)
        assert abs(loss.item() - lref) < 1e-5 + 1e-4 * lref, (step, loss.item(), lref)
        if step == 0:
            for k, net in nets.items():
                for n, p in net.named_parameters():
                    ref = ot.nets[k][n]
                    _close(p.grad, ref.grad, rel_scale=True, what=f"net{k} clipped grad {n}")
                    lr = 1e-3 if n.startswith("color_mlp") else 2e-3
                    _adam_step1_close(p, ref, p.grad, ref.grad, lr, what=f"net{k} post-Adam {n}")


def test_autocast_dispatches_16bit_kernels(K):
    """Inside autocast(float16) VanillaNeRF.forward is bitwise the fp16 kernel build, inside autocast(bfloat16) the
    bf16 one; outside autocast the fp32 engine."""
    from nerf_amd.vanilla import VanillaNeRF, amp_precision
    net = VanillaNeRF().load_reference_state(O.init_vanilla_params(3)).to(DEV)
    g = torch.Generator().manual_seed(3)
    x = torch.cat([torch.rand(3000, 3, generator=g) * 3 - 1.5,
                   torch.nn.functional.normalize(torch.randn(3000, 3, generator=g), dim=-1)], -1).to(DEV)
    w = net.packed().detach()
    ref = {p: K.mlp_fwd(w, x, K.mlp_workspace(3000, False, DEV, p), False, precision=p)
           for p in ("fp32", "bf16", "fp16")}
    assert amp_precision() == "fp32"
    assert not torch.equal(ref["bf16"], ref["fp16"])
    with torch.no_grad():
        assert torch.equal(net(x), ref["fp32"])
        for dt, p in ((torch.float16, "fp16"), (torch.bfloat16, "bf16")):
            with torch.autocast("cuda", dtype=dt):
                assert amp_precision() == p
                out = net(x)
            assert out.dtype == torch.float32 and torch.equal(out, ref[p]), dt
    with torch.autocast("cuda", dtype=torch.float16):   # training forward (autograd Function) as well
        out = net(x)
    assert out.requires_grad and torch.equal(out.detach(), ref["fp16"])


def test_reference_amp_loop_body_with_gradscaler(K):
    """runtime_adapt.py:290-310 with use_amp=True, as written, on the drop-in surface: 40 steps of 1024-ray batches
    from a synthetic 100x100 scene, 64 + 128.  The AMP loop learns, its loss stays within 15 % of the fp32 loop's
    (same seed, same batches, same jitter draws), and GradScaler's skipped steps are counted from its scale history
    (it halves the scale on every step whose gradient holds an inf / nan and skips that step): at most 4 of 40, each
    printed with its step (fp16 rounding of a large gradient can overflow once in a while; the 6-step oracle test
    pins the scale exactly)."""
    from nerf_amd.losses import compute_mse_loss
    from nerf_amd.scene import make_blender_scene
    from nerf_amd.trainer import RayBatcher
    scene = make_blender_scene(n_train=4, n_test=1, H=100, W=100, seed=1, device=DEV)
    rb = RayBatcher(scene, DEV)
    P = types.SimpleNamespace(ray_samples=64, n_importance=128, chunk_points=1 << 22, color_space="linear")
    pc, pf = O.init_vanilla_params(1), O.init_vanilla_params(2)
    curves = {}
    for use_amp in (False, True):
        torch.manual_seed(0)
        base = _model(pc, pf).train()
        optimizer = _adam(base, 2e-3, 2e-3)
        scaler = torch.amp.GradScaler("cuda", enabled=use_amp)
        ls, scales = [], []
        for step in range(40):
            rays, rgbs = rb.batch(1024, seed=step)
            optimizer.zero_grad()
            with torch.cuda.amp.autocast(enabled=use_amp, dtype=torch.float16):
                loss = compute_mse_loss(P, model=base, data={"rays": rays, "rgbs": rgbs}, params=None,
                                        active_module=None, reduction="mean")
            scaler.scale(loss).backward()
            scaler.unscale_(optimizer)
            torch.nn.utils.clip_grad_norm_(base.parameters(), 1.0)
            scaler.step(optimizer)
            scaler.update()
            ls.append(float(loss.detach()))
            scales.append(scaler.get_scale() if use_amp else 1.0)
        if use_amp:
            prev = [65536.0] + scales[:-1]
            skipped = [i for i, (a0, a1) in enumerate(zip(prev, scales)) if a1 < a0]
            print(f"GradScaler: scale after 40 AMP steps {scaler.get_scale()}, skipped steps {skipped}")
            assert len(skipped) <= 4, f"GradScaler skipped {len(skipped)} steps: {skipped}"
            assert all(a1 in (a0 / 2, a0) for a0, a1 in zip(prev, scales)), scales  # no growth inside 40 steps
        curves[use_amp] = torch.tensor(ls)
    a, b = curves[True], curves[False]
    assert torch.isfinite(a).all()
    assert a[-10:].mean() < 0.8 * a[:5].mean(), a   # it learns
    assert (a[-10:].mean() - b[-10:].mean()).abs() <= 0.15 * b[-10:].mean(), (a[-10:].mean(), b[-10:].mean())
    assert not torch.equal(a, b)  # the AMP loop did run the 16-bit kernels


def test_amp_trunc_exp_beyond_fp16_clamp_golden(K):
    """te16_x = [-30, -12, 0, 11, 12, 15, 30] as the sigma head's pre-activation (weights 0, bias x) under
    autocast(float16): sigma equals the imported reference's (tests/golden/amp.npz) to 1e-5 — exp(x) without fp16's
    11.09 clamp (sigma(15) = 3.27e6) — and so does d sigma / d bias (the bias gradient is an fp32 sum in the reference
    and in the fp16 kernels: only the matmul operands are rounded)."""
    from nerf_amd.vanilla import VanillaNeRF
    from golden_io import mlp_params
    z = load("amp")
    x_d = load("mlp")["x_d"][:64].to(DEV)
    for x, y, gref in zip(z["te16_x"].tolist(), z["te16_y"].tolist(), z["te16_g"].tolist()):
        q = dict(mlp_params("w/"))
        q["sigma_head.weight"] = torch.zeros(1, 256)
        q["sigma_head.bias"] = torch.tensor([x])
        net = VanillaNeRF().load_reference_state(q).to(DEV)
        with torch.autocast("cuda", dtype=torch.float16):
            out = net(x_d)
        sig = out[:, 3].detach().cpu()
        assert ((sig - y).abs() <= 1e-5 * y).all(), f"x={x}: sigma {sig[:3].tolist()} vs reference {y}"
        net.zero_grad()
        out[:, 3].sum().backward()
        gb = net.sigma_head.bias.grad.item() / 64.0
        # exp(x) past +-11.09, not the clamp's exp(11.09); summed in fp32 as the reference's bias gradient
        assert abs(gb - gref) <= 1e-5 * gref, f"x={x}: d sigma / d bias {gb} vs reference {gref}"


def test_amp_dropin_step_gradients_vs_oracle_amp(K):
    """runtime_adapt.py:290-305 with use_amp=True on the drop-in surface (HierarchicalNeRF, compute_mse_loss,
    GradScaler at its initial 2^16), 1024 golden rays x (64 + 128), injected jitter: the unscaled first-step
    gradient of each net against OracleTrainer(amp="fp16") — the reference's autocast(float16) restatement — per
    tensor within 1e-2 relative error norm and at flat cosine >= 0.9999, the loss within 1e-4.  Both are printed
    against the fp32 oracle too."""
    from nerf_amd.losses import compute_mse_loss
    pc, pf = O.init_vanilla_params(1), O.init_vanilla_params(2)
    model = _model(pc, pf).train()
    opt = _adam(model, 2e-3, 1e-3)
    scaler = torch.amp.GradScaler("cuda")
    P = types.SimpleNamespace(ray_samples=64, n_importance=128, chunk_points=1 << 22, color_space="linear")
    rays = load("render")["rays"]
    g = torch.Generator().manual_seed(23)
    gt = torch.rand(rays.shape[0], 3, generator=g) * 0.5 + 0.25
    us, up = torch.rand(rays.shape[0], 64, generator=g), torch.rand(rays.shape[0], 128, generator=g)
    opt.zero_grad()
    with torch.cuda.amp.autocast(dtype=torch.float16):
        loss = compute_mse_loss(P, model, {"rays": rays.to(DEV), "rgbs": gt.to(DEV)}, u_strat=us.to(DEV),
                                u_pdf=up.to(DEV))
    scaler.scale(loss).backward()
    scaler.unscale_(opt)
    refs = {}
    for amp in ("fp16", None):
        ot = O.OracleTrainer(pc, pf, amp=amp, grad_clip=None)
        ot.opt.step = lambda: None
        refs[amp] = (ot.step(rays, gt, 64, n_importance=128, training=True, u_strat=us, u_pdf=up), ot)
    lref = refs["fp16"][0]
    assert abs(loss.item() - lref) <= 1e-4 * lref, (loss.item(), lref)
    for k, net in enumerate((model.coarse, model.fine)):
        names = [n for n, _ in net.named_parameters()]
        a = torch.cat([q.grad.detach().double().cpu().flatten() for q in net.parameters()])
        cos = {}
        for amp, (_, ot) in refs.items():
            b = torch.cat([ot.nets[k][n].grad.double().flatten() for n in names])
            cos[amp] = float(a @ b / (a.norm() * b.norm()))
        b16 = torch.cat([refs["fp16"][1].nets[k][n].grad.double().flatten() for n in names])
        b32 = torch.cat([refs[None][1].nets[k][n].grad.double().flatten() for n in names])
        ref_vs_fp32 = float(b16 @ b32 / (b16.norm() * b32.norm()))
        print(f"net {k}: cos(drop-in AMP, reference AMP) {cos['fp16']:.6f}, cos(drop-in AMP, fp32) {cos[None]:.6f}, "
              f"cos(reference AMP, fp32) {ref_vs_fp32:.6f}")
        assert cos["fp16"] >= 0.9999, f"net {k}: cosine vs the reference's AMP gradient {cos['fp16']:.6f}"
        worst = (0.0, "")
        for n, q in net.named_parameters():
            r = refs["fp16"][1].nets[k][n].grad.double()
            err = float((q.grad.detach().double().cpu() - r).norm() / r.norm().clamp_min(1e-30))
            worst = max(worst, (err, n))
            assert err <= 1e-2, f"net {k} {n}: relative error norm {err:.3e} vs the reference's AMP gradient"
        print(f"net {k}: worst per-tensor relative error norm {worst[0]:.3e} ({worst[1]})")


def test_amp_dropin_loop_vs_oracle_amp_multistep(K):
    """Six steps of the use_amp=True loop body (runtime_adapt.py:286-310: autocast(float16) -> GradScaler scale ->
    backward -> unscale_ -> clip_grad_norm_(1.0) -> step -> update) on the drop-in surface against
    OracleTrainer(amp="fp16"), which mirrors GradScaler's unscale / skip / update, from the same weights with the
    same rays, targets and jitter every step: each step's loss within 1e-3 relative, the GradScaler scale equal, and
    after the last step every parameter tensor within 5e-3 relative error norm of the oracle's (Adam's first steps
    move a weight by ~lr whatever its gradient's size, so a gradient near zero whose sign an fp16 rounding flip
    changes moves by 2 lr), and the whole parameter vector closer to the AMP oracle's than to the fp32 oracle's
    trajectory from the same inputs."""
    from nerf_amd.losses import compute_mse_loss
    pc, pf = O.init_vanilla_params(1), O.init_vanilla_params(2)
    model = _model(pc, pf).train()
    opt = _adam(model, 2e-3, 1e-3)
    scaler = torch.amp.GradScaler("cuda")
    ot = O.OracleTrainer(pc, pf, lr_sigma=2e-3, lr_color=1e-3, amp="fp16")
    o32 = O.OracleTrainer(pc, pf, lr_sigma=2e-3, lr_color=1e-3)
    P = types.SimpleNamespace(ray_samples=64, n_importance=128, chunk_points=1 << 22, color_space="linear")
    rays_all = load("render")["rays"]
    for step in range(6):
        g = torch.Generator().manual_seed(100 + step)
        idx = torch.randperm(rays_all.shape[0], generator=g)[:512]
        rays = rays_all[idx].contiguous()
        gt = torch.rand(rays.shape[0], 3, generator=g) * 0.5 + 0.25
        us, up = torch.rand(rays.shape[0], 64, generator=g), torch.rand(rays.shape[0], 128, generator=g)
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.float16):
            loss = compute_mse_loss(P, model, {"rays": rays.to(DEV), "rgbs": gt.to(DEV)}, u_strat=us.to(DEV),
                                    u_pdf=up.to(DEV))
        scaler.scale(loss).backward()
        scaler.unscale_(opt)
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        scaler.step(opt)
        scaler.update()
        lref = ot.step(rays, gt, 64, n_importance=128, training=True, u_strat=us, u_pdf=up)
        o32.step(rays, gt, 64, n_importance=128, training=True, u_strat=us, u_pdf=up)
        print(f"step {step}: loss {loss.item():.7f} vs oracle AMP {float(lref):.7f}, scale {scaler.get_scale():.0f} / "
              f"{ot.loss_scale:.0f}")
        assert abs(loss.item() - float(lref)) <= 1e-3 * float(lref), (step, loss.item(), float(lref))
        assert scaler.get_scale() == ot.loss_scale
    worst = (0.0, "")
    d16, d32 = 0.0, 0.0
    for k, net in enumerate((model.coarse, model.fine)):
        for n, q in net.named_parameters():
            a = q.detach().double().cpu()
            r = ot.nets[k][n].detach().double()
            err = float((a - r).norm() / r.norm().clamp_min(1e-30))
            worst = max(worst, (err, f"net{k} {n}"))
            assert err <= 5e-3, f"net {k} {n}: relative error norm {err:.3e} after 6 AMP steps"
            d16 += float((a - r).pow(2).sum())
            d32 += float((a - o32.nets[k][n].detach().double()).pow(2).sum())
    print(f"after 6 AMP steps: worst per-tensor parameter relative error norm {worst[0]:.3e} ({worst[1]}); "
          f"distance to the AMP oracle {d16 ** 0.5:.3e}, to the fp32 oracle {d32 ** 0.5:.3e}")
    assert d16 < d32, (d16, d32)
