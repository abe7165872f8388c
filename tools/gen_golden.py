#!/usr/bin/env python3
"""Generate golden vectors by IMPORTING THE REFERENCE (never copied) — runs only in the build
container, where /root/reference exists.  Writes small .npz fixtures into tests/golden/.

The reference is imported from /root/reference/adaptive_nerf (PYTHONPATH style of
mediator.py:112-113).  Three modules it imports at top level but never calls on the
stratified/vanilla path are absent from the image and are stubbed in
sys.modules for the import only: ``nerfacc`` (ray_rendering.py:9, used only by the occupancy
renderer), ``jaxtyping`` (scene_box.py:3, a type annotation), ``viser.transforms``
(scene_box.py:7, used only by OrientedBox).  No reference code runs through a stub.

MetaNeRF's (x,d,params)->dict forward is wrapped in a 6-line adapter to the container
contract expert(x_d (M,6), params) -> (M,4) (SURVEY.md §0 defect 2).

Usage:  PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden.py [--only-ngp | --only-moe | --only-data | --only-meta |
        --only-amp | --only-maml]
"""
import math
import os
import sys
import types
from collections import OrderedDict
from types import SimpleNamespace

import numpy as np
import torch

REF = "/root/reference/adaptive_nerf"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")


def _install_stubs():
    nerfacc = types.ModuleType("nerfacc")
    nerfacc.OccGridEstimator = object
    jax = types.ModuleType("jaxtyping")

    class _Sub:
        def __class_getitem__(cls, item):
            return torch.Tensor

    jax.Float = _Sub
    viser = types.ModuleType("viser")
    vtf = types.ModuleType("viser.transforms")
    viser.transforms = vtf
    for name, mod in (("nerfacc", nerfacc), ("jaxtyping", jax), ("viser", viser), ("viser.transforms", vtf)):
        sys.modules.setdefault(name, mod)


def main():
    if not os.path.isdir(REF):
        print("reference absent; nothing to do")
        return
    sys.dont_write_bytecode = True
    _install_stubs()
    sys.path.insert(0, REF)
    torch.set_num_threads(8)
    from nerfs import ray_rendering as rr          # noqa: E402
    from nerfs import ray_sampling as rs           # noqa: E402
    from nerfs.scene_box import SceneBox           # noqa: E402
    from nerfs.losses import compute_mse_loss     # noqa: E402
    from models.encodings import FrequencyEncoder  # noqa: E402
    from models.inr.meta_vanilla import MetaNeRF   # noqa: E402
    from models.trunc_exp import trunc_exp         # noqa: E402

    os.makedirs(OUT, exist_ok=True)
    g = torch.Generator().manual_seed(1234)

    # ---------------------------------------------------------------- frequency encoder
    x = (torch.rand(512, 3, generator=g) * 12 - 6)
    d = torch.nn.functional.normalize(torch.randn(512, 3, generator=g), dim=-1)
    fx = FrequencyEncoder(3, 10, include_input=True, use_pi=False)
    fd = FrequencyEncoder(3, 4, include_input=True, use_pi=False)
    f2 = FrequencyEncoder(3, 2, include_input=True, use_pi=False)
    np.savez_compressed(os.path.join(OUT, "freq.npz"), x=x.numpy(), enc_x=fx(x).numpy(), d=d.numpy(),
                        enc_d=fd(d).numpy(), small_in=np.array([[0.1, 0.2, 0.3]], np.float32),
                        small_out=f2(torch.tensor([[0.1, 0.2, 0.3]])).numpy())

    # ---------------------------------------------------------------- rays
    H = W = 800
    focal = 0.5 * W / np.tan(0.5 * 0.6911112)
    dirs = rs.get_ray_directions(H, W, focal, focal, W / 2, H / 2, center_pixels=True, device="cpu")
    c2w = torch.tensor([[-0.9999, 0.0042, -0.0134, -0.0538],
                        [-0.0140, -0.2997, 0.9539, 3.8455],
                        [0.0000, 0.9540, 0.2997, 1.2081]], dtype=torch.float32)
    crop = dirs[350:450, 350:450]                      # C1: centre 100x100 crop
    rays_const = rs.get_rays(crop, c2w, near=2.0, far=6.0).reshape(-1, 8)
    box = SceneBox(aabb=torch.tensor([[-1.5, -1.5, -1.5], [1.5, 1.5, 1.5]]))
    dirs_small = rs.get_ray_directions(24, 40, 30.0, 28.0, 19.3, 12.1, center_pixels=True, device="cpu")
    c2w_b = torch.tensor([[0.8, 0.0, 0.6, 3.0], [0.0, 1.0, 0.0, 0.4], [-0.6, 0.0, 0.8, 3.5]])
    rays_aabb = rs.get_rays(dirs_small, c2w_b, scene_box=box).reshape(-1, 8)
    clamped, valid = rs.clamp_rays_near_far(rays_aabb, near_far_override=(0.5, 4.0))
    dirs_nc = rs.get_ray_directions(7, 9, 5.0, 6.0, 4.0, 3.5, center_pixels=False, device="cpu")
    np.savez_compressed(os.path.join(OUT, "rays.npz"), focal=np.float32(focal), c2w=c2w.numpy(),
                        dirs_crop=crop.numpy(), rays_const=rays_const.numpy(),
                        dirs_small=dirs_small.numpy(), c2w_b=c2w_b.numpy(), rays_aabb=rays_aabb.numpy(),
                        clamped=clamped.numpy(), valid=valid.numpy(), dirs_nc=dirs_nc.numpy())

    # ---------------------------------------------------------------- MLP (MetaNeRF, frequency dirs)
    torch.manual_seed(0)
    net = MetaNeRF(encoding_dir="frequency")

    class Adapter(torch.nn.Module):  # expert(x_d (M,6), params) -> (M,4)
        def __init__(self, n):
            super().__init__(); self.net = n; self.use_occ = False; self.submodules = [n]

        def forward(self, x_d, params=None):
            o = self.net(x_d[:, :3], x_d[:, 3:6], params=params)
            return torch.cat([o["rgb"], o["sigma"]], -1)

        def get_param_groups(self):  # meta_ngp.py:446-469 grouping
            sig = [p for n, p in self.net.named_parameters() if not n.startswith("color_mlp")]
            col = [p for n, p in self.net.named_parameters() if n.startswith("color_mlp")]
            return {"sigma": {"params": sig}, "color": {"params": col}}

    model = Adapter(net)
    state = OrderedDict((n, p.detach().clone()) for n, p in net.meta_named_parameters())
    M = 1024
    pts = torch.rand(M, 3, generator=g) * 3 - 1.5
    dd = torch.nn.functional.normalize(torch.randn(M, 3, generator=g), dim=-1)
    x_d = torch.cat([pts, dd], -1)
    out = model(x_d)
    gup = torch.randn(M, 4, generator=g)
    grads = torch.autograd.grad((out * gup).sum(), list(net.parameters()))
    names = [n for n, _ in net.named_parameters()]
    # a fast-weights forward through params= (MetaLinear path) must equal the module forward
    fast = OrderedDict((n, p * 1.0) for n, p in net.meta_named_parameters())
    out_fast = model(x_d, params=fast)
    assert torch.equal(out_fast, out)
    # trunc_exp backward outside the clamp
    te_x = torch.tensor([-100.0, -5.0, 0.0, 3.0, 100.0], requires_grad=True)
    te_y = trunc_exp(te_x)
    te_g, = torch.autograd.grad(te_y.sum(), te_x)
    arr = {f"w/{n}": v.numpy() for n, v in state.items()}
    arr.update({f"g/{n}": gr.numpy() for n, gr in zip(names, grads)})
    np.savez_compressed(os.path.join(OUT, "mlp.npz"), x_d=x_d.numpy(), out=out.detach().numpy(),
                        gup=gup.numpy(), te_x=te_x.detach().numpy(), te_y=te_y.detach().numpy(),
                        te_g=te_g.numpy(), **arr)

    # ---------------------------------------------------------------- volume_render
    vr = {}
    for tag, (N, S) in (("s64", (128, 64)), ("s192", (64, 192))):
        t = torch.sort(torch.rand(N, S, generator=g) * 4 + 2, -1)[0]
        t[0, 5] = t[0, 4]  # a zero-length interval (clamp_min(1e-4) branch)
        rgbs = torch.rand(N, S, 4, generator=g)
        rgbs[..., :3] = rgbs[..., :3] * 1.2 - 0.1  # exercise rgb clamp(0,1)
        rgbs[..., 3] = torch.exp(torch.randn(N, S, generator=g) * 2.0)
        rgbs[:8, :, 3] *= -1.0  # negative sigma rows (clamp_min(0))
        rgbs[8:16, :, 3] = 1e4  # fully opaque rays (alpha clamp at 1-1e-7)
        rgbs.requires_grad_(True)
        bg = torch.ones(N, 3)
        rgb, depth, w, acc = rr.volume_render(rgbs, t, bg_rgb=bg)
        g_rgb, g_d, g_a, g_w = (torch.randn(N, 3, generator=g), torch.randn(N, generator=g),
                                torch.randn(N, generator=g), torch.randn(N, S, generator=g))
        grad_all, = torch.autograd.grad((rgb * g_rgb).sum() + (depth * g_d).sum() + (acc * g_a).sum()
                                        + (w * g_w).sum(), rgbs)
        grad_rgb, = torch.autograd.grad((rr.volume_render(rgbs, t, bg_rgb=bg)[0] * g_rgb).sum(), rgbs)
        vr.update({f"{tag}/t": t, f"{tag}/rgbs": rgbs.detach(), f"{tag}/rgb": rgb.detach(),
                   f"{tag}/depth": depth.detach(), f"{tag}/w": w.detach(), f"{tag}/acc": acc.detach(),
                   f"{tag}/g_rgb": g_rgb, f"{tag}/g_d": g_d, f"{tag}/g_a": g_a, f"{tag}/g_w": g_w,
                   f"{tag}/grad_all": grad_all, f"{tag}/grad_rgb": grad_rgb})
    np.savez_compressed(os.path.join(OUT, "volume_render.npz"), **{k: v.numpy() for k, v in vr.items()})

    # ---------------------------------------------------------------- render_rays end to end
    idx = torch.randperm(rays_const.shape[0], generator=g)[:128]
    rays = rays_const[idx].contiguous()
    model.eval()
    with torch.no_grad():
        e_rgb, e_depth, e_w, e_acc = rr.render_rays(model, rays, ray_samples=64, chunk=4096)
    model.train()
    torch.manual_seed(77)
    u = torch.rand(128, 64)
    torch.manual_seed(77)
    with torch.no_grad():
        t_rgb, t_depth, t_w, t_acc = rr.render_rays(model, rays, ray_samples=64, chunk=4096)
    # reproduce the reference's jitter draw exactly: stratified_t_vals draws rand_like((N,S))
    torch.manual_seed(77)
    tv = rr.stratified_t_vals(rays[:, 6], rays[:, 7], 64, randomized=True)
    np.savez_compressed(os.path.join(OUT, "render.npz"), rays=rays.numpy(), e_rgb=e_rgb.numpy(),
                        e_depth=e_depth.numpy(), e_w=e_w.numpy(), e_acc=e_acc.numpy(), u=u.numpy(),
                        t_train=tv.numpy(), t_rgb=t_rgb.numpy(), t_depth=t_depth.numpy(),
                        t_w=t_w.numpy(), t_acc=t_acc.numpy())

    # ---------------------------------------------------------------- one train step (runtime_adapt.py:286-310)
    gt = torch.rand(128, 3, generator=g)
    P = SimpleNamespace(optimizer="adam", sigma_lr=2e-3, color_lr=2e-3, lr=1e-4, weight_decay=0.0,
                        ray_samples=64, chunk_points=4096, color_space="linear")
    # common/utils.py:16-76 get_optimizer(P) with P.optimizer="adam" (not importable here: its module
    # imports torchvision, absent from the image) — same groups/lrs built directly:
    grp = model.get_param_groups()
    optimizer = torch.optim.Adam([{"params": grp["sigma"]["params"], "lr": P.sigma_lr, "name": "sigma"},
                                  {"params": grp["color"]["params"], "lr": P.color_lr, "name": "color"}],
                                 lr=P.lr, weight_decay=P.weight_decay)
    model.train()
    optimizer.zero_grad()
    torch.manual_seed(77)  # same jitter u as above
    loss = compute_mse_loss(P, model, {"rays": rays, "rgbs": gt})
    loss.backward()
    gnorm = torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
    optimizer.step()
    keep = ["trunk.0.linear.weight", "trunk.4.linear.weight", "trunk.7.linear.bias", "sigma_head.weight",
            "sigma_head.bias", "geo_head.weight", "color_mlp.layer0.linear.weight",
            "color_mlp.color_out.weight", "color_mlp.color_out.bias"]
    after = {f"p/{n}": p.detach().numpy() for n, p in net.named_parameters() if n in keep}
    np.savez_compressed(os.path.join(OUT, "train_step.npz"), gt=gt.numpy(), loss=np.float32(loss.item()),
                        gnorm=np.float32(gnorm.item()), lr=np.float32(2e-3), **after)
    gen_ngp()
    gen_moe()
    gen_data()
    for f in sorted(os.listdir(OUT)):
        print(f, os.path.getsize(os.path.join(OUT, f)))


def gen_ngp():
    """Instant-NGP expert fixtures: SHEncoder, HashGridEncoder (torch backend,
    several level/feature/interpolation configs, incl. points outside [0,1]) and MetaNGP forward +
    every parameter gradient (hash table included) for two network shapes."""
    from models.encodings import SHEncoder, HashGridEncoder   # noqa: E402
    from models.inr.meta_ngp import MetaNGP                    # noqa: E402
    from nerfs.scene_box import SceneBox                       # noqa: E402
    g = torch.Generator().manual_seed(4321)
    arr = {}
    d = torch.randn(256, 3, generator=g) * 2.0
    arr["sh_d"] = d.numpy()
    for lv in range(1, 6):
        arr[f"sh_{lv}"] = SHEncoder(levels=lv, implementation="torch")(d).numpy()
    hcfg = {"a": dict(levels=4, features_per_level=2, log2_hashmap_size=12, min_res=16, max_res=4096,
                      interpolation="Linear"),
            "b": dict(levels=16, features_per_level=2, log2_hashmap_size=12, min_res=16, max_res=2048,
                      interpolation="Smoothstep"),
            "c": dict(levels=8, features_per_level=4, log2_hashmap_size=10, min_res=4, max_res=300,
                      interpolation="Nearest"),
            "d": dict(levels=8, features_per_level=1, log2_hashmap_size=11, min_res=16, max_res=512,
                      interpolation="Linear")}
    x = torch.rand(256, 3, generator=g)
    x[:8] = torch.rand(8, 3, generator=g) * 1.4 - 0.2   # a few points outside [0,1]: negative floors
    arr["hash_x"] = x.numpy()
    for tag, c in hcfg.items():
        enc = HashGridEncoder(implementation="torch", **c)
        with torch.no_grad():
            enc.hash_table.copy_(torch.randn(enc.hash_table.shape, generator=g) * 0.5)
        y = enc(x)
        gup = torch.randn(y.shape, generator=g)
        gt, = torch.autograd.grad((y * gup).sum(), [enc.hash_table])
        arr[f"hash_{tag}_table"] = enc.hash_table.detach().numpy()
        arr[f"hash_{tag}_res"] = enc.level_resolutions.numpy()
        arr[f"hash_{tag}_out"] = y.detach().numpy()
        arr[f"hash_{tag}_gup"] = gup.numpy()
        arr[f"hash_{tag}_gtable"] = gt.numpy()
    mcfg = {"m1": dict(hidden=64, sigma_depth=2, color_hidden=64, color_depth=2, dir_encoding="spherical",
                       hash_enc_conf=dict(levels=8, features_per_level=2, log2_hashmap_size=12, min_res=16,
                                          max_res=1024, interpolation="Linear")),
            "m2": dict(hidden=32, sigma_depth=1, color_hidden=48, color_depth=3, dir_encoding="frequency",
                       hash_enc_conf=dict(levels=16, features_per_level=2, log2_hashmap_size=11, min_res=16,
                                          max_res=2048, interpolation="Linear"))}
    aabb = torch.tensor([[-1.0, -2.0, -1.5], [2.0, 1.0, 1.5]])
    M = 512
    pts = torch.rand(M, 3, generator=g) * 3.4 + aabb[0] - 0.2      # some samples outside the box
    dd = torch.randn(M, 3, generator=g)                              # non-unit: MetaNGP normalises
    x_d = torch.cat([pts, dd], -1)
    arr["ngp_aabb"] = aabb.numpy()
    arr["ngp_x_d"] = x_d.numpy()
    for tag, c in mcfg.items():
        torch.manual_seed(7)
        net = MetaNGP(occ_conf={}, scene_box=SceneBox(aabb=aabb.clone()), **c)
        with torch.no_grad():
            net.xyz_encoder.hash_table.copy_(torch.randn(net.xyz_encoder.hash_table.shape, generator=g) * 0.5)
        out = net(x_d)
        gup = torch.randn(M, 4, generator=g)
        names = [n for n, _ in net.named_parameters()]
        grads = torch.autograd.grad((out * gup).sum(), list(net.parameters()))
        fast = OrderedDict((n, p * 1.0) for n, p in net.meta_named_parameters())
        assert "xyz_encoder.hash_table" not in fast          # the hash table is not a fast weight
        assert torch.equal(net(x_d, params=fast), out)
        arr[f"{tag}_res"] = net.xyz_encoder.level_resolutions.numpy()
        arr[f"{tag}_out"] = out.detach().numpy()
        arr[f"{tag}_gup"] = gup.numpy()
        for n, p in net.named_parameters():
            arr[f"{tag}_w/{n}"] = p.detach().numpy()
        for n, gr in zip(names, grads):
            arr[f"{tag}_g/{n}"] = gr.numpy()
    np.savez_compressed(os.path.join(OUT, "ngp.npz"), **arr)


def gen_moe():
    """MetaContainer fixtures: routing weights, the routed expert mix (soft margin
    1.05 on (y,z), hard argmin on xyz) with every parameter gradient, and background_color + grads."""
    from models.inr.meta_container import MetaContainer        # noqa: E402
    from nerfs.scene_box import SceneBox                       # noqa: E402
    g = torch.Generator().manual_seed(777)
    arr = {}
    K = 3
    boxes = [torch.tensor([[-1.5, -1.5, -1.5], [0.2, 1.5, 1.5]]),
             torch.tensor([[-0.2, -1.5, -1.5], [1.5, 0.2, 1.5]]),
             torch.tensor([[-0.2, -0.2, -1.5], [1.5, 1.5, 1.5]])]
    cents = torch.tensor([[-0.7, -0.4, 0.3], [0.6, -0.8, -0.2], [0.7, 0.7, 0.1]])
    gaabb = torch.tensor([[-1.5, -1.5, -1.5], [1.5, 1.5, 1.5]])
    M = 600
    x = torch.rand(M, 3, generator=g) * 3 - 1.5
    dd = torch.randn(M, 3, generator=g)
    x_d = torch.cat([x, dd], -1)
    arr["centroids"] = cents.numpy()
    arr["x_d"] = x_d.numpy()
    for i, b in enumerate(boxes):
        arr[f"box{i}"] = b.numpy()
    kw = dict(hidden=32, sigma_depth=1, color_hidden=32, color_depth=1, dir_encoding="spherical",
              hash_enc_conf=dict(levels=4, features_per_level=2, log2_hashmap_size=10, min_res=8, max_res=128,
                                 interpolation="Linear"))
    for tag, bm, c2d in (("soft", 1.05, True), ("hard", 1.0, False)):
        torch.manual_seed(11)
        mc = MetaContainer(num_submodules=K, centroids=cents.clone(), aabb=gaabb.clone(), nerf_variant="instant",
                           boundary_margin=bm, cluster_2d=c2d, use_bg_nerf=True, bg_hidden=32,
                           bg_encoding="spherical", occ_conf={},
                           expert_box_list=[SceneBox(aabb=b.clone()) for b in boxes], **kw)
        with torch.no_grad():
            for sub in mc.submodules:
                sub.xyz_encoder.hash_table.copy_(torch.randn(sub.xyz_encoder.hash_table.shape, generator=g) * 0.5)
        w, hard = mc._routing(x_d[:, :3])
        out = mc(x_d)
        gup = torch.randn(M, 4, generator=g)
        names = [n for n, _ in mc.named_parameters()]
        grads = torch.autograd.grad((out * gup).sum(), list(mc.parameters()), allow_unused=True)
        arr[f"{tag}_route"] = (w if w is not None else torch.nn.functional.one_hot(hard, K).float()).numpy()
        arr[f"{tag}_out"] = out.detach().numpy()
        arr[f"{tag}_gup"] = gup.numpy()
        for n, p in mc.named_parameters():
            arr[f"{tag}_w/{n}"] = p.detach().numpy()
        for n, gr in zip(names, grads):
            if gr is not None:
                arr[f"{tag}_g/{n}"] = gr.numpy()
        groups = mc.get_param_groups()
        arr[f"{tag}_groups"] = np.array([len(groups[k]["params"]) for k in ("encoding", "sigma", "color", "background")])
        if tag == "soft":
            dirs = torch.randn(300, 3, generator=g)
            bg = mc.background_color(dirs)
            gb = torch.randn(300, 3, generator=g)
            bgn = [n for n, _ in mc.named_parameters() if n.startswith("bg_mlp")]
            bgg = torch.autograd.grad((bg * gb).sum(), [dict(mc.named_parameters())[n] for n in bgn])
            arr["bg_d"] = dirs.numpy()
            arr["bg_out"] = bg.detach().numpy()
            arr["bg_gup"] = gb.numpy()
            for n, gr in zip(bgn, bgg):
                arr[f"bg_g/{n}"] = gr.numpy()
    np.savez_compressed(os.path.join(OUT, "moe.npz"), **arr)


def gen_data():
    """Data-path fixtures: RamRaysDataset's per-image ray generation
    (_process_single_image, data/ram_rays_dataset.py:46-121) on in-memory images: AABB near/far with misses,
    a pixel mask, a near/far override; and one first-order task_adapt inner loop
    (pipelines/offline_stage/meta_core.py:14-68) of MetaNeRF(frequency) on support rays."""
    from data.ram_rays_dataset import _process_single_image     # noqa: E402
    from nerfs.scene_box import SceneBox                        # noqa: E402
    g = torch.Generator().manual_seed(99)
    arr = {}

    class MD:  # ImageMetadata surface used by _process_single_image (load_image / load_mask / fields)
        def __init__(self, i, H, W, c2w, K, img, mask):
            self.H, self.W, self.c2w, self.intrinsics, self.image_index, self.is_val = H, W, c2w, K, i, False
            self._img, self._mask = img, mask

        def load_image(self):
            return self._img

        def load_mask(self):
            return self._mask

    H, W = 24, 32
    box = SceneBox(aabb=torch.tensor([[-1.5, -1.5, -1.5], [1.5, 1.5, 1.5]]))
    cases = []
    for i in range(2):
        ang = 0.4 + 0.9 * i
        c2w = torch.tensor([[math.cos(ang), 0.0, math.sin(ang), 4.0 * math.sin(ang)],
                            [0.0, 1.0, 0.0, 0.3],
                            [-math.sin(ang), 0.0, math.cos(ang), 4.0 * math.cos(ang)]])
        K = torch.tensor([40.0, 38.0, 15.7, 12.2]) if i == 1 else torch.tensor([9.0, 8.5, 15.7, 12.2])  # d0: wide, some rays miss
        img = torch.randint(0, 256, (H, W, 3), generator=g, dtype=torch.uint8)
        mask = (torch.rand(H, W, generator=g) > 0.3) if i == 1 else None
        md = MD(7 + i, H, W, c2w, K, img, mask)
        ovr = (0.5, 4.0) if i == 1 else None
        rgbs, rays, idx = _process_single_image(md, True, False, {"scene_box": box, "near_far_override": ovr})
        arr[f"d{i}_c2w"], arr[f"d{i}_K"], arr[f"d{i}_img"] = c2w.numpy(), K.numpy(), img.numpy()
        if mask is not None:
            arr[f"d{i}_mask"] = mask.numpy()
        arr[f"d{i}_rgbs"], arr[f"d{i}_rays"], arr[f"d{i}_idx"] = rgbs.numpy(), rays.numpy(), idx.numpy()
    np.savez_compressed(os.path.join(OUT, "data.npz"), **arr)
    gen_meta()


def gen_meta():
    """task_adapt (first-order, pipelines/offline_stage/meta_core.py:14-68) of MetaNeRF(frequency) with the
    mlp.npz weights on 64 support rays (eval-mode t, linear colour space, white bg), then reptile_meta_update
    (:145-176) with two fast lists, one NaN tensor and one zero-delta tensor (the per-tensor guard)."""
    from models.inr.meta_vanilla import MetaNeRF                      # noqa: E402
    from pipelines.offline_stage.meta_core import task_adapt, reptile_meta_update  # noqa: E402
    z = np.load(os.path.join(OUT, "mlp.npz"))
    zr = np.load(os.path.join(OUT, "rays.npz"))
    net = MetaNeRF(encoding_dir="frequency")
    with torch.no_grad():
        for n, p in net.meta_named_parameters():
            p.copy_(torch.from_numpy(z[f"w/{n}"]))

    class Expert(torch.nn.Module):  # expert(x_d (M,6), params) -> (M,4) over MetaNeRF's own fast-weight names
        def __init__(self, n):
            super().__init__(); self.net = n

        def forward(self, x_d, params=None):
            o = self.net(x_d[:, :3], x_d[:, 3:6], params=params)
            return torch.cat([o["rgb"], o["sigma"]], -1)

        def meta_named_parameters(self):
            return self.net.meta_named_parameters()

    class Model(torch.nn.Module):
        def __init__(self, e):
            super().__init__(); self.submodules = torch.nn.ModuleList([e]); self.use_occ = False

        def meta_named_parameters(self):
            return self.submodules[0].meta_named_parameters()

    model = Model(Expert(net)).eval()
    g = torch.Generator().manual_seed(4321)
    rays = torch.from_numpy(zr["rays_const"])[torch.randperm(10000, generator=g)[:64]].contiguous()
    gt = torch.rand(64, 3, generator=g)
    P = SimpleNamespace(algo="fomaml", fim=False, use_amp=False, ray_samples=32, chunk_points=1 << 20,
                        color_space="linear", lr=0.5)
    fast, losses = task_adapt(P, model, {"rays": rays, "rgbs": gt}, inner_lr=0.05, iterations=3, active_module=0)
    arr = {"rays": rays.numpy(), "gt": gt.numpy(), "losses": torch.stack(losses).numpy()}
    arr.update({f"fast/{n}": v.detach().numpy() for n, v in fast.items()})
    # reptile: theta = the mlp.npz weights, fast_list = [task_adapt result, a second perturbed copy]
    fast1 = OrderedDict((n, v.detach().clone()) for n, v in fast.items())
    fast2 = OrderedDict((n, v.detach() + 0.01 * torch.randn(v.shape, generator=g)) for n, v in fast.items())
    fast2["trunk.3.linear.bias"][5] = float("nan")                 # non-finite delta -> tensor skipped
    theta = OrderedDict((n, p.detach().clone()) for n, p in net.meta_named_parameters())
    fast1["geo_head.bias"] = theta["geo_head.bias"].clone()         # zero delta -> tensor skipped
    fast2["geo_head.bias"] = theta["geo_head.bias"].clone()
    reptile_meta_update(P, model, [fast1, fast2])
    # stored for a subset of tensors (the fixture stays small); the guard cases are among them
    keep = ("trunk.0.linear.weight", "trunk.3.linear.bias", "trunk.7.linear.bias", "sigma_head.weight",
            "geo_head.bias", "color_mlp.color_out.weight", "color_mlp.color_out.bias")
    new = dict(net.meta_named_parameters())
    for n in keep:
        arr[f"fast2/{n}"], arr[f"reptile/{n}"] = fast2[n].numpy(), new[n].detach().numpy()
    np.savez_compressed(os.path.join(OUT, "meta.npz"), **arr)


def gen_maml():
    """Second-order MAML (pipelines/offline_stage/meta_core.py:14-68 with algo="maml": create_graph=True, no
    autocast) of MetaNeRF(frequency) with the mlp.npz weights: 2 inner steps on 32 support rays, then the query loss
    on 32 other rays with the adapted fast weights and its backward to the MODULE parameters (meta_core.py:119-142
    fp32 branch, without the clip / step) — those gradients carry the second-order terms.  Also the same outer
    gradient with the inner gradient detached (first order), so a test can tell the two apart."""
    from models.inr.meta_vanilla import MetaNeRF                      # noqa: E402
    from nerfs.losses import compute_loss                              # noqa: E402
    from pipelines.offline_stage.meta_core import task_adapt          # noqa: E402
    z = np.load(os.path.join(OUT, "mlp.npz"))
    zr = np.load(os.path.join(OUT, "rays.npz"))
    torch.set_num_threads(8)

    class Expert(torch.nn.Module):  # as gen_meta
        def __init__(self, n):
            super().__init__(); self.net = n

        def forward(self, x_d, params=None):
            o = self.net(x_d[:, :3], x_d[:, 3:6], params=params)
            return torch.cat([o["rgb"], o["sigma"]], -1)

        def meta_named_parameters(self):
            return self.net.meta_named_parameters()

    class Model(torch.nn.Module):
        def __init__(self, e):
            super().__init__(); self.submodules = torch.nn.ModuleList([e]); self.use_occ = False

        def meta_named_parameters(self):
            return self.submodules[0].meta_named_parameters()

    g = torch.Generator().manual_seed(777)
    perm = torch.randperm(10000, generator=g)
    rays_s = torch.from_numpy(zr["rays_const"])[perm[:32]].contiguous()
    rays_q = torch.from_numpy(zr["rays_const"])[perm[32:64]].contiguous()
    gt_s, gt_q = torch.rand(32, 3, generator=g), torch.rand(32, 3, generator=g)
    arr = {"rays_s": rays_s.numpy(), "rays_q": rays_q.numpy(), "gt_s": gt_s.numpy(), "gt_q": gt_q.numpy()}
    keep = ("trunk.0.linear.weight", "trunk.4.linear.weight", "trunk.7.linear.bias", "sigma_head.weight",
            "geo_head.weight", "color_mlp.layer0.linear.weight", "color_mlp.color_out.bias")
    for algo in ("maml", "fomaml"):
        net = MetaNeRF(encoding_dir="frequency")
        with torch.no_grad():
            for n, p in net.meta_named_parameters():
                p.copy_(torch.from_numpy(z[f"w/{n}"]))
        model = Model(Expert(net)).eval()
        P = SimpleNamespace(algo=algo, fim=False, use_amp=False, ray_samples=32, chunk_points=1 << 20,
                            color_space="linear")
        fast, losses = task_adapt(P, model, {"rays": rays_s, "rgbs": gt_s}, inner_lr=0.05, iterations=2,
                                  active_module=0)
        q = compute_loss(P, model, {"rays": rays_q, "rgbs": gt_q}, params=fast, active_module=0)
        q.backward()
        grads = dict(net.meta_named_parameters())
        arr[f"{algo}/losses"] = torch.stack(losses).numpy()
        arr[f"{algo}/query"] = np.float32(q.item())
        for n in keep:
            arr[f"{algo}/grad/{n}"] = grads[n].grad.numpy()
            if algo == "maml":
                arr[f"{algo}/fast/{n}"] = fast[n].detach().numpy()
    np.savez_compressed(os.path.join(OUT, "maml.npz"), **arr)
    d = max(float(np.abs(arr[f"maml/grad/{n}"] - arr[f"fomaml/grad/{n}"]).max()) for n in keep)
    print("maml: query", arr["maml/query"], "max |grad maml - fomaml|", d)


def gen_amp():
    """The reference's AMP numerics (configs/train.json "use_amp": true; pipelines/online_stage/runtime_adapt.py:290-310:
    autocast(float16) around compute_mse_loss, scaler.scale(loss).backward() outside it).  Run on the CPU autocast,
    whose fp16 cast policy for matmul is CUDA's (lower-precision list); the arithmetic inside one fp16 matmul is the
    host's, so the fixture pins dtypes / clamps exactly and values to fp16 rounding.
      * dtype of trunc_exp's input: MetaLinear (metamodule.py:140-156) adds its fp32 bias to the fp16 matmul output,
        so type promotion makes the sigma pre-activation fp32 and trunc_exp clamps at 88.72, not 11.09;
      * te16: sigma_head weight 0, bias = x for x beyond +-11.09 -> sigma and d sigma / d bias under autocast;
      * a MetaNeRF forward + parameter gradients under autocast (mlp.npz weights, 256 samples);
      * one coarse-only train-loss + loss-scaled gradient (scale 2^16, unscaled) through render_rays on 64 rays."""
    from models.inr.meta_vanilla import MetaNeRF                      # noqa: E402
    from nerfs.losses import compute_mse_loss                         # noqa: E402
    z = np.load(os.path.join(OUT, "mlp.npz"))
    zr = np.load(os.path.join(OUT, "rays.npz"))
    net = MetaNeRF(encoding_dir="frequency")
    with torch.no_grad():
        for n, p in net.meta_named_parameters():
            p.copy_(torch.from_numpy(z[f"w/{n}"]))
    seen = []
    act = net.sigma_act

    def spy(x):
        seen.append(x.dtype)
        return act(x)

    net.sigma_act = spy

    class Expert(torch.nn.Module):
        def __init__(self, n):
            super().__init__(); self.net = n; self.use_occ = False; self.submodules = [self]

        def forward(self, x_d, params=None):
            o = self.net(x_d[:, :3], x_d[:, 3:6], params=params)
            return torch.cat([o["rgb"], o["sigma"]], -1)

    model = Expert(net).train()
    arr = {}
    x_d = torch.from_numpy(z["x_d"][:256])
    gup = torch.from_numpy(z["gup"][:256])
    with torch.autocast("cpu", dtype=torch.float16):
        out = model(x_d)
    grads = torch.autograd.grad((out * gup).sum(), list(net.parameters()))
    arr["out"] = out.detach().float().numpy()
    arr["out_bits"] = np.int32(torch.finfo(out.dtype).bits)            # 32: the expert's output is fp32
    arr["sigma_in_bits"] = np.int32(torch.finfo(seen[-1]).bits)       # 32: trunc_exp sees an fp32 tensor
    arr.update({f"g/{n}": gr.float().numpy() for (n, _), gr in zip(net.named_parameters(), grads)})
    # trunc_exp beyond the fp16 clamp, through the module under autocast
    te_x = [-30.0, -12.0, 0.0, 11.0, 12.0, 15.0, 30.0]
    ys, gs = [], []
    w0, b0 = net.sigma_head.weight.detach().clone(), net.sigma_head.bias.detach().clone()
    for x in te_x:
        with torch.no_grad():
            net.sigma_head.weight.zero_()
            net.sigma_head.bias.fill_(x)
        with torch.autocast("cpu", dtype=torch.float16):
            o = model(x_d[:8])
        gb, = torch.autograd.grad(o[:, 3].sum(), [net.sigma_head.bias])
        ys.append(float(o[0, 3])); gs.append(float(gb[0]) / 8.0)
    with torch.no_grad():
        net.sigma_head.weight.copy_(w0); net.sigma_head.bias.copy_(b0)
    arr["te16_x"], arr["te16_y"], arr["te16_g"] = (np.array(v, np.float32) for v in (te_x, ys, gs))
    # one coarse-only loss + scaled backward, as runtime_adapt.py:291-305 runs it
    g = torch.Generator().manual_seed(99)
    rays = torch.from_numpy(zr["rays_const"])[torch.randperm(10000, generator=g)[:64]].contiguous()
    gt = torch.rand(64, 3, generator=g)
    P = SimpleNamespace(ray_samples=32, chunk_points=1 << 20, color_space="linear")
    torch.manual_seed(5)  # stratified_t_vals' jitter draw (ray_rendering.py:286) is recorded below
    u = torch.rand(64, 32)
    torch.manual_seed(5)
    with torch.autocast("cpu", dtype=torch.float16):
        loss = compute_mse_loss(P, model, {"rays": rays, "rgbs": gt})
    scale = 65536.0
    sg = torch.autograd.grad(loss * scale, list(net.parameters()))
    arr["step_rays"], arr["step_gt"], arr["step_u"] = rays.numpy(), gt.numpy(), u.numpy()
    arr["step_loss"] = np.float32(loss.item())
    arr.update({f"sg/{n}": (gr.float() / scale).numpy() for (n, _), gr in zip(net.named_parameters(), sg)})
    np.savez_compressed(os.path.join(OUT, "amp.npz"), **arr)
    print("amp: sigma_in_dtype", seen[-1], "out", out.dtype, "te16_y", ys)


if __name__ == "__main__":
    if "--only-amp" in sys.argv:
        sys.dont_write_bytecode = True
        _install_stubs()
        sys.path.insert(0, REF)
        torch.set_num_threads(8)
        gen_amp()
    elif "--only-maml" in sys.argv:
        sys.dont_write_bytecode = True
        _install_stubs()
        sys.path.insert(0, REF)
        gen_maml()
    elif "--only-meta" in sys.argv:
        sys.dont_write_bytecode = True
        _install_stubs()
        sys.path.insert(0, REF)
        gen_meta()
    elif "--only-data" in sys.argv:
        sys.dont_write_bytecode = True
        _install_stubs()
        sys.path.insert(0, REF)
        gen_data()
    elif "--only-ngp" in sys.argv or "--only-moe" in sys.argv:
        sys.dont_write_bytecode = True
        _install_stubs()
        sys.path.insert(0, REF)
        torch.set_num_threads(8)
        gen_ngp() if "--only-ngp" in sys.argv else gen_moe()
    else:
        main()

