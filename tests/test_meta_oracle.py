"""CPU: the data-path / meta-learning oracle (oracle/meta_oracle.py) against the reference's golden vectors
(tests/golden/data.npz, meta.npz — tools/gen_golden.py gen_data / gen_meta), plus host-side pieces of
nerf_amd.data / nerf_amd.meta that need no GPU (DRZ layout discovery, metadata loading, val balancing)."""
import os
import sys
from collections import OrderedDict

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "nerf-sys_amd"))

from oracle import meta_oracle as MO  # noqa: E402
from oracle import nerf_oracle as O  # noqa: E402
from tests.golden_io import load, mlp_params  # noqa: E402

BOX = torch.tensor([[-1.5, -1.5, -1.5], [1.5, 1.5, 1.5]])


@pytest.mark.parametrize("i", [0, 1])
def test_process_single_image_golden(i):
    z = load("data")
    img = z[f"d{i}_img"]
    H, W = img.shape[:2]
    mask = z.get(f"d{i}_mask")
    ovr = (0.5, 4.0) if i == 1 else None
    rgbs, rays, idx = MO.process_single_image(img, mask, H, W, z[f"d{i}_K"], z[f"d{i}_c2w"], BOX,
                                              near_far_override=ovr, image_index=7 + i)
    assert torch.equal(idx, z[f"d{i}_idx"])
    assert torch.equal(rgbs, z[f"d{i}_rgbs"])
    torch.testing.assert_close(rays, z[f"d{i}_rays"], rtol=0, atol=2e-6)


def test_process_single_image_empty():
    z = load("data")
    img = z["d0_img"]
    H, W = img.shape[:2]
    assert MO.process_single_image(img, torch.zeros(H, W, dtype=torch.bool), H, W, z["d0_K"], z["d0_c2w"], BOX) is None
    # every ray misses the box -> no valid ray -> image dropped
    far = z["d0_c2w"].clone()
    far[:, 3] = torch.tensor([50.0, 50.0, 50.0])
    far[:, :3] = torch.eye(3)
    narrow = torch.tensor([100.0, 100.0, 15.7, 12.2])
    assert MO.process_single_image(img, None, H, W, narrow, far, BOX) is None


def test_task_adapt_golden():
    z = load("meta")
    p = mlp_params("w/")
    fast, losses = MO.task_adapt(O.vanilla_forward, p, z["rays"], z["gt"], 32, 0.05, 3)
    torch.testing.assert_close(torch.stack(losses), z["losses"], rtol=1e-5, atol=1e-7)
    for n, v in fast.items():
        torch.testing.assert_close(v.detach(), z[f"fast/{n}"], rtol=1e-4, atol=1e-6, msg=n)


def test_reptile_golden():
    z = load("meta")
    keep = [k[len("reptile/"):] for k in z if k.startswith("reptile/")]
    p = mlp_params("w/")
    theta = OrderedDict((n, p[n].clone()) for n in keep)
    f1 = OrderedDict((n, z[f"fast/{n}"].clone()) for n in keep)
    f1["geo_head.bias"] = p["geo_head.bias"].clone()
    f2 = OrderedDict((n, z[f"fast2/{n}"]) for n in keep)
    done = MO.reptile_update(theta, [f1, f2], 0.5)
    assert "trunk.3.linear.bias" not in done and "geo_head.bias" not in done
    for n in keep:
        assert torch.equal(theta[n], z[f"reptile/{n}"]), n


def test_val_balancing_moves_right_half():
    torch.manual_seed(0)
    H, W = 6, 8
    keep = torch.rand(H, W) > 0.5
    out = MO.val_balancing(keep, H, W).view(H, W)
    assert not out[:, W // 2:].any()
    assert out[:, : W // 2][keep[:, : W // 2]].all()      # kept left pixels stay kept
    n_free = int((~keep[:, : W // 2]).sum())
    assert int(out.sum()) == int(keep[:, : W // 2].sum()) + min(int(keep[:, W // 2:].sum()), n_free)


def test_host_val_balancing_matches_oracle():
    from nerf_amd.data import RamRaysDataset
    H, W = 10, 12
    keep = torch.rand(H, W, generator=torch.Generator().manual_seed(3)) > 0.6
    torch.manual_seed(11)
    a = RamRaysDataset._apply_meganerf_val_balancing_static(keep.clone(), H, W)
    torch.manual_seed(11)
    b = MO.val_balancing(keep.clone(), H, W)
    assert torch.equal(a, b)


def test_drz_layout_discovery(tmp_path):
    """dataset.py:185-291 layouts: split train/val with indices over the sorted union; metadata .pt files are
    read with weights_only=True; masks as plain .pt; PIL image decode."""
    from PIL import Image
    from nerf_amd.data import ImageMetadata, get_image_metadata, get_meta_lookups, load_coordinates
    import numpy as np
    torch.save({"origin_drb": torch.tensor([1.0, 2.0, 3.0]), "pose_scale_factor": 2.5}, tmp_path / "coordinates.pt")
    for split, names in (("train", ["a", "c"]), ("val", ["b"])):
        (tmp_path / split / "metadata").mkdir(parents=True)
        (tmp_path / split / "rgbs").mkdir()
        for nm in names:
            torch.save({"W": 8, "H": 6, "c2w": torch.eye(4)[:3], "intrinsics": torch.tensor([5.0, 5.0, 4.0, 3.0])},
                       tmp_path / split / "metadata" / f"{nm}.pt")
            Image.fromarray(np.full((6, 8, 3), ord(nm), np.uint8)).save(tmp_path / split / "rgbs" / f"{nm}.png")
    (tmp_path / "masks").mkdir()
    torch.save(torch.ones(6, 8, dtype=torch.bool), tmp_path / "masks" / "b.pt")
    o, s = load_coordinates(tmp_path)
    assert torch.equal(o, torch.tensor([1.0, 2.0, 3.0])) and s == 2.5
    tr, va = get_image_metadata(tmp_path, 0.5, mask_dir=tmp_path / "masks")
    assert [m.image_index for m in tr] == [0, 2] and [m.image_index for m in va] == [1]
    assert (tr[0].W, tr[0].H) == (4, 3) and torch.equal(tr[0].intrinsics, torch.tensor([2.5, 2.5, 2.0, 1.5]))
    img = tr[0].load_image()
    assert img.shape == (3, 4, 3) and img.dtype == torch.uint8          # LANCZOS-resized to (W, H)
    m = va[0].load_mask()
    assert m.shape == (3, 4) and m.all()                                 # nearest-resized mask
    assert tr[0].load_mask() is None
    lt, lv = get_meta_lookups(tr, va)
    assert lt == {0: {"H": 3, "W": 4}, 2: {"H": 3, "W": 4}} and lv == {1: {"H": 3, "W": 4}}
    assert isinstance(va[0], ImageMetadata)


def test_second_order_context():
    """second_order() (MAML create_graph=True, nerf_amd/second_order.py): active only inside the context with grad
    mode on; refuse() raises there and is a no-op outside."""
    from nerf_amd import second_order as so
    assert not so.active()
    so.refuse("x")
    with so.second_order():
        assert so.active()
        with torch.no_grad():
            assert not so.active()
            so.refuse("x")
        with pytest.raises(NotImplementedError):
            so.refuse("the Instant-NGP expert")
        with so.second_order():
            assert so.active()
        assert so.active()
    assert not so.active()


def test_second_order_volume_render_matches_oracle():
    """The torch composite of volume_render (second_order.py) equals the oracle's restatement on CPU tensors, and its
    gradient is itself differentiable (create_graph=True) — the property second-order MAML needs."""
    from nerf_amd import second_order as so
    from oracle import nerf_oracle as O
    g = torch.Generator().manual_seed(3)
    rs = torch.rand(5, 16, 4, generator=g, dtype=torch.float64)
    rs[..., 3] = torch.exp(torch.randn(5, 16, generator=g, dtype=torch.float64))
    t = torch.sort(torch.rand(5, 16, generator=g, dtype=torch.float64) * 4 + 2, dim=1).values
    bg = torch.rand(5, 3, generator=g, dtype=torch.float64)
    ours = so.volume_render(rs, t, bg)
    ref = O.volume_render(rs, t, bg)
    for a, b in zip(ours, ref):
        torch.testing.assert_close(a, b, rtol=1e-12, atol=1e-12)
    x = rs.clone().requires_grad_(True)
    gx, = torch.autograd.grad(so.volume_render(x, t, bg)[0].square().sum(), x, create_graph=True)
    hx, = torch.autograd.grad(gx.square().sum(), x)
    assert torch.isfinite(hx).all() and hx.abs().sum() > 0
