"""CPU: the Instant-NGP restatement (oracle/ngp_oracle.py) against the reference's golden vectors
(tests/golden/ngp.npz, made by importing the reference: tools/gen_golden.py --only-ngp)."""
from collections import OrderedDict

import pytest
import torch

from golden_io import load
from oracle import ngp_oracle as NO

HCFG = {"a": (4, 2, 12, 16, 4096, "Linear"), "b": (16, 2, 12, 16, 2048, "Smoothstep"),
        "c": (8, 4, 10, 4, 300, "Nearest"), "d": (8, 1, 11, 16, 512, "Linear")}
MCFG = {"m1": dict(levels=8, F=2, log2T=12, min_res=16, max_res=1024, hidden=64, sigma_depth=2, color_hidden=64,
                   color_depth=2, dir_encoding="spherical"),
        "m2": dict(levels=16, F=2, log2T=11, min_res=16, max_res=2048, hidden=32, sigma_depth=1, color_hidden=48,
                   color_depth=3, dir_encoding="frequency")}


@pytest.fixture(scope="module")
def z():
    return load("ngp")


@pytest.mark.parametrize("lv", [1, 2, 3, 4, 5])
def test_sh(z, lv):
    torch.testing.assert_close(NO.sh_encode(z["sh_d"], lv), z[f"sh_{lv}"], rtol=0, atol=1e-6)


@pytest.mark.parametrize("tag", list(HCFG))
def test_hash_encode(z, tag):
    L, F, log2T, mn, mx, interp = HCFG[tag]
    res, _ = NO.hash_resolutions(L, mn, mx)
    assert torch.equal(res, z[f"hash_{tag}_res"])
    table = z[f"hash_{tag}_table"].clone().requires_grad_(True)
    y = NO.hash_encode(table, z["hash_x"], res, log2T, F, interp)
    assert torch.equal(y.detach(), z[f"hash_{tag}_out"])
    gt, = torch.autograd.grad((y * z[f"hash_{tag}_gup"]).sum(), [table])
    torch.testing.assert_close(gt, z[f"hash_{tag}_gtable"], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("tag", list(MCFG))
def test_ngp_forward_backward(z, tag):
    c = MCFG[tag]
    res, _ = NO.hash_resolutions(c["levels"], c["min_res"], c["max_res"])
    assert torch.equal(res, z[f"{tag}_res"])
    w = OrderedDict((k[len(tag) + 3:], v.clone().requires_grad_(True)) for k, v in z.items()
                    if k.startswith(f"{tag}_w/"))
    table = w.pop("xyz_encoder.hash_table")
    out = NO.ngp_forward_ad(w, table, z["ngp_x_d"], z["ngp_aabb"], res, c["log2T"], c["F"],
                            sigma_depth=c["sigma_depth"], color_depth=c["color_depth"],
                            dir_encoding=c["dir_encoding"])
    torch.testing.assert_close(out.detach(), z[f"{tag}_out"], rtol=1e-5, atol=1e-6)
    names = list(w) + ["xyz_encoder.hash_table"]
    grads = torch.autograd.grad((out * z[f"{tag}_gup"]).sum(), list(w.values()) + [table])
    for n, gr in zip(names, grads):
        ref = z[f"{tag}_g/{n}"]
        torch.testing.assert_close(gr, ref, rtol=1e-4, atol=1e-5 * max(1.0, float(ref.abs().max())), msg=n)


def test_shapes_match_reference(z):
    for tag, c in MCFG.items():
        dd = 16 if c["dir_encoding"] == "spherical" else 27
        shapes = NO.ngp_param_shapes(c["levels"] * c["F"], c["hidden"], c["sigma_depth"], 15, c["color_hidden"],
                                     c["color_depth"], dd)
        ref = {k[len(tag) + 3:]: tuple(v.shape) for k, v in z.items() if k.startswith(f"{tag}_w/")}
        ref.pop("xyz_encoder.hash_table")
        assert list(ref) == list(shapes) and all(ref[k] == shapes[k] for k in ref)
