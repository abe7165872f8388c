"""CPU: the MoE-container restatement (oracle/moe_oracle.py) against the reference's golden vectors
(tests/golden/moe.npz, made by importing the reference: tools/gen_golden.py --only-moe)."""
from collections import OrderedDict

import pytest
import torch

from golden_io import load
from oracle import moe_oracle as MO
from oracle import ngp_oracle as NO

K = 3
CASES = {"soft": (1.05, True), "hard": (1.0, False)}


@pytest.fixture(scope="module")
def z():
    return load("moe")


def _experts(z, tag, leaves):
    res, _ = NO.hash_resolutions(4, 8, 128)
    exps = []
    for k in range(K):
        pre = f"{tag}_w/submodules.{k}."
        p = OrderedDict((n[len(pre):], leaves[n]) for n in leaves if n.startswith(pre))
        table = p.pop("xyz_encoder.hash_table")
        box = z[f"box{k}"]
        exps.append(lambda x_d, p=p, table=table, box=box: NO.ngp_forward(
            p, table, x_d, box, res, 10, 2, sigma_depth=1, color_depth=1))
    return exps


@pytest.mark.parametrize("tag", list(CASES))
def test_routing(z, tag):
    bm, c2d = CASES[tag]
    w, hard = MO.routing(z["x_d"][:, :3], z["centroids"], bm, c2d)
    if w is None:
        w = torch.nn.functional.one_hot(hard, K).float()
    torch.testing.assert_close(w, z[f"{tag}_route"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("tag", list(CASES))
def test_container_forward_backward(z, tag):
    bm, c2d = CASES[tag]
    leaves = OrderedDict((k, v.clone().requires_grad_(True)) for k, v in z.items() if k.startswith(f"{tag}_w/"))
    out = MO.container_forward(_experts(z, tag, leaves), z["x_d"], z["centroids"], bm, c2d)
    torch.testing.assert_close(out.detach(), z[f"{tag}_out"], rtol=1e-5, atol=1e-6)
    names = [n for n in leaves if "bg_mlp" not in n]
    grads = torch.autograd.grad((out * z[f"{tag}_gup"]).sum(), [leaves[n] for n in names], allow_unused=True)
    for n, gr in zip(names, grads):
        ref = z[f"{tag}_g/" + n[len(tag) + 3:]]
        gr = torch.zeros_like(ref) if gr is None else gr
        torch.testing.assert_close(gr, ref, rtol=1e-4, atol=1e-5 * max(1.0, float(ref.abs().max())), msg=n)


def test_background_color(z):
    p = {k[len("soft_w/"):]: v.clone().requires_grad_(True) for k, v in z.items() if k.startswith("soft_w/bg_mlp")}
    out = MO.background_color(z["bg_d"], p["bg_mlp.0.weight"], p["bg_mlp.0.bias"], p["bg_mlp.2.weight"],
                              p["bg_mlp.2.bias"])
    torch.testing.assert_close(out.detach(), z["bg_out"], rtol=1e-6, atol=1e-6)
    grads = torch.autograd.grad((out * z["bg_gup"]).sum(), list(p.values()))
    for (n, _), gr in zip(p.items(), grads):
        torch.testing.assert_close(gr, z[f"bg_g/{n}"], rtol=1e-5, atol=1e-6)
