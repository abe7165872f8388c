"""CPU-only checks: the C-ABI library loads and exports every symbol include/nerf_amd.h declares, the
host-side packed layout, and the product path's refusal to run on CPU tensors (no fallback)."""
import os
import re
import subprocess

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    txt = open(os.path.join(ROOT, "include", "nerf_amd.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(nerf_[a-z_0-9]+)\s*\(", txt, flags=re.M)))


def test_library_exports_header_symbols():
    from nerf_amd._lib import LIB_PATH, EXPORTS, lib
    assert os.path.exists(LIB_PATH), "build first: make -C nerf-sys_amd"
    syms = _header_symbols()
    assert len(syms) >= 17
    out = subprocess.run(["nm", "-D", "--defined-only", LIB_PATH], capture_output=True, text=True).stdout
    exported = set(l.split()[-1] for l in out.splitlines() if l.strip())
    missing = [s for s in syms if s not in exported]
    assert not missing, missing
    assert set(syms) == set(EXPORTS)
    L = lib()
    assert b"gfx950" in L.nerf_version()


def test_library_built_from_this_tree():
    """nerf_version() carries the hash of the sources the .so was linked from (Makefile): a prebuilt library that
    does not match HEAD's csrc/ + include/ fails here instead of being tested silently."""
    from nerf_amd._lib import built_hash, source_hash
    assert built_hash() == source_hash(), "libnerf_amd.so is stale: rebuild with `make -C nerf-sys_amd`"


def test_packed_layout_roundtrip():
    from nerf_amd.vanilla import PackedLayout, PARAM_SHAPES, NUM_PARAMS
    L = PackedLayout.get()
    assert NUM_PARAMS == 503059
    assert L.total >= NUM_PARAMS and L.total % 32 == 0
    assert L.all_index.unique().numel() == NUM_PARAMS  # injective
    assert L.all_index.max() < L.total
    g = torch.Generator().manual_seed(0)
    ts = [torch.randn(s, generator=g) for s in PARAM_SHAPES.values()]
    packed = L.pack([t.requires_grad_(True) for t in ts])
    un = L.unpack(packed)
    for (n, s), t in zip(PARAM_SHAPES.items(), ts):
        assert torch.equal(un[n], t.detach())
    # pack is differentiable: gradient of sum(packed * c) w.r.t. each tensor = c at its slots
    c = torch.randn(L.total, generator=g)
    grads = torch.autograd.grad((packed * c).sum(), ts)
    for (n, _), gr in zip(PARAM_SHAPES.items(), grads):
        assert torch.equal(gr.reshape(-1), c[L.index[n]])
    # padding slots are zero
    mask = torch.ones(L.total, dtype=torch.bool)
    mask[L.all_index] = False
    assert (packed.detach()[mask] == 0).all()


def test_workspace_sizes():
    from nerf_amd._lib import lib
    L = lib()
    a = L.nerf_mlp_workspace_bytes(4096 * 192, 1)
    b = L.nerf_mlp_workspace_bytes(4096 * 192, 0)
    assert a > b > 0
    assert L.nerf_mlp_workspace_bytes(1, 1) > 0
    assert L.nerf_mlp_workspace_bytes(-1, 1) == -1


def test_no_cpu_fallback():
    from nerf_amd import kernels as K
    with pytest.raises(ValueError, match="no CPU fallback"):
        K.freq_encode(torch.zeros(4, 3), 4)
    from nerf_amd.vanilla import VanillaNeRF
    with pytest.raises(ValueError):
        VanillaNeRF()(torch.zeros(8, 6))


def test_graft_build_entry_imports():
    import importlib.util
    spec = importlib.util.spec_from_file_location("ge", os.path.join(ROOT, "__graft_entry__.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    assert callable(m.build) and callable(m.smoke)


def test_engine_refuses_fp16():
    """The fused engine has no loss scaling / inf-skip: fp16 is for the autocast + GradScaler drop-in loop only
    (ADVICE r05)."""
    from nerf_amd.trainer import NeRFTrainer
    from nerf_amd.vanilla import VanillaNeRF
    with pytest.raises(ValueError, match="fp16"):
        NeRFTrainer(VanillaNeRF(), VanillaNeRF(), device="cpu", precision="fp16")


def test_engine_overlap_with_values():
    """The coarse backward's stream placement: "bwd" (default, beside the fine backward) or "fwd"; anything else is
    refused.  (On a CPU device there is no side stream: overlap is off.)"""
    from nerf_amd.trainer import NeRFTrainer
    from nerf_amd.vanilla import VanillaNeRF
    tr = NeRFTrainer(VanillaNeRF(), VanillaNeRF(), device="cpu")
    assert tr.overlap_with == "bwd" and not tr.overlap
    with pytest.raises(ValueError, match="overlap_with"):
        NeRFTrainer(VanillaNeRF(), VanillaNeRF(), device="cpu", overlap_with="tail")
