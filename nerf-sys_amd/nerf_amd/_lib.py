"""ctypes binding of libnerf_amd.so (include/nerf_amd.h).

This is the only place the product path touches native code.  There is NO CPU fallback: if the
library is missing the import of any op raises, and every op requires CUDA(=HIP) tensors.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_double, c_float, c_int, c_int64, c_uint64, c_void_p

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NERF_AMD_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libnerf_amd.so"))

_ERR = {-1: "invalid argument", -2: "pointer not 16-byte aligned", -3: "unknown enum value",
        -4: "workspace too small"}

_lib = None


def source_hash() -> str:
    """The hash the Makefile bakes into nerf_version(): sha256 over csrc/*.hip + csrc/*.hpp (byte order of their
    paths) followed by include/nerf_amd.h, first 16 hex digits.  Equal to the loaded library's `src=` field iff that
    library was built from this tree's sources."""
    import glob
    import hashlib
    pkg = os.path.dirname(_HERE)
    rel = sorted(os.path.relpath(p, pkg) for p in glob.glob(os.path.join(pkg, "csrc", "*.hip")) +
                 glob.glob(os.path.join(pkg, "csrc", "*.hpp")))
    h = hashlib.sha256()
    for r in rel + [os.path.join("..", "include", "nerf_amd.h")]:
        with open(os.path.join(pkg, r), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def built_hash() -> str:
    """The `src=` field of the loaded library's nerf_version()."""
    v = lib().nerf_version().decode()
    return v.split("src=", 1)[1] if "src=" in v else ""


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libnerf_amd.so not built ({LIB_PATH}); run `python __graft_entry__.py build`"
                               " or `make -C nerf-sys_amd` — there is no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        P, I, I64, F, D, U64 = c_void_p, c_int, c_int64, c_float, c_double, c_uint64
        sig = {
            "nerf_rays_gen": [P, I, P, I64, I, I, F, F, F, F, I, F, F, P, F, F, P, P, P, P],
            "nerf_pick_pixels": [I64, I, I, I, U64, P, P],
            "nerf_pick_pixels_dseed": [I64, I, I, I, U64, U64, P, P, P],
            "nerf_adam_dstep": [P, P, P, P, I64, P, P, I, D, D, F, F, P, P, F, P],
            "nerf_occ_march_multi_staged_dseed": [P, P, P, P, I, P, I64, F, F, F, I, U64, I, P, P, I, P, P, P, P, P,
                                                  U64, P],
            "nerf_clamp_near_far": [P, I64, I, F, I, F, F, F, P, P],
            "nerf_rays_ndc": [P, I64, I, I, F, F, P, P],
            "nerf_sample_stratified": [P, I64, I, I, P, U64, P, P],
            "nerf_build_xd": [P, P, I64, I, P, P],
            "nerf_sample_pdf": [P, P, I64, I, I, P, I, U64, P, P],
            "nerf_freq_encode": [P, I64, I, I, I, P, I, P],
            "nerf_mlp_layout": [P],
            "nerf_mlp_workspace_bytes": [I64, I],
            "nerf_mlp_fwd": [P, P, I64, P, P, I64, I, P, P],
            "nerf_mlp_bwd": [P, I64, P, P, I, P, I64, P, P],
            "nerf_mlp_workspace_bytes_2s": [I64],
            "nerf_mlp_bwd_2s": [P, I64, P, P, I, P, I64, P, P, P, P],
            "nerf_mlp_fwd_ex": [P, P, I64, P, P, I64, I, I, P, P],
            "nerf_mlp_bwd_ex": [P, I64, P, P, I, P, I64, I, P, P],
            "nerf_mlp_bwd_2s_ex": [P, I64, P, P, I, P, I64, I, P, P, P, P],
            "nerf_mlp_workspace_bytes_bf16": [I64, I],
            "nerf_mlp_fwd_bf16": [P, P, I64, P, P, I64, I, I, P, P],
            "nerf_mlp_bwd_bf16": [P, I64, P, P, I, P, I64, I, P, P],
            "nerf_mlp_workspace_bytes_f16": [I64, I],
            "nerf_mlp_fwd_f16": [P, P, I64, P, P, I64, I, I, P, P],
            "nerf_mlp_bwd_f16": [P, I64, P, P, I, P, I64, I, P, P],
            "nerf_composite_fwd": [P, P, P, I64, I, F, P, P, P, P, P, I, F, P, P, P],
            "nerf_composite_bwd": [P, P, P, I64, I, F, P, P, P, P, P, P],
            "nerf_grad_sqnorm": [P, I64, P, P],
            "nerf_adam": [P, P, P, P, I64, P, P, I, D, D, F, F, I, P, F, P],
            "nerf_version": [],
            "nerf_hash_encode": [P, P, P, I64, I64, P, F, P, I, P],
            "nerf_hash_encode_bwd": [P, P, I64, I64, P, F, P, I, P, P],
            "nerf_sh_encode": [P, I64, I64, I, P, I, P],
            "nerf_ngp_layout": [P, P, P],
            "nerf_ngp_workspace_bytes": [P, I64],
            "nerf_ngp_fwd": [P, P, P, I, P, I64, P, P],
            "nerf_ngp_density": [P, P, P, I, I64, P, P],
            "nerf_ngp_density_enc": [P, P, P, P, P, I64, I64, P, F, P, P],
            "nerf_ngp_fwd_enc": [P, P, P, P, P, I64, P, F, P, I, P, P],
            "nerf_ngp_bwd_hash": [P, P, P, P, I, P, I64, P, P, F, P, P, I, P, I64, P],
            "nerf_ngp_fwd_enc_n": [P, P, P, P, P, I64, P, P, F, P, I, P, P],
            "nerf_ngp_density_enc_rng": [P, P, P, P, P, I64, I64, P, P, F, P, P],
            "nerf_ngp_bwd_hash_n": [P, P, P, P, I, P, I64, P, P, P, F, P, P, I, P, I64, P],
            "nerf_moe_dispatch_n": [P, I64, P, I, F, P, P, P, I64, P],
            "nerf_gather_rows_rng": [P, I64, P, P, I64, I, P, I64, P],
            "nerf_moe_blend_rng": [P, I64, P, P, P, I, I, P, P, P],
            "nerf_moe_blend_finish_n": [P, P, I64, P, P, P],
            "nerf_moe_blend_bwd_rng": [P, I64, P, P, P, I, I, P, P, P, P, P],
            "nerf_ngp_bwd": [P, P, P, I, P, I64, P, P, P, I, P, I64, P],
            "nerf_moe_route": [P, I64, I64, P, I, I, F, P, P],
            "nerf_moe_route_n": [P, I64, I64, P, P, I, I, F, P, P],
            "nerf_moe_dispatch_workspace_bytes": [I64, I],
            "nerf_moe_dispatch": [P, I64, I, F, P, P, P, I64, P],
            "nerf_gather_rows": [P, I64, P, I64, I, P, I64, P],
            "nerf_moe_combine": [P, I64, I, P, P, I, I, P, P],
            "nerf_moe_combine_bwd": [P, I64, I, P, P, I, I, P, P],
            "nerf_bg_mlp_fwd": [P, I64, I64, P, I, P, P],
            "nerf_bg_mlp_workspace_bytes": [I64, I],
            "nerf_bg_mlp_bwd": [P, I64, I64, P, I, P, P, P, I64, P],
            "nerf_occ_march": [P, P, P, I64, F, F, F, F, I, P, U64, I, P, P, P, P, P, P],
            "nerf_scan_workspace_bytes": [I64],
            "nerf_exclusive_scan_i32": [P, I64, P, P, I64, P],
            "nerf_packed_composite_fwd": [P, P, P, P, I64, P, P, P, P, P, P],
            "nerf_packed_composite_bwd": [P, P, P, P, I64, P, P, P, P, P, P, P],
            "nerf_packed_visibility": [P, P, P, P, I64, F, F, P, P],
            "nerf_packed_visibility_groups": [P, P, P, P, I64, I64, F, F, P, P, P],
            "nerf_occ_march_multi": [P, P, P, P, I, P, I64, F, F, F, I, U64, I, P, P, P, P, P, P],
            "nerf_occ_march_multi_staged": [P, P, P, P, I, P, I64, F, F, F, I, U64, I, P, P, I, P, P, P, P, P],
            "nerf_packed_compact": [P, P, I64, P, P, P, P, P, P, P, P],
            "nerf_occ_cell_points": [P, P, I64, U64, P, P],
            "nerf_occ_update": [P, P, P, I64, F, P],
            "nerf_occ_sample_cells": [P, P, I, I64, I64, U64, P, P],
            "nerf_occ_threshold": [P, I64, F, P, P],
            "nerf_occ_binarize": [P, I64, P, P, P],
            "nerf_occ_mark_invisible": [P, P, P, I, I, I, F, P, P],
            "nerf_ray_counts": [P, I64, I64, P, P],
            "nerf_packed_points": [P, P, P, P, I64, P, P],
            "nerf_packed_points_n": [P, P, P, P, I64, P, P, P],
            "nerf_rays_aabb_hit": [P, I64, P, P, P],
            "nerf_occ_threshold_floats": [],
            "nerf_sgd_multi": [I, P, P, P, P, F, P],
            "nerf_reptile_workspace_bytes": [I],
            "nerf_reptile_update": [I, P, P, I, P, F, P, I64, P],
            "nerf_dataset_rays": [P, P, P, I, I, I, I, P, I, F, I, F, P, P, P, P, P, P, P, P],
            "nerf_flag_compact": [P, P, I64, P, P],
            "nerf_scatter_counts": [P, P, I64, P, P],
            "nerf_segments_union": [P, P, P, I, I64, P, P, P, P, P, P],
            "nerf_moe_blend": [P, I64, P, P, I, I, P, P, P],
            "nerf_moe_blend_finish": [P, P, I64, P, P],
            "nerf_moe_blend_bwd": [P, I64, P, P, I, I, P, P, P, P, P],
        }
        ab = "NERF_AMD_LIB" in os.environ  # an A/B build of an older revision may lack the newer entry points
        for name, args in sig.items():
            try:
                fn = getattr(L, name)
            except AttributeError:
                if ab:
                    continue
                raise
            fn.argtypes = args
            fn.restype = c_int
        L.nerf_mlp_layout.restype = c_int64
        L.nerf_mlp_workspace_bytes.restype = c_int64
        L.nerf_mlp_workspace_bytes_2s.restype = c_int64
        L.nerf_mlp_workspace_bytes_bf16.restype = c_int64
        L.nerf_mlp_workspace_bytes_f16.restype = c_int64
        L.nerf_version.restype = ctypes.c_char_p
        L.nerf_ngp_layout.restype = c_int64
        L.nerf_ngp_workspace_bytes.restype = c_int64
        L.nerf_moe_dispatch_workspace_bytes.restype = c_int64
        L.nerf_bg_mlp_workspace_bytes.restype = c_int64
        L.nerf_scan_workspace_bytes.restype = c_int64
        L.nerf_occ_threshold_floats.restype = c_int64
        L.nerf_reptile_workspace_bytes.restype = c_int64
        _lib = L
    return _lib


EXPORTS = ("nerf_rays_gen", "nerf_pick_pixels", "nerf_clamp_near_far", "nerf_rays_ndc",
           "nerf_sample_stratified", "nerf_build_xd", "nerf_sample_pdf", "nerf_freq_encode",
           "nerf_mlp_layout", "nerf_mlp_workspace_bytes", "nerf_mlp_fwd", "nerf_mlp_bwd",
           "nerf_mlp_workspace_bytes_2s", "nerf_mlp_bwd_2s", "nerf_mlp_fwd_ex", "nerf_mlp_bwd_ex", "nerf_mlp_bwd_2s_ex",
           "nerf_mlp_workspace_bytes_bf16", "nerf_mlp_fwd_bf16", "nerf_mlp_bwd_bf16",
           "nerf_mlp_workspace_bytes_f16", "nerf_mlp_fwd_f16", "nerf_mlp_bwd_f16",
           "nerf_composite_fwd", "nerf_composite_bwd", "nerf_grad_sqnorm", "nerf_adam", "nerf_version",
           "nerf_hash_encode", "nerf_hash_encode_bwd", "nerf_sh_encode", "nerf_ngp_layout",
           "nerf_ngp_workspace_bytes", "nerf_ngp_fwd", "nerf_ngp_bwd", "nerf_moe_route",
           "nerf_moe_dispatch_workspace_bytes", "nerf_moe_dispatch", "nerf_gather_rows", "nerf_moe_combine",
           "nerf_moe_combine_bwd", "nerf_bg_mlp_fwd", "nerf_bg_mlp_workspace_bytes", "nerf_bg_mlp_bwd",
           "nerf_occ_march", "nerf_scan_workspace_bytes", "nerf_exclusive_scan_i32", "nerf_packed_composite_fwd",
           "nerf_packed_composite_bwd", "nerf_packed_visibility", "nerf_packed_compact", "nerf_occ_cell_points",
           "nerf_occ_update", "nerf_occ_threshold", "nerf_occ_binarize", "nerf_occ_mark_invisible", "nerf_ray_counts",
           "nerf_packed_points", "nerf_rays_aabb_hit", "nerf_flag_compact", "nerf_scatter_counts", "nerf_segments_union",
           "nerf_moe_blend", "nerf_moe_blend_finish", "nerf_moe_blend_bwd", "nerf_occ_threshold_floats",
           "nerf_sgd_multi", "nerf_reptile_workspace_bytes", "nerf_reptile_update", "nerf_dataset_rays",
           "nerf_occ_march_multi", "nerf_occ_march_multi_staged", "nerf_packed_visibility_groups", "nerf_ngp_density", "nerf_ngp_density_enc", "nerf_ngp_fwd_enc", "nerf_ngp_bwd_hash",
           "nerf_occ_sample_cells", "nerf_moe_route_n", "nerf_ngp_fwd_enc_n", "nerf_ngp_density_enc_rng",
           "nerf_ngp_bwd_hash_n", "nerf_moe_dispatch_n", "nerf_gather_rows_rng", "nerf_moe_blend_rng",
           "nerf_moe_blend_finish_n", "nerf_moe_blend_bwd_rng",
           "nerf_packed_points_n", "nerf_pick_pixels_dseed", "nerf_adam_dstep", "nerf_occ_march_multi_staged_dseed")


def check(status: int, what: str) -> None:
    if status != 0:
        msg = _ERR.get(status, f"hipError {status}")
        if status in (-1, -3):
            raise ValueError(f"{what}: {msg}")
        raise RuntimeError(f"{what}: {msg}")


def ptr(t):
    """Device pointer of a CUDA tensor (None -> NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError("nerf_amd ops take HIP device tensors only (no CPU fallback)")
    return c_void_p(t.data_ptr())


def stream():
    """The current HIP stream of the current device (the raw handle torch's own kernel launchers use)."""
    return c_void_p(torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice()))


def need(t, name, dtype=torch.float32):
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise ValueError(f"{name} must be a HIP device tensor (no CPU fallback)")
    if t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    return t
