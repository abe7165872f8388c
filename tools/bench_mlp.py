#!/usr/bin/env python3
"""Kernel-level timing of the MLP passes alone (no compositing, no overlap): HIP-event time of nerf_mlp_fwd /
nerf_mlp_bwd (fp32 or bf16) at the C2 fine-net size (M = 4096 x 192 = 786,432 samples), training and inference,
with the algorithmic rates: MFMA FLOP = 2 * 500,864 MAC per sample (forward), 4 * MAC (backward).

  python tools/bench_mlp.py [--precision bf16] [--M 786432] [--iters 20]

--bf16-flags selects the layered bf16 launches for A/B runs (1 = layer-by-layer forward, 2 = layered backward)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "nerf-sys_amd")]

import torch  # noqa: E402

MAC = 500864


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="bf16", choices=["fp32", "bf16"])
    ap.add_argument("--M", type=int, default=786432)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--bf16-flags", type=int, default=0)
    a = ap.parse_args()
    from nerf_amd import kernels as K
    from nerf_amd.vanilla import VanillaNeRF
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    w = VanillaNeRF().to(dev).packed().detach().contiguous()
    g = torch.Generator().manual_seed(1)
    x = torch.cat([torch.rand(a.M, 3, generator=g) * 3 - 1.5,
                   torch.nn.functional.normalize(torch.randn(a.M, 3, generator=g), dim=-1)], -1).to(dev)
    gup = (torch.randn(a.M, 4, generator=g) * 1e-3).to(dev)
    ws_t = K.mlp_workspace(a.M, True, dev, a.precision)
    ws_i = K.mlp_workspace(a.M, False, dev, a.precision)
    out = torch.empty(a.M, 4, device=dev)
    d_w = torch.empty_like(w)

    def timeit(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.iters

    res = {"precision": a.precision, "M": a.M, "bf16_flags": a.bf16_flags}
    fl = a.bf16_flags
    res["fwd_infer_ms"] = timeit(lambda: K.mlp_fwd(w, x, ws_i, False, out=out, precision=a.precision, bf16_flags=fl))
    res["fwd_train_ms"] = timeit(lambda: K.mlp_fwd(w, x, ws_t, True, out=out, precision=a.precision, bf16_flags=fl))
    K.mlp_fwd(w, x, ws_t, True, out=out, precision=a.precision, bf16_flags=fl)
    res["bwd_ms"] = timeit(lambda: K.mlp_bwd(w, a.M, gup, ws_t, d_w=d_w, precision=a.precision, bf16_flags=fl))
    for k in ("fwd_infer", "fwd_train"):
        res[k + "_tflops"] = round(2 * MAC * a.M / (res[k + "_ms"] * 1e-3) / 1e12, 1)
    res["bwd_tflops"] = round(4 * MAC * a.M / (res["bwd_ms"] * 1e-3) / 1e12, 1)
    for k in ("fwd_infer_ms", "fwd_train_ms", "bwd_ms"):
        res[k] = round(res[k], 4)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
