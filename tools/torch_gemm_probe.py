#!/usr/bin/env python3
"""Reference point for the fp32 trunk GEMMs: what the vendor library (torch.mm -> hipBLASLt / rocBLAS) reaches on the
C2 fine-net shapes (M = 786,432 rows, 256 x 256 weights, fp32, no TF32 on gfx950) next to this repo's kernels
(bench.py roofline classes: fwd / dgrad / wgrad).  HIP-event time per call, best of 10 after warm-up."""
import json

import torch


def t(fn, it=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(it):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return best


def main():
    torch.backends.cuda.matmul.allow_tf32 = False
    M, N, K = 786432, 256, 256
    g = torch.Generator(device="cuda").manual_seed(0)
    X = torch.randn(M, K, device="cuda", generator=g)
    W = torch.randn(N, K, device="cuda", generator=g)
    G = torch.randn(M, N, device="cuda", generator=g)
    out = torch.empty(M, N, device="cuda")
    dw = torch.empty(N, K, device="cuda")
    flop = 2.0 * M * N * K
    res = {}
    res["fwd X@W^T"] = t(lambda: torch.mm(X, W.t(), out=out))
    res["dgrad G@W"] = t(lambda: torch.mm(G, W, out=out))
    res["wgrad G^T@X"] = t(lambda: torch.mm(G.t(), X, out=dw))
    print(json.dumps({k: {"ms": round(v, 4), "tflops": round(flop / (v * 1e-3) / 1e12, 1),
                          "frac_of_157.3": round(flop / (v * 1e-3) / 1e12 / 157.3, 3)} for k, v in res.items()}))


if __name__ == "__main__":
    main()
