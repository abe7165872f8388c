#!/usr/bin/env python3
"""Where a split NT GEMM workgroup's time goes, from the s_memtime stamps of a diagnostic build
(tools/build_exp.sh stamps "-DNERF_X6W_STAMPS"; gemm_x6.hpp X6W_STAMP): workgroup 777 of the last forward
(64-row waves, bias + ReLU) and of the last input-gradient (BIGSMALL) launch records, per wave, the shader clock at
every pipeline point of each slab.  Runs one C2 fine-net MLP forward + backward (M = 786,432) and prints, per kernel,
the mean per-slab segment lengths over the 8 waves and the middle slabs (cycles):
  split ks0 | mfma ks0 | split ks1 | mfma ks1 | A-load issue + weight wait | weight LDS store + barrier

  NERF_AMD_LIB=exp/stamps.so python tools/x6_stamps.py"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "nerf-sys_amd")]

import torch  # noqa: E402


def main():
    from nerf_amd import kernels as K
    from nerf_amd._lib import lib
    from nerf_amd.vanilla import VanillaNeRF
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    M = 786432
    w = VanillaNeRF().to(dev).packed().detach().contiguous()
    g = torch.Generator().manual_seed(1)
    x = torch.cat([torch.rand(M, 3, generator=g) * 3 - 1.5,
                   torch.nn.functional.normalize(torch.randn(M, 3, generator=g), dim=-1)], -1).to(dev)
    gup = (torch.randn(M, 4, generator=g) * 1e-3).to(dev)
    ws = K.mlp_workspace(M, True, dev)
    buf = (ctypes.c_ulonglong * (2 * 8 * 128))()
    L = lib()
    L.nerf_debug_x6_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    for _ in range(2):
        K.mlp_fwd(w, x, ws, True)
        K.mlp_bwd(w, M, gup, ws)
    torch.cuda.synchronize()
    assert L.nerf_debug_x6_stamps(None, 1) == 0  # clear: only the last forward / backward below leave stamps
    K.mlp_fwd(w, x, ws, True)
    K.mlp_bwd(w, M, gup, ws)
    torch.cuda.synchronize()
    rc = L.nerf_debug_x6_stamps(ctypes.addressof(buf), 0)
    assert rc == 0, rc
    names = ["split ks0", "mfma ks0", "split ks1", "mfma ks1", "A issue+B wait", "B store+barrier"]
    out = {}
    for kind, kname in ((0, "fwd (64-row waves)"), (1, "dgrad (BIGSMALL, 32-row waves)")):
        waves = []
        for wv in range(8):
            st = [buf[(kind * 8 + wv) * 128 + i] for i in range(128)]
            # the last launch of each kind (trunk.7 forward, trunk.1 input gradient) has K = 256: 8 slabs, 1 + 8 x 6
            # stamps + the epilogue's; entries past them are stale from the K = 320 trunk.4 launch
            waves.append(st[:2 + 8 * 6])
        # layout: s0 = loop start; per slab 6 stamps (V0 M0 V1 M1 W T), then the epilogue end
        per_wave = []
        for st in waves:
            if len(st) < 8:
                continue
            slabs = (len(st) - 2) // 6
            segs = []
            for k in range(slabs):
                base = st[k * 6]  # the previous slab's post-barrier stamp (or the loop start)
                pts = st[k * 6 + 1:k * 6 + 7]
                prev = [base] + pts[:-1]
                segs.append([b - a for a, b in zip(prev, pts)])
            epi = st[-1] - st[slabs * 6]
            per_wave.append((segs, epi, st[-1] - st[0]))
        if not per_wave:
            out[kname] = "no stamps"
            continue
        slabs = len(per_wave[0][0])
        mid = range(1, max(2, slabs - 1))
        mean_seg = [sum(pw[0][k][s] for pw in per_wave for k in mid) / (len(per_wave) * len(mid)) for s in range(6)]
        out[kname] = {"slabs": slabs, "mean_segment_cycles": {n: round(v) for n, v in zip(names, mean_seg)},
                      "slab_cycles": round(sum(mean_seg)),
                      "epilogue_cycles": round(sum(pw[1] for pw in per_wave) / len(per_wave)),
                      "tile_cycles": round(sum(pw[2] for pw in per_wave) / len(per_wave)),
                      "per_wave_slab_cycles": [round(sum(sum(pw[0][k]) for k in mid) / len(mid)) for pw in per_wave]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
