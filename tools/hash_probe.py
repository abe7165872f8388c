#!/usr/bin/env python3
"""Per-level cost probe of the hash-grid kernels (forward gather / backward scatter) on the NGP bench's
sample distribution: 4096 random pixels x 96 stratified samples through the [-1.5,1.5]^3 box, the
production 16-level grid (2^20 entries, F=2).  Times subsets of levels by passing sub-grids."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "nerf-sys_amd"), ROOT]
import torch  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    from nerf_amd import ngp as G, kernels as K
    from nerf_amd.scene import make_blender_scene
    from nerf_amd.trainer import RayBatcher
    torch.manual_seed(0)
    scene = make_blender_scene(n_train=20, n_test=1, H=800, W=800, seed=0, device=dev)
    rays, _ = RayBatcher(scene, dev).batch(4096, seed=1)
    t = K.sample_stratified(rays, 96, True, None, 1)
    xd = K.build_xd(rays, t)
    res, _ = G.level_resolutions(16, 16, 4096)
    T = 2 ** 20
    table = torch.randn(16 * T, 2, device=dev) * 0.1
    aabb = [-1.5, -1.5, -1.5, 1.5, 1.5, 1.5]
    M = xd.shape[0]

    def grid_of(levels):
        g = G.NerfHashGrid()
        g.levels, g.features_per_level, g.log2_hashmap_size, g.interpolation = len(levels), 2, 20, 1
        for i, l in enumerate(levels):
            g.resolutions[i] = int(res[l])
        return g

    def timeit(fn, n=10):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n

    print(f"M = {M} samples; resolutions {res.tolist()}")
    for levels in [list(range(16)), [0, 1, 2, 3], [4, 5, 6, 7], [8, 9, 10, 11], [12, 13, 14, 15], [0], [1], [2], [15]]:
        g = grid_of(levels)
        tb = table[: len(levels) * T]
        enc = G.hash_encode(g, tb, xd, aabb, 1e-6)
        d = torch.randn_like(enc)
        dt = torch.zeros_like(tb)
        f_ms = timeit(lambda: G.hash_encode(g, tb, xd, aabb, 1e-6))
        b_ms = timeit(lambda: G.hash_encode_bwd(g, xd, d, 0, aabb, 1e-6, d_table=dt))
        print(f"levels {levels}: fwd {f_ms:.3f} ms  bwd {b_ms:.3f} ms")


if __name__ == "__main__":
    main()
