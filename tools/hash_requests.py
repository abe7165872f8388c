"""64-B atomic requests issued by hash_bwd_f2_agg_kernel for a set of sample positions (the memory-side float
atomic unit's work, MI355X_MICROARCH.md § Global float atomics: ~20 G requests/s chip-wide = 1.3 TB/s of added
bytes / 64 B).  Mirrors the kernel's lane layout (nerf-sys_amd/csrc/ngp.hip hash_bwd_f2_agg_kernel): a wave holds
16 consecutive samples x 4 lanes (x-corner dx = q >> 1, feature f = q & 1); per (level, yz-corner) one atomic
wave-instruction whose active lanes are the run heads (a lane whose sample's table entry differs from the previous
sample's in its sub-sequence); its 64-B requests = the distinct 64-B segments those lanes touch."""
import torch

ATOMIC_REQ_PEAK = 1.3e12 / 64  # requests / s


def ngp_hash(ix, iy, iz, mask):
    return (ix ^ ((iy * 2654435761) & 0xFFFFFFFF) ^ ((iz * 805459861) & 0xFFFFFFFF)) & mask


@torch.no_grad()
def count_requests(x, resolutions, log2T, aabb, eps=1e-6):
    """x: (M, >=3) positions (the kernel's x rows); aabb: 6 floats or None.  Returns the request count."""
    p = x[:, :3].float()
    if aabb is not None:
        a = torch.tensor(list(aabb), dtype=torch.float32, device=p.device)
        p = ((p - a[:3]) / (a[3:] - a[:3])).clamp(eps, 1 - eps)
    M = p.shape[0]
    W = (M + 15) // 16
    pad = W * 16 - M
    mask, T = (1 << log2T) - 1, 1 << log2T
    total = 0
    for l, r in enumerate(resolutions):
        s = p * float(r)
        i0 = torch.floor(s).to(torch.int64)
        base = l * T * 2
        for yz in range(4):
            dy, dz = yz >> 1, yz & 1
            idx = []
            for q in range(4):
                dx, f = q >> 1, q & 1
                h = ngp_hash(i0[:, 0] + dx, i0[:, 1] + dy, i0[:, 2] + dz, mask)
                idx.append(h * 2 + f)
            idx = torch.stack(idx, 1)                      # (M, 4) float index within the level
            if pad:
                idx = torch.cat([idx, torch.full((pad, 4), -1, dtype=idx.dtype, device=idx.device)])
            idx = idx.view(W, 16, 4)
            prev = torch.cat([torch.full_like(idx[:, :1], -2), idx[:, :-1]], 1)
            head = (idx != prev) & (idx >= 0)
            seg = torch.where(head, (base + idx) * 4 // 64, torch.full_like(idx, -1)).view(W, 64)
            seg, _ = seg.sort(1)
            distinct = ((seg[:, 1:] != seg[:, :-1]) & (seg[:, 1:] >= 0)).sum(1) + (seg[:, 0] >= 0).long()
            total += int(distinct.sum())
    return total
