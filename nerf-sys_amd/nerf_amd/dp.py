"""Data-parallel scheme of the train step: rays shard across ranks, weights replicate,
and the only exchange is one SUM all-reduce of the flat [grads | loss] buffer per step.

The reference's own sharding idiom is rank-strided (`an/scripts/create_clusters.py:799`,
`np.arange(rank, len, world)`); for random training batches the equivalent is a disjoint counter-RNG
stream per (step, rank)."""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_seed(step: int, rank: int, world: int) -> int:
    """Disjoint per-rank RNG stream for the ray draw of a step (rank-strided like create_clusters.py:799)."""
    return step * world + rank


def inv_count(n_local: int, world: int) -> float:
    """MSE normaliser 1/(3 N_global): the SUM all-reduce of per-rank gradients is the global mean."""
    return 1.0 / (3.0 * n_local * world)


def allreduce_flat(buf: torch.Tensor, world: int, async_op: bool = False):
    """SUM all-reduce of the flat buffer in place.  async_op=True returns the work handle (the caller waits on the
    stream that consumes the result), else the buffer after a blocking call."""
    if world <= 1:
        return None if async_op else buf
    work = dist.all_reduce(buf, op=dist.ReduceOp.SUM, async_op=async_op)
    return work if async_op else buf


def params_checksum(params, world):
    """After the timed region: every rank's flat parameter buffer reduced to (fp64 sum, position-weighted int64 hash of
    the fp32 bit patterns) and all-gathered — data parallel with one gradient all-reduce keeps the replicas bitwise
    equal, so an N-GPU run validates itself from its own line (params_equal_across_ranks)."""
    bits = params.detach().contiguous().view(torch.int32).to(torch.int64)
    wpos = torch.arange(bits.numel(), device=bits.device, dtype=torch.int64) % 1048573 + 1
    h = (bits * wpos).sum().view(1)                      # int64, wraps on overflow identically on every rank
    f = params.detach().double().sum().view(1)
    hs, fs = [torch.zeros_like(h) for _ in range(world)], [torch.zeros_like(f) for _ in range(world)]
    dist.all_gather(hs, h)
    dist.all_gather(fs, f)
    rows = [(float(x.item()), int(y.item())) for x, y in zip(fs, hs)]
    return {"params_equal_across_ranks": all(r == rows[0] for r in rows), "world_size_checked": dist.get_world_size(),
            "params_sum_per_rank": [r[0] for r in rows], "params_bit_hash_per_rank": [r[1] for r in rows]}
