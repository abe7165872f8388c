"""World-size-2 data-parallel check on the CPU (gloo): the trainer's exchange scheme — per-rank MSE
normalised by 1/(3 N_global) and ONE SUM all-reduce of the flat packed [grads | loss] buffer — equals
the single-process full-batch gradient and loss.  The per-rank gradient comes from the CPU oracle (the
HIP kernels need a GPU); the packing, normaliser and all-reduce are the product's own code."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import nerf_oracle as O


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(n=32):
    g = torch.Generator().manual_seed(7)
    o = torch.tensor([0.0, -4.0, 0.5]).expand(n, 3)
    d = torch.nn.functional.normalize(torch.randn(n, 3, generator=g) * 0.15 + torch.tensor([0.0, 1.0, -0.12]), dim=-1)
    rays = torch.cat([o, d, torch.full((n, 1), 2.0), torch.full((n, 1), 6.0)], -1)
    gt = torch.rand(n, 3, generator=g)
    us = torch.rand(n, 16, generator=g)
    return rays, gt, us


def _flat_grad(p, rays, gt, us, inv_count):
    from nerf_amd.vanilla import PackedLayout
    L = PackedLayout.get()
    pg = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    rgb = O.render_rays(pg, rays, 16, training=True, u_strat=us)[0]
    a, b = O.color_space_transformer(rgb, gt, "linear")
    loss = ((a - b) ** 2).sum() * inv_count
    grads = torch.autograd.grad(loss, list(pg.values()))
    flat = L.pack([g.detach() for g in grads]).detach()
    return torch.cat([flat, loss.detach().view(1)])


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "nerf-sys_amd"), os.path.join(root, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from nerf_amd.dp import allreduce_flat, inv_count, shard_seed
    torch.set_num_threads(2)
    rays, gt, us = _batch()
    n_local = rays.shape[0] // world
    sl = slice(rank * n_local, (rank + 1) * n_local)
    buf = _flat_grad(O.init_vanilla_params(3), rays[sl], gt[sl], us[sl], inv_count(n_local, world))
    buf_async = buf.clone()
    allreduce_flat(buf, world)
    work = allreduce_flat(buf_async, world, async_op=True)  # the trainer's form: issue, then wait where consumed
    work.wait()
    assert torch.equal(buf, buf_async)
    seeds = [shard_seed(s, rank, world) for s in range(5)]
    if rank == 0:
        q.put((buf.numpy(), seeds))  # numpy: pickled by value (a tensor's shared-memory handle dies with the worker)
    else:
        q.put((None, seeds))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_allreduce_equals_full_batch():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    dp = torch.from_numpy(next(b for b, _ in res if b is not None))
    seeds = [s for _, s in res]
    assert not set(seeds[0]) & set(seeds[1])  # disjoint per-rank ray streams
    from nerf_amd.dp import inv_count
    rays, gt, us = _batch()
    full = _flat_grad(O.init_vanilla_params(3), rays, gt, us, inv_count(rays.shape[0], 1))
    torch.testing.assert_close(dp, full, rtol=1e-4, atol=1e-7)


def _flat_adam_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "nerf-sys_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from nerf_amd.optim import FlatAdam
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(5, 3)), torch.nn.Parameter(torch.randn(7))]
    opt = FlatAdam([{"params": ps[:1], "lr": 1e-3}, {"params": ps[1:], "lr": 1e-2}], world_size=world)
    with torch.no_grad():
        for i, p in enumerate(ps):
            p.grad.copy_(torch.full_like(p, float(rank + 1) * (i + 1)))
    opt.allreduce_grads()
    q.put((rank, [p.grad.clone().numpy() for p in ps]))
    dist.destroy_process_group()


def test_flat_adam_data_parallel_mean_gloo():
    """FlatAdam's data-parallel exchange (the container / NGP path): one all-reduce of the flat gradient buffer
    and the mean over ranks, landing in every parameter's .grad view."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_flat_adam_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        g0, g1 = (torch.from_numpy(a) for a in out[r])
        assert torch.allclose(g0, torch.full((5, 3), 1.5)) and torch.allclose(g1, torch.full((7,), 3.0))


def _bucket_worker(rank, world, port, q):
    """Three bucketed 'tables' (bucket_min_numel 64) and one small tensor.  Rank 0's backward writes tables 2 and 0
    (in that order), rank 1's only table 1 — as when an expert gets no samples on a rank (container.py skips its
    backward).  The collective sequence must still match: every rank ends with the mean gradient."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "nerf-sys_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from nerf_amd.optim import FlatAdam
    ps = [torch.nn.Parameter(torch.zeros(100)), torch.nn.Parameter(torch.zeros(5)),
          torch.nn.Parameter(torch.zeros(80)), torch.nn.Parameter(torch.zeros(70))]
    tables = [ps[0], ps[2], ps[3]]
    opt = FlatAdam([{"params": ps, "lr": 1e-3}], world_size=world, bucket_min_numel=64)
    for step in range(3):
        opt.zero_grad()
        fired = {0: [2, 0], 1: [1]}[rank] if step != 1 else {0: [], 1: [0, 1, 2]}[rank]
        with torch.no_grad():
            ps[1].grad.fill_(float(rank + 1))
            for t in fired:
                tables[t].grad.fill_(float(10 * (t + 1) * (rank + 1)))
                tables[t]._nerf_grad_ready(tables[t])
        opt.allreduce_grads()
        q.put((rank, step, [p.grad.clone().numpy() for p in ps]))
    dist.destroy_process_group()


def test_flat_adam_buckets_data_dependent_firing_gloo():
    """a bucket's all-reduce used to start from the expert's backward, so ranks whose experts got
    different samples issued different collective sequences (hang or mismatched buffers under RCCL).  Buckets are
    now issued in one fixed order and step() issues the ones that did not fire: any firing pattern gives every rank
    the rank-mean gradient."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bucket_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world * 3):
        r, step, g = q.get(timeout=120)
        got[(r, step)] = [torch.from_numpy(a) for a in g]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for step in range(3):
        fired = {0: [2, 0], 1: [1]} if step != 1 else {0: [], 1: [0, 1, 2]}
        want_t = [sum(10.0 * (t + 1) * (r + 1) for r in range(world) if t in fired[r]) / world for t in range(3)]
        for r in range(world):
            g = got[(r, step)]
            assert torch.allclose(g[1], torch.full((5,), 1.5)), (r, step, g[1])
            for t, i in enumerate((0, 2, 3)):
                assert torch.allclose(g[i], torch.full_like(g[i], want_t[t])), (r, step, t, g[i][:3], want_t[t])


def _checksum_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    p = torch.randn(100003, generator=torch.Generator().manual_seed(5))
    same = bench.params_checksum(p, world)
    if rank == 1:  # one flipped low mantissa bit on one rank: the fp64 sum may not see it, the bit hash does
        p.view(torch.int32)[77777] ^= 1
    diff = bench.params_checksum(p, world)
    q.put((rank, same, diff))
    dist.destroy_process_group()


def test_bench_params_checksum_gloo():
    """bench.py's dp record: after the timed region the ranks all-gather a checksum of their
    parameters, so an N-GPU run reports whether the replicas stayed bitwise equal."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_checksum_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict((r, (a, b)) for r, a, b in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        same, diff = out[r]
        assert same["params_equal_across_ranks"] and same["world_size_checked"] == 2
        assert not diff["params_equal_across_ranks"]
        assert diff["params_bit_hash_per_rank"][0] != diff["params_bit_hash_per_rank"][1]
