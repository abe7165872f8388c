"""The product trainer's data-parallel step at world size 2, on the GPU.

Two processes share cuda:0 and talk over gloo (RCCL refuses two ranks on one device; gloo all-reduces CUDA
tensors through the host).  Each runs ``NeRFTrainer(world_size=2)`` — the HIP step, the 1/(3 N_global) loss
normaliser, ``allreduce_flat`` of the flat [grads | loss] buffer (the real ``dist.all_reduce``), clip and the HIP
Adam — on its rank-strided half of a fixed batch (an/scripts/create_clusters.py:799) with injected jitter.
The result must equal the single-process full-batch step: loss, reduced flat gradient, post-Adam parameters
(both ranks bitwise equal to each other), and the second step's loss."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from oracle import nerf_oracle as O

pytestmark = pytest.mark.gpu
N, S, NI = 256, 64, 128


def _by_value(x):
    """Results cross the queue BY VALUE (numpy): a torch CPU tensor is sent as a shared-memory file descriptor that the
    parent can only fetch while the worker still lives — a worker that exits first makes the parent's get() fail."""
    if torch.is_tensor(x):
        return x.numpy()
    if isinstance(x, dict):
        return {k: _by_value(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_by_value(v) for v in x)
    return x


def _to_torch(x):
    import numpy as np
    if isinstance(x, np.ndarray):
        return torch.from_numpy(x)
    if isinstance(x, dict):
        return {k: _to_torch(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_to_torch(v) for v in x)
    return x


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs():
    g = torch.Generator().manual_seed(17)
    o = torch.tensor([0.0, -4.0311, 0.5]).expand(N, 3)
    d = torch.nn.functional.normalize(torch.randn(N, 3, generator=g) * 0.2 + torch.tensor([0.0, 1.0, -0.12]), dim=-1)
    rays = torch.cat([o, d, torch.full((N, 1), 2.0), torch.full((N, 1), 6.0)], -1)
    gt = torch.rand(N, 3, generator=g)
    us = [torch.rand(N, S, generator=g) for _ in range(2)]
    up = [torch.rand(N, NI, generator=g) for _ in range(2)]
    return rays, gt, us, up


def _run(world, rank, dev):
    from nerf_amd.trainer import NeRFTrainer
    from nerf_amd.vanilla import VanillaNeRF
    rays, gt, us, up = _inputs()
    sl = slice(rank, None, world)
    tr = NeRFTrainer(VanillaNeRF().load_reference_state(O.init_vanilla_params(1)).to(dev),
                     VanillaNeRF().load_reference_state(O.init_vanilla_params(2)).to(dev),
                     n_samples=S, n_importance=NI, world_size=world, device=dev)
    out = {"loss": [], "grad": [], "params": []}
    for step in range(2):
        loss = tr.step(rays[sl].contiguous().to(dev), gt[sl].contiguous().to(dev), seed=step,
                       u_strat=us[step][sl].contiguous().to(dev), u_pdf=up[step][sl].contiguous().to(dev))
        torch.cuda.synchronize()
        out["loss"].append(float(loss.item()))
        out["grad"].append(tr.grads.detach().cpu().clone())
        out["params"].append(tr.params.detach().cpu().clone())
    return out


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "nerf-sys_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        q.put((rank, _by_value(_run(world, rank, dev))))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent on q.get
        q.put((rank, repr(e)))
        raise


def test_trainer_world2_equals_full_batch():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: _to_torch(v) for r, v in (q.get(timeout=100) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert isinstance(res[r], dict), f"rank {r} failed: {res[r]}"
        assert procs[r].exitcode == 0
    full = _run(1, 0, torch.device("cuda", 0))
    r0, r1 = res[0], res[1]
    for step in range(2):
        # every rank holds the same reduced buffer and applies the same update
        assert torch.equal(r0["grad"][step], r1["grad"][step]), f"step {step}: ranks disagree on the reduced gradient"
        assert torch.equal(r0["params"][step], r1["params"][step]), f"step {step}: ranks diverged"
        assert r0["loss"][step] == r1["loss"][step]
        lf = full["loss"][step]
        assert abs(r0["loss"][step] - lf) <= 1e-6 * max(1.0, lf), (step, r0["loss"][step], lf)
    # step 0: reduced flat gradient (same start point) within rounding of the full-batch one
    g, gf = r0["grad"][0].double(), full["grad"][0].double()
    P = g.numel() // 2
    for k in range(2):
        a, b = g[k * P:(k + 1) * P], gf[k * P:(k + 1) * P]
        err = (a - b).abs().max().item()
        assert err <= 1e-5 * b.abs().max().item(), f"net {k}: grad max err {err:.3e} vs scale {b.abs().max():.3e}"
    # post-Adam parameters of step 0: the update difference the two measured gradients imply (Adam's first step is
    # lr * g/(|g|+eps): rounding-level gradient differences at the 1e-8 noise floor can move an element by <= 2 lr)
    norm = gf.norm().item()
    coef = min(1.0, 1.0 / (norm + 1e-6))
    phi = lambda x: x * coef / ((x * coef).abs() + 1e-8)
    bound = 2e-3 * (phi(g) - phi(gf)).abs() * 1.02 + 2e-9 + 2.5e-7 * (1 + full["params"][0].double().abs())
    perr = (r0["params"][0].double() - full["params"][0].double()).abs()
    assert (perr <= bound).all(), f"post-Adam: {int((perr > bound).sum())} elements beyond the implied bound"


def _adam_run(world, rank, mode):
    """Three FlatAdam steps on rank-dependent gradients (the clip binds): parameters after each step.  mode: "shard"
    (reduce-scatter + all-gather), "replicated" (one all-reduce) or "bucketed" (a 1 M-float parameter whose gradient
    is written in place and announced as complete, as the Instant-NGP table backward does, starting its all-reduce
    before step(); the other ranges are all-reduced in step())."""
    from nerf_amd.optim import FlatAdam
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    big = mode == "bucketed"
    shapes = [(37, 11), (1000,), (5, 3)] + ([((1 << 20) + 37,)] if big else []) + [(7,)]
    ps = [torch.nn.Parameter(torch.randn(sh, device=dev)) for sh in shapes]
    opt = FlatAdam([{"params": ps[:1], "lr": 1e-2}, {"params": ps[1:], "lr": 3e-3}], world_size=world,
                   shard=(mode == "shard"), bucket_tables=big)
    out = []
    g = torch.Generator().manual_seed(123)
    gr = [[torch.randn(p.shape, generator=g) for p in ps] for _ in range(3 * max(world, 2))]
    for step in range(3):
        opt.zero_grad()
        with torch.no_grad():
            for i, p in enumerate(ps):
                if world == 1:  # the full batch: the mean of the two ranks' gradients
                    p.grad.copy_(((gr[2 * step][i] + gr[2 * step + 1][i]) * 0.5).to(dev))
                else:
                    p.grad.copy_(gr[2 * step + rank][i].to(dev))
                if big and world > 1 and p.numel() >= (1 << 20):
                    assert getattr(p, "_nerf_grad_ready", None) is not None
                    p._nerf_grad_ready(p)  # its all-reduce starts here, before step()
                    assert len(opt._inflight) == 1
        opt.step()
        torch.cuda.synchronize()
        out.append(torch.cat([p.detach().reshape(-1).cpu() for p in ps]))
    return out


def _adam_worker(rank, world, port, q, mode):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "nerf-sys_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        q.put((rank, _by_value(_adam_run(world, rank, mode))))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, repr(e)))
        raise


@pytest.mark.parametrize("mode", ["shard", "replicated", "bucketed"])
def test_flat_adam_world2(mode):
    """FlatAdam at world 2 — sharded (reduce-scatter, clip + Adam on a 1/N slice, all-gather), replicated (one
    all-reduce) and bucketed (the in-place table bucket's all-reduce started before step()) — against the
    single-process step on the mean gradient; both ranks bitwise equal."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_adam_worker, args=(r, world, port, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: _to_torch(v) for r, v in (q.get(timeout=100) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert isinstance(res[r], list), f"rank {r} failed: {res[r]}"
    full = _adam_run(1, 0, mode)
    for step in range(3):
        assert torch.equal(res[0][step], res[1][step]), f"step {step}: ranks diverged"
        # the rank mean (a + b) / 2 vs the full batch's (a + b) * 0.5 is exact; the clip norm's partial sums are
        # grouped differently under sharding: rounding-level differences only
        torch.testing.assert_close(res[0][step], full[step], rtol=2e-6, atol=2e-7)


def test_bench_engine_run_world2_gloo():
    """bench.py's own data-parallel path (engine_run at --gpus 2, two ranks sharing cuda:0 over gloo): the line's dp
    record says the replicas stayed bitwise equal (an all-gathered fp64 sum + bit hash of every rank's parameters),
    both all-reduce buckets were bracketed by events on their consuming streams, and the exposed-exchange leg ran."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_PORT=str(_free_port()), HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dist-backend", "gloo", "--steps", "3",
           "--warmup", "1", "--train-views", "4", "--no-psnr", "--no-cpu-baseline", "--no-llff", "--no-sweep",
           "--no-dropin", "--no-other-precision", "--no-native-ref"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    out = json.loads(line)
    dp = out["dp"]
    print(json.dumps({k: dp[k] for k in dp if "note" not in k}))
    assert out["n_gpus"] == 2 and dp["world_size"] == 2 and dp["world_size_checked"] == 2
    assert dp["params_equal_across_ranks"] is True
    assert len(set(dp["params_bit_hash_per_rank"])) == 1
    for rank_times in dp["allreduce_ms_per_rank"]:
        assert len(rank_times) == 2 and all(t > 0.0 for t in rank_times), dp["allreduce_ms_per_rank"]
    assert "exposed_exchange_ms" in dp and dp["step_ms_no_exchange"] > 0


def test_bench_world2_line_complete_gloo():
    """The N > 1 bench line carries what the N = 1 line does: rank 0's CPU baseline (the other
    rank waiting in the final barrier), the PSNR leg trained data parallel on both ranks and rendered by rank 0 with
    the replicas checked equal, and the production container on FlatAdam(world_size=2) with a `dp` block whose
    all-gathered parameter checksum says the replicas stayed bitwise equal.  Two ranks share cuda:0 over gloo."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_PORT=str(_free_port()), HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dist-backend", "gloo", "--steps", "2",
           "--warmup", "1", "--timing-steps", "1", "--train-views", "4", "--psnr-steps", "8", "--psnr-views", "1",
           "--cpu-batch", "32", "--cpu-steps", "1", "--no-llff", "--no-sweep", "--no-dropin", "--no-other-precision",
           "--no-native-ref", "--container-steps", "3", "--container-warmup", "4", "--prod-cpu-seconds", "1"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    print(json.dumps({k: out[k] for k in ("value", "psnr", "cpu_baseline")}))
    assert out["n_gpus"] == 2 and out["dp"]["params_equal_across_ranks"] is True
    cb = out["cpu_baseline"]
    assert cb and cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] == "port"
    ps = out["psnr"]
    assert ps["n_gpus"] == 2 and ps["params_equal_across_ranks"] == {"fp32": True}
    assert ps["fp32"]["steps"] == 8 and ps["fp32"]["psnr"] > 0
    c = out["container"]
    assert c["n_gpus"] == 2 and c["value"] > 0
    assert c["dp"]["world_size"] == 2 and c["dp"]["flat_adam"]["world_size"] == 2
    assert c["dp"]["params_equal_across_ranks"] is True and len(set(c["dp"]["params_bit_hash_per_rank"])) == 1
    assert c["exchange"]["bucketed"] is True
