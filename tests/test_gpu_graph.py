"""The production container train step replayed as ONE captured hipGraph (nerf_amd/graph_step.py,
tools/bench_container.py --graph) against the same step launched eagerly.

A replay runs the eager step's kernels with the seeds, the Adam step count and the visibility thresholds read from
HBM, so from one snapshot of the trainer state a replay and an eager step must give the same loss and parameters.
They are not bitwise equal: the hash-table backward scatters with float atomics, whose order differs run to run
(tests/test_gpu_moe.py, the same caveat).  Tolerances: loss 1e-5 relative, parameters 1e-5 absolute (Adam steps of
lr 1e-2 .. 1e-3 scale the ~1e-7 relative gradient differences of one step)."""
import os
import sys
from types import SimpleNamespace

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def built():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_container
    a = SimpleNamespace(steps=4, warmup=12, batch=1024, train_views=4, cpu_seconds=0.0, no_cpu_baseline=True,
                        shard=False, no_bucket=True, graph=True, host_sized=False)
    one, model = bench_container.build_step(a, torch.device(DEV))
    return one, model


def _state(one, model):
    torch.cuda.synchronize()                     # the steps run on the graph's own stream
    opt = one.opt
    return [t.detach().clone() for t in (opt.flat, opt.m, opt.v, opt.grad, opt.step_dev)]


def _restore(one, saved):
    opt = one.opt
    with torch.no_grad():
        for t, s in zip((opt.flat, opt.m, opt.v, opt.grad, opt.step_dev), saved):
            t.copy_(s)
    torch.cuda.synchronize()


def test_graph_replay_equals_eager_step(built):
    one, model = built
    losses = []
    for s in range(14):                          # eager steps, then the GraphedStep's warm-up, capture and replays
        losses.append(float(one(s).item()))
    gs = one.graphed
    assert gs.graph is not None, "the step was not captured"
    assert all(l == l and l < 1.0 for l in losses), losses
    assert losses[-1] != losses[-2]              # every replay draws its own batch (the seed counter advanced)
    step = 17                                    # no occupancy update at this step (every 16)
    saved = _state(one, model)
    lg = float(one.on_S(lambda: gs(step)).item())
    torch.cuda.synchronize()
    pg = one.opt.flat.detach().clone()
    sg = int(one.opt.step_dev.item())
    _restore(one, saved)
    le = float(one.eager(step).item())
    torch.cuda.synchronize()
    pe = one.opt.flat.detach().clone()
    assert sg == int(one.opt.step_dev.item()) == int(saved[4].item()) + 1
    assert abs(lg - le) <= 1e-5 * abs(le), (lg, le)
    err = (pg - pe).abs().max().item()
    assert err <= 1e-5, err
    assert (pg - saved[0]).abs().max().item() > 0    # the replay did update the parameters
    mx, over = model.__dict__["_dev_sizes"].frozen_report()
    assert mx > 0 and not over, (mx, model.__dict__["_dev_sizes"].cap)


def test_graph_replay_after_occupancy_update(built):
    """An occupancy update (eager, between replays, every 16 steps) rewrites the grids and the visibility thresholds
    in place; the replay that follows must read them: from the same state (parameters, updated grids, thresholds,
    seed counter) the replay and the eager step agree as in the test above."""
    from nerf_amd.container import vis_thresholds
    one, model = built
    gs = one.graphed
    assert gs.graph is not None
    step = 32                                    # an update step (32 % 16 == 0)
    saved = _state(one, model)
    occ = [sub.occ_grid.occs.clone() for sub in model.submodules]
    thr_buf = model.__dict__["_vis_thr_state"]["buf"]
    lg = float(one.on_S(lambda: gs(step)).item())   # pre_fn: the update + in-place threshold refresh, then the replay
    torch.cuda.synchronize()
    pg = one.opt.flat.detach().clone()
    assert any(not torch.equal(a, sub.occ_grid.occs) for a, sub in zip(occ, model.submodules)), "no update ran"
    assert model.__dict__["_vis_thr_state"]["buf"] is thr_buf          # the captured address is still the one used
    _restore(one, saved)                         # parameters back; the grids stay as the update left them
    def eager_body():
        vis_thresholds(model)
        one.ctr.fill_(step)
        return one.body()

    le = float(one.on_S(eager_body).item())
    torch.cuda.synchronize()
    pe = one.opt.flat.detach().clone()
    assert abs(lg - le) <= 1e-5 * abs(le), (lg, le)
    err = (pg - pe).abs().max().item()
    assert err <= 1e-5, err
