"""Per-step wall times of the container train step (tools/bench_container.py's step): shows the cost of the
occupancy-grid update steps (every 16 steps) next to the ordinary ones."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "nerf-sys_amd"), ROOT, os.path.dirname(os.path.abspath(__file__))]
import torch  # noqa: E402
import bench_container as BC  # noqa: E402


def main():
    sys.argv = sys.argv[:1]
    a = BC.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    one, model = BC.build_step(a, dev)
    for s in range(a.warmup):
        one(s)
    torch.cuda.synchronize()
    ts = []
    for s in range(a.warmup, a.warmup + 48):
        t0 = time.perf_counter()
        one(s)
        torch.cuda.synchronize()
        ts.append((s, (time.perf_counter() - t0) * 1e3))
    srt = sorted(t for _, t in ts)
    print("median ms", round(srt[len(srt) // 2], 3), "mean", round(sum(srt) / len(srt), 3))
    print("slowest", [(s, round(t, 2)) for s, t in sorted(ts, key=lambda x: -x[1])[:5]])


if __name__ == "__main__":
    main()
