"""cProfile of the container train step's host side (what bounds the step when the GPU idles between
launches).  Usage: python tools/cpu_profile_container.py [steps]"""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "nerf-sys_amd"))
sys.path.insert(0, ROOT)


def main():
    import bench_container as B
    import torch
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    sys.argv = [sys.argv[0], "--steps", str(steps), "--warmup", "40", "--no-cpu-baseline"]
    # run the bench's setup + warmup via its main but profile only a plain loop afterwards
    a = B.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    one, model = B.build_step(a, dev)
    for s in range(a.warmup):
        one(s)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for s in range(a.warmup, a.warmup + steps):
        one(s)
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(35)
    st.sort_stats("cumulative").print_stats(45)
    st.print_callers("_named_members|named_modules|data_ptr")


if __name__ == "__main__":
    main()
