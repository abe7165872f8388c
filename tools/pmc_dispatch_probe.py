#!/usr/bin/env python3
"""How many kernel dispatches a rocprofv3 --pmc pass survives on this image, with NO code of this repository loaded:
N launches of one tiny torch elementwise kernel, a progress line (flushed) every --every dispatches.  Round 5 used it
to separate the C5-leg SIGSEGV from this library's kernels ("rocprofv3 PMC").

  timeout -s KILL 600 rocprofv3 --pmc SQ_WAVE_CYCLES ... --kernel-trace -- python3 tools/pmc_dispatch_probe.py"""
import argparse
import faulthandler
import sys
import time

import torch

faulthandler.enable(all_threads=True)
ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=200000)
ap.add_argument("--every", type=int, default=2000)
ap.add_argument("--streams", type=int, default=1, help="alternate the launches over this many HIP streams")
a = ap.parse_args()
xs = [torch.zeros(1024, device="cuda") for _ in range(a.streams)]
ss = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(a.streams - 1)]
t0 = time.perf_counter()
for i in range(1, a.n + 1):
    with torch.cuda.stream(ss[i % a.streams]):
        xs[i % a.streams].add_(1.0)
    if i % a.every == 0:
        torch.cuda.synchronize()
        print(f"[probe {time.perf_counter() - t0:7.1f}s] {i} dispatches", flush=True)
torch.cuda.synchronize()
print(f"probe done: {a.n} dispatches over {a.streams} stream(s), sum = {sum(x[0].item() for x in xs)}", flush=True)
