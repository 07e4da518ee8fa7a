"""Per-kernel cost of a graph-replayed chain of trivial kernels on this part: N one-element torch
kernels captured into one hipGraph and replayed; (replay time) / N is the floor that every decode
launch pays (dispatch, completion, the next dispatch) before any memory traffic.  Usage:
python scripts/launch_gap_probe.py"""
import time

import torch

x = torch.zeros(1, device="cuda")
for n in (64, 256, 1024):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            x.add_(1)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            x.add_(1)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    print(f"graph of {n} trivial kernels: {dt * 1e6 / n:.2f} us per kernel", flush=True)
