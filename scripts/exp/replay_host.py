"""Experiment (profiling only): host cost of torch's CUDAGraph.replay() for step graphs
of 20 and 100 nodes, and the GPU time of a 20-node replay when its packets are all
queued before the GPU reaches them (stream held by a preceding ~1 ms torch kernel)
versus submitted to an idle GPU (the bench's timed-region situation)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "marl-delivery_amd"))
import marl_gpu  # noqa: E402
from marl_gpu.maps import grid_array, load_map, map_path  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
E, A = 4096, 5
env = marl_gpu.BatchedEnv(grid_array(load_map(map_path("map1.txt"))), E, A, 50, 500, seed=42, tracker="mappo",
                          device=dev)
env.reset()
acts = torch.randint(0, 15, (100, E, A), device=dev, dtype=torch.uint8)
r = torch.zeros(E, dtype=torch.float64, device=dev)
sh = torch.zeros(E, dtype=torch.float32, device=dev)
dn = torch.zeros(E, dtype=torch.uint8, device=dev)


def one(k):
    env.step(acts[k % 100], out=(r, sh, dn))


for k in range(10):
    one(k)
torch.cuda.synchronize()


def capture(G):
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        one(0)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            for k in range(G):
                one(k)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    return g


graphs = {G: capture(G) for G in (20, 100)}
big = torch.randn(8192, 8192, device=dev)
for G, g in graphs.items():
    hs = []
    for _ in range(20):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        hs.append((time.perf_counter() - t0) * 1e6)
        torch.cuda.synchronize()
    hs.sort()
    print(f"G={G}: replay() host us median {hs[len(hs) // 2]:.1f} min {hs[0]:.1f} ({hs[len(hs) // 2] / G:.2f} per node)")
g = graphs[20]
for mode in ("idle", "queued"):
    res = []
    for _ in range(10):
        torch.cuda.synchronize()
        if mode == "queued":
            big @ big   # ~ms of work ahead of the graph on the same stream
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) * 1e3 / 20)
    res.sort()
    print(f"20-node replay, {mode}: event us/step median {res[5]:.2f} min {res[0]:.2f}")
env.close()
