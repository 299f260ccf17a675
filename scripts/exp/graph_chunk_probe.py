"""Round 4 probe (profiling only): bench.py's timed region (K config-2 steps, synchronize on both
sides, wall clock and HIP events) with the K steps replayed as K/G graphs of G steps each, for
several G: a graph's first kernel starts only after the host has written all G packets
(~0.8 us per node), so small graphs pipeline the submission with the GPU's execution."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "marl-delivery_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import marl_gpu  # noqa: E402
from marl_gpu.maps import grid_array, load_map, map_path  # noqa: E402

dev = torch.device("cuda", 0)
E, A, P, T = 4096, 5, 50, 500
env = marl_gpu.BatchedEnv(grid_array(load_map(map_path("map1.txt"))), E, A, P, T, seeds=[42 + i for i in range(E)],
                          tracker="mappo", shaping="mappo", max_packages_obs=5)
env.reset()
gen = torch.Generator(device=dev).manual_seed(0)
acts = torch.randint(0, 15, (100, E, A), generator=gen, device=dev, dtype=torch.int32).to(torch.uint8)
r = torch.zeros(E, dtype=torch.float64, device=dev)
sh = torch.zeros(E, dtype=torch.float32, device=dev)
dn = torch.zeros(E, dtype=torch.uint8, device=dev)


def step(k):
    env.step(acts[k % 100], auto_reset=True, out=(r, sh, dn))


def capture(G, base):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        step(0)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            for k in range(G):
                step(base + k)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    return g


def timed(graphs, reps):
    walls, evs = [], []
    for _ in range(reps):
        for g in graphs[:2]:   # a few warm steps before each timed region
            g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        t0 = time.perf_counter()
        for g in graphs:
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t0)
        evs.append(e0.elapsed_time(e1) / 1e3)
    return float(np.median(walls)), float(np.median(evs))


for K in (20, 100, 2000):
    for G in (1, 2, 4, 5, 10, 20, 100):
        if G > K or K % G:
            continue
        nb = min(K // G, 100 // G if G < 100 else 1)   # distinct graphs (action slices), reused cyclically
        gs = [capture(G, i * G) for i in range(nb)]
        seq = [gs[i % nb] for i in range(K // G)]
        reps = 15 if K <= 100 else 5
        w, e = timed(seq, reps)
        print(json.dumps({"K": K, "G": G, "wall_us_per_step": round(w / K * 1e6, 3),
                          "event_us_per_step": round(e / K * 1e6, 3),
                          "agent_steps_per_s": round(E * A * K / w / 1e9, 4)}), flush=True)
