"""Experiment (profiling only): where the wall time of bench.py's timed region goes at the driver's
20 steps -- the host cost of each call in it (event records, graph replay, the closing
synchronise) measured call by call, against the same region without the event records."""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "marl-delivery_amd"))
import marl_gpu  # noqa: E402
from marl_gpu.maps import grid_array, load_map, map_path  # noqa: E402

E, A, P, K = 4096, 5, 50, 20
dev = torch.device("cuda", 0)
env = marl_gpu.BatchedEnv(grid_array(load_map(map_path("map1.txt"))), E, A, P, 500, seeds=[42 + i for i in range(E)],
                          tracker="mappo", shaping="mappo", device=dev)
env.reset()
acts = torch.randint(0, 15, (K, E, A), device=dev, dtype=torch.int32).to(torch.uint8)
r = torch.zeros(E, dtype=torch.float64, device=dev)
sh = torch.zeros(E, dtype=torch.float32, device=dev)
dn = torch.zeros(E, dtype=torch.uint8, device=dev)
s = torch.cuda.Stream(device=dev)
g = torch.cuda.CUDAGraph()
with torch.cuda.stream(s):
    env.step(acts[0], out=(r, sh, dn))
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        for k in range(K):
            env.step(acts[k], out=(r, sh, dn))
torch.cuda.synchronize()
g.replay()
torch.cuda.synchronize()

rows = {k: [] for k in ("ev0", "replay", "ev1", "sync", "total_with_events", "total_no_events")}
for it in range(60):
    for k in range(5):
        env.step(acts[k], out=(r, sh, dn))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    t1 = time.perf_counter()
    g.replay()
    t2 = time.perf_counter()
    e1.record()
    t3 = time.perf_counter()
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    for k, v in (("ev0", t1 - t0), ("replay", t2 - t1), ("ev1", t3 - t2), ("sync", t4 - t3), ("total_with_events", t4 - t0)):
        rows[k].append(v * 1e6)
    for k in range(5):
        env.step(acts[k], out=(r, sh, dn))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    rows["total_no_events"].append((time.perf_counter() - t0) * 1e6)
for k, v in rows.items():
    print(f"{k:20s} median {statistics.median(v[10:]):8.1f} us")
print(f"per step: with events {statistics.median(rows['total_with_events'][10:]) / K:.2f} us, "
      f"without {statistics.median(rows['total_no_events'][10:]) / K:.2f} us")
