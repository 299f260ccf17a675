"""Round 4 probe (profiling only): host cost of one hipGraphLaunch of G config-2 steps against the
GPU time of the same G steps, for G = 20 / 100, the engine's step graph and a graph of G tiny torch
kernels; eager ctypes launches per step.  Prints one JSON line per case."""
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
x = torch.zeros(1, device=dev)


def step(k):
    env.step(acts[k % 100], auto_reset=True, out=(r, sh, dn))


def tiny(k):
    x.add_(1.0)


def capture(fn, G):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        fn(0)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            for k in range(G):
                fn(k)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    return g


def measure(name, g, G, reps=40):
    host, total, gpu = [], [], []
    for _ in range(reps):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        t0 = time.perf_counter()
        g.replay()
        t1 = time.perf_counter()
        e1.record()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        host.append((t1 - t0) * 1e6)
        total.append((t2 - t0) * 1e6)
        gpu.append(e0.elapsed_time(e1) * 1e3)
    med = lambda v: float(np.median(v[5:]))
    print(json.dumps({"case": name, "G": G, "host_launch_us": round(med(host), 2), "wall_us": round(med(total), 2),
                      "event_us": round(med(gpu), 2), "per_node_event_us": round(med(gpu) / G, 3),
                      "per_node_host_us": round(med(host) / G, 3)}), flush=True)


for G in (20, 100):
    measure("step_graph", capture(step, G), G)
    measure("tiny_graph", capture(tiny, G), G)
# eager: host cost per ctypes launch
torch.cuda.synchronize()
t0 = time.perf_counter()
for k in range(200):
    step(k)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(json.dumps({"case": "eager_step", "host_per_launch_us": round((t1 - t0) / 200 * 1e6, 2),
                  "wall_per_step_us": round((t2 - t0) / 200 * 1e6, 2)}), flush=True)
