"""Experiment (profiling only): the driver's short timed region (20 graph-replayed steps
after 5 eager warmup steps) with torch's CUDAGraph.replay() against a direct
hipGraphLaunch of the same instantiated graph (graph.raw_cuda_graph_exec()), which skips
torch's per-replay prologue (generator seed/offset updates).  Interleaved repeats."""
import ctypes as C
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "marl-delivery_amd"))
import marl_gpu  # noqa: E402
from marl_gpu.maps import grid_array, load_map, map_path  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
E, A, G, W = 4096, 5, 20, 5
env = marl_gpu.BatchedEnv(grid_array(load_map(map_path("map1.txt"))), E, A, 50, 500, seed=42, tracker="mappo",
                          shaping="mappo", max_packages_obs=5, device=dev)
env.reset()
gen = torch.Generator(device=dev).manual_seed(0)
acts = torch.randint(0, 15, (G, E, A), generator=gen, device=dev, dtype=torch.int32).to(torch.uint8)
r = torch.zeros(E, dtype=torch.float64, device=dev)
sh = torch.zeros(E, dtype=torch.float32, device=dev)
dn = torch.zeros(E, dtype=torch.uint8, device=dev)


def one(k):
    env.step(acts[k % G], auto_reset=True, out=(r, sh, dn))


s = torch.cuda.Stream(device=dev)
s.wait_stream(torch.cuda.current_stream())
graph = torch.cuda.CUDAGraph()
with torch.cuda.stream(s):
    one(0)
    torch.cuda.synchronize()
    with torch.cuda.graph(graph, stream=s):
        for k in range(G):
            one(k)
torch.cuda.synchronize()
graph.replay()
torch.cuda.synchronize()

hip = C.CDLL("libamdhip64.so")
hip.hipGraphLaunch.argtypes = [C.c_void_p, C.c_void_p]
hip.hipGraphLaunch.restype = C.c_int
gexec = C.c_void_p(graph.raw_cuda_graph_exec())


def raw_replay():
    rc = hip.hipGraphLaunch(gexec, C.c_void_p(torch.cuda.current_stream().cuda_stream))
    if rc != 0:
        raise RuntimeError("hipGraphLaunch %d" % rc)


def leg(replay):
    time.sleep(0.02)   # idle pause, as between the driver's phases
    for k in range(W):
        one(k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    replay()
    e1.record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    return {"wall_us": wall / G * 1e6, "event_us": e0.elapsed_time(e1) / G * 1e3}


out = {"torch_replay": [], "raw_launch": []}
for rep in range(8):
    out["torch_replay"].append(leg(graph.replay))
    out["raw_launch"].append(leg(raw_replay))
# the raw launch must run the same steps: compare one more step of each path from one state
med = {k: {m: sorted(x[m] for x in v)[len(v) // 2] for m in ("wall_us", "event_us")} for k, v in out.items()}
print(json.dumps({"median": med, "runs": out}, indent=1))
