"""Experiment (profiling only): where a SHORT timed region (the driver runs
bench.py --steps 20 --warmup 5) loses time against the long-run per-step figure.

Legs, each timed K=20 steps of mdl_step over 4096 map1 envs, event + wall clock:
  graph_cold   one replay of a 20-step graph after an idle pause
  graph_hot    the same right after 2000 graph-replayed steps
  eager_py     BatchedEnv.step x20
  eager_lean   the ctypes entry called directly with prebuilt arguments x20
  graph_long   per-step figure of 20 replays of a 100-step graph
"""
import ctypes as C
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "marl-delivery_amd"))
import marl_gpu  # noqa: E402
from marl_gpu import _lib  # noqa: E402
from marl_gpu.maps import grid_array, load_map, map_path  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
grid = grid_array(load_map(map_path("map1.txt")))
E, A, K = 4096, 5, 20
env = marl_gpu.BatchedEnv(grid, E, A, 50, 500, seed=42, tracker="mappo", shaping="mappo", device=dev)
env.reset()
gen = torch.Generator(device=dev).manual_seed(0)
acts = torch.randint(0, 15, (100, E, A), generator=gen, device=dev, dtype=torch.int32).to(torch.uint8)
r = torch.zeros(E, dtype=torch.float64, device=dev)
sh = torch.zeros(E, dtype=torch.float32, device=dev)
dn = torch.zeros(E, dtype=torch.uint8, device=dev)


def one(k):
    env.step(acts[k % 100], auto_reset=True, out=(r, sh, dn))


for k in range(5):
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


g20, g100 = capture(20), capture(100)


def timed(fn, steps):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    return {"wall_us": wall / steps * 1e6, "event_us": e0.elapsed_time(e1) / steps * 1e3}


L = _lib.lib()
stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
h = env._h
aptr = [C.c_void_p(acts[k].data_ptr()) for k in range(100)]
rp, shp, dp = C.c_void_p(r.data_ptr()), C.c_void_p(sh.data_ptr()), C.c_void_p(dn.data_ptr())
fn_step = L.mdl_step


def lean():
    for k in range(K):
        fn_step(h, aptr[k], 0, None, E, 1, rp, shp, dp, stream)


def eager():
    for k in range(K):
        one(k)


out = {}
for trial in range(5):
    time.sleep(0.3)
    out.setdefault("graph_cold", []).append(timed(g20.replay, K))
for trial in range(5):
    time.sleep(0.3)
    out.setdefault("eager_py_cold", []).append(timed(eager, K))
for trial in range(5):
    time.sleep(0.3)
    out.setdefault("eager_lean_cold", []).append(timed(lean, K))
for trial in range(5):
    for _ in range(20):
        g100.replay()
    out.setdefault("graph_hot", []).append(timed(g20.replay, K))
for trial in range(5):
    for _ in range(20):
        g100.replay()
    out.setdefault("eager_lean_hot", []).append(timed(lean, K))
for trial in range(3):
    out.setdefault("graph_long", []).append(timed(lambda: [g100.replay() for _ in range(20)], 2000))
for trial in range(3):
    out.setdefault("lean_long", []).append(
        timed(lambda: [fn_step(h, aptr[k % 100], 0, None, E, 1, rp, shp, dp, stream) for k in range(2000)], 2000))
# host cost of one call of each kind (no sync inside)
t0 = time.perf_counter()
for k in range(2000):
    fn_step(h, aptr[k % 100], 0, None, E, 1, rp, shp, dp, stream)
host_lean = (time.perf_counter() - t0) / 2000 * 1e6
torch.cuda.synchronize()
t0 = time.perf_counter()
for k in range(2000):
    one(k)
host_py = (time.perf_counter() - t0) / 2000 * 1e6
torch.cuda.synchronize()
out["host_call_us"] = {"lean": host_lean, "py": host_py}
for k, v in out.items():
    if isinstance(v, list):
        print(k, " ".join("%.2f/%.2f" % (x["event_us"], x["wall_us"]) for x in v))
    else:
        print(k, v)
os.makedirs("gpurun_out", exist_ok=True)
json.dump(out, open("gpurun_out/short_k.json", "w"), indent=1)
env.close()
