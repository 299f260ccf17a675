"""Experiment (profiling only): host cost per BatchedEnv.step call (no sync inside the
loop) vs the bare ctypes entry, and the pieces of the Python path."""
import ctypes as C
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "marl-delivery_amd"))
import marl_gpu  # noqa: E402
from marl_gpu import _lib  # noqa: E402
from marl_gpu.maps import grid_array, load_map, map_path  # noqa: E402

dev = torch.device("cuda", 0)
E, A = 4096, 5
env = marl_gpu.BatchedEnv(grid_array(load_map(map_path("map1.txt"))), E, A, 50, 500, seed=42, device=dev)
env.reset()
acts = torch.randint(0, 15, (100, E, A), device=dev, dtype=torch.uint8)
views = [acts[k] for k in range(100)]
r = torch.zeros(E, dtype=torch.float64, device=dev)
sh = torch.zeros(E, dtype=torch.float32, device=dev)
dn = torch.zeros(E, dtype=torch.uint8, device=dev)
out = (r, sh, dn)


def bench(name, fn, n=3000):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(n):
        fn(k)
    host = (time.perf_counter() - t0) / n * 1e6
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / n * 1e6
    print(f"{name:32s} host {host:6.2f} us/call, wall {wall:6.2f} us/step")


L = _lib.lib()
h = env._h
st = torch.cuda.current_stream().cuda_stream
ap = [v.data_ptr() for v in views]
bench("ctypes mdl_step", lambda k: L.mdl_step(h, ap[k % 100], 0, None, E, 1, r.data_ptr(), sh.data_ptr(),
                                               dn.data_ptr(), st))
bench("env.step(view, out=...)", lambda k: env.step(views[k % 100], out=out))
bench("env.step(acts[k], out=...)", lambda k: env.step(acts[k % 100], out=out))
bench("env.step(view)", lambda k: env.step(views[k % 100]))
bench("acts[k] slicing only", lambda k: acts[k % 100])
bench("raw_stream only", lambda k: _lib.raw_stream(0))
env.close()
