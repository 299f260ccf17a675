"""Experiment (profiling only): time of Environment.reset() for all envs (mdl_reset)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "marl-delivery_amd"))
import marl_gpu  # noqa: E402
from marl_gpu.maps import grid_array, load_map, map_path  # noqa: E402

out = {}
for E in (1024, 4096):
    env = marl_gpu.BatchedEnv(grid_array(load_map(map_path("map1.txt"))), E, 5, 50, 500, seed=42, tracker="mappo")
    env.reset()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        env.reset()
    e.record()
    torch.cuda.synchronize()
    out[f"reset_E{E}_us"] = round(s.elapsed_time(e) / 20 * 1e3, 1)
    env.close()
print(json.dumps(out))
