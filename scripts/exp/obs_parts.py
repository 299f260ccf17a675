"""Time mdl_build_obs on config 3 per output subset (profiling only)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "marl-delivery_amd"))
import marl_gpu  # noqa: E402
from marl_gpu.maps import grid_array, load_map, map_path  # noqa: E402

E, A, P, T = 16384, 5, 50, 500
MO, MP = (int(x) for x in os.environ.get("OBS_MO_MP", "4,5").split(","))   # config 3b: 100,100
env = marl_gpu.BatchedEnv(grid_array(load_map(map_path("map1.txt"))), E, A, P, T, seed=42, tracker="mappo",
                          max_other_robots=MO, max_packages_obs=MP)
env.reset()
g = torch.Generator(device="cuda").manual_seed(0)
for k in range(60):
    env.step(torch.randint(0, 15, (E, A), dtype=torch.uint8, device="cuda", generator=g))
bufs = env.obs_buffers()
res = {}
ALL = [("actor_map",), ("actor_vec",), ("critic_map",), ("critic_vec",), ("actor_map", "actor_vec", "critic_map", "critic_vec")]
sel = os.environ.get("OBS_WHICH")   # one subset only (PMC passes): "all" or an output name
todo = ALL if not sel else [ALL[-1]] if sel == "all" else [(sel,)]
for which in todo:
    for _ in range(3):
        env.build_obs(out=bufs, which=which)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        env.build_obs(out=bufs, which=which)
    e.record()
    torch.cuda.synchronize()
    res["+".join(which)] = round(s.elapsed_time(e) / 20 * 1e3, 1)
print(json.dumps(res))
