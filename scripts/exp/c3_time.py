"""Config 3 / 3b timing for builder A/Bs (profiling only): mdl_build_obs and mdl_step_obs over
16384 map1 envs, each as a hipGraph of G calls replayed R times; per-replay HIP-event times,
median and min per call (us).  OBS_MO_MP=4,5 (config 3, default) or 100,100 (3b)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "marl-delivery_amd"))
import marl_gpu  # noqa: E402
from marl_gpu.maps import grid_array, load_map, map_path  # noqa: E402

E, A, P, T = int(os.environ.get("C3_ENVS", "16384")), 5, 50, 500
MO, MP = (int(x) for x in os.environ.get("OBS_MO_MP", "4,5").split(","))
G, R = int(os.environ.get("C3_G", "20")), int(os.environ.get("C3_R", "15"))
env = marl_gpu.BatchedEnv(grid_array(load_map(map_path("map1.txt"))), E, A, P, T, seed=42, tracker="mappo",
                          max_other_robots=MO, max_packages_obs=MP)
env.reset()
gen = torch.Generator(device="cuda").manual_seed(0)
acts = torch.randint(0, 15, (G, E, A), generator=gen, device="cuda", dtype=torch.int32).to(torch.uint8)
for k in range(60):
    env.step(acts[k % G])
bufs = env.obs_buffers()
r = torch.zeros(E, dtype=torch.float64, device="cuda")
sh = torch.zeros(E, dtype=torch.float32, device="cuda")
dn = torch.zeros(E, dtype=torch.uint8, device="cuda")


def timed(fn):
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
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(R):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / G * 1e3)
    ts.sort()
    return {"median": round(ts[len(ts) // 2], 2), "min": round(ts[0], 2)}


legs = {"obs": lambda k: env.build_obs(out=bufs),
        "step_obs": lambda k: env.step_obs(acts[k % G], out=(r, sh, dn), obs_out=bufs),
        "step": lambda k: env.step(acts[k % G], out=(r, sh, dn))}
only = os.environ.get("C3_ONLY")
out = {k: timed(f) for k, f in legs.items() if not only or k == only}
print(json.dumps(out))
