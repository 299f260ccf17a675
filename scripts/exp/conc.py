"""Experiment (profiling only): per-step time of graph-replayed mdl_step vs the
env count, and with the envs split into G groups whose graphs replay
concurrently on G streams (async env groups)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "marl-delivery_amd"))
import marl_gpu  # noqa: E402
from marl_gpu.maps import grid_array, load_map, map_path  # noqa: E402

dev = torch.device("cuda", 0)
grid = grid_array(load_map(map_path("map1.txt")))
GS = 100


def make(E, seed):
    env = marl_gpu.BatchedEnv(grid, E, 5, 50, 500, seed=seed, tracker="mappo", shaping="mappo", device=dev)
    env.reset()
    gen = torch.Generator(device=dev).manual_seed(seed)
    acts = torch.randint(0, 15, (GS, E, 5), generator=gen, device=dev, dtype=torch.int32).to(torch.uint8)
    r = torch.zeros(E, dtype=torch.float64, device=dev)
    sh = torch.zeros(E, dtype=torch.float32, device=dev)
    dn = torch.zeros(E, dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream(device=dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        for k in range(20):
            env.step(acts[k], auto_reset=True, out=(r, sh, dn))
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            for k in range(GS):
                env.step(acts[k], auto_reset=True, out=(r, sh, dn))
    torch.cuda.synchronize()
    return env, g, (acts, r, sh, dn, s)


def run(groups, reps=20):
    for _ in range(2):
        for _, g, x in groups:
            with torch.cuda.stream(x[4]):
                g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        for _, g, x in groups:
            with torch.cuda.stream(x[4]):
                g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / (reps * GS) * 1e6


out = {}
for E in (1024, 2048, 4096, 8192, 16384):
    grp = [make(E, 42)]
    out[f"single_E{E}_us"] = round(run(grp), 3)
    for e, _, _ in grp:
        e.close()
for G, E in ((2, 2048), (4, 1024), (2, 4096)):
    grp = [make(E, 42 + i * E) for i in range(G)]
    out[f"groups{G}x{E}_us"] = round(run(grp), 3)
    for e, _, _ in grp:
        e.close()
print(json.dumps(out))


# per-step fork/join: step k of every group depends on step k-1 of all groups
def make_fj(E, G):
    envs = []
    for i in range(G):
        env = marl_gpu.BatchedEnv(grid, E, 5, 50, 500, seed=42 + i * E, tracker="mappo", shaping="mappo", device=dev)
        env.reset()
        gen = torch.Generator(device=dev).manual_seed(i)
        acts = torch.randint(0, 15, (GS, E, 5), generator=gen, device=dev, dtype=torch.int32).to(torch.uint8)
        bufs = (torch.zeros(E, dtype=torch.float64, device=dev), torch.zeros(E, dtype=torch.float32, device=dev),
                torch.zeros(E, dtype=torch.uint8, device=dev))
        envs.append((env, acts, bufs))
    main = torch.cuda.Stream(device=dev)
    side = [torch.cuda.Stream(device=dev) for _ in range(G - 1)]
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(main):
        for k in range(5):
            for env, acts, bufs in envs:
                env.step(acts[k], auto_reset=True, out=bufs)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=main):
            for k in range(GS):
                for i, s2 in enumerate(side):
                    s2.wait_stream(main)
                    with torch.cuda.stream(s2):
                        env, acts, bufs = envs[i + 1]
                        env.step(acts[k], auto_reset=True, out=bufs)
                env, acts, bufs = envs[0]
                env.step(acts[k], auto_reset=True, out=bufs)
                for s2 in side:
                    main.wait_stream(s2)
    torch.cuda.synchronize()
    return envs, g, main


for G, E in ((2, 2048), (4, 1024), (2, 4096), (4, 2048)):
    envs, g, main = make_fj(E, G)
    out[f"forkjoin{G}x{E}_us"] = round(run([(None, g, (None, None, None, None, main))]), 3)
    for e, _, _ in envs:
        e.close()
print(json.dumps(out))
