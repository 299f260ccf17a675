"""Secondary measurements for BASELINE.json configs 3-5 (single GPU slices).

  --config 1   map1, A=5, ONE env driven through the dict API by a random agent (plumbing)
  --config 3   map1, A=5, E=16384: step + full observation build every step
               (actor 6ch map + vector 52 (MO=4, MP=5), critic 4ch map + vector 1301)
  --config 3b  as 3 with the 1007-dim actor vector (MO=MP=100)
  --config 4   map1..map5 mixed, A=5, E=65536/8 per GPU (one GPU's shard), step only
  --config 5   synthetic 64x64, A=16, P=100, E=131072/8 per GPU, step; full observations per
               chunk of 4096 envs (MDL_OBS_CHUNK)
  --config rollout / rollout_graph   MAPPO rollout on the device
  --config alt      IDQ/qmix featurizers (§8(f)2)
  --config greedy   batched greedy baseline (§8(f)3)

Prints one JSON line per config with per-kernel HIP-event times and the
algorithmic-bytes roofline of SURVEY.md §8(d).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "marl-delivery_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM = 8000.0


def timed(fn, n):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for k in range(n):
        fn(k)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3  # us per call


def graph_timed(fn, G, reps):
    """us per step of G captured calls fn(0..G-1) replayed `reps` times (after one untimed
    replay): the kernels without the host launch path."""
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
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / (G * reps) * 1e3


def run(cfg, steps, warmup):
    import marl_gpu
    from marl_gpu.maps import grid_array, load_map, map_path
    dev = torch.device("cuda", 0)
    if cfg in ("3", "3b"):
        E, A, P, T = 16384, 5, 50, 500
        mo, mp = (4, 5) if cfg == "3" else (100, 100)
        env = marl_gpu.BatchedEnv(grid_array(load_map(map_path("map1.txt"))), E, A, P, T, seed=42, tracker="mappo",
                                  max_other_robots=mo, max_packages_obs=mp)
        groups = [(0, E)]
    elif cfg == "4":
        E, A, P, T = 65536 // 8, 5, 50, 500
        maps = [grid_array(load_map(map_path(f"map{i}.txt"))) for i in range(1, 6)]
        sizes = [E // 5 + (1 if i < E % 5 else 0) for i in range(5)]
        env_map = np.concatenate([np.full(s, i) for i, s in enumerate(sizes)])
        env = marl_gpu.BatchedEnv(maps, E, A, P, T, seed=42, env_map=env_map, tracker="mappo", max_packages_obs=5)
        starts = np.cumsum([0] + sizes)
        groups = [(int(starts[i]), int(sizes[i])) for i in range(5)]
    else:
        E, A, P, T = 131072 // 8, 16, 100, 500
        env = marl_gpu.BatchedEnv(grid_array(load_map(map_path("synthetic64.txt"))), E, A, P, T, seed=7,
                                  tracker="mappo", max_other_robots=15, max_packages_obs=20, max_robots_state=16,
                                  max_packages_state=100)
        groups = [(0, E)]
    env.reset()
    gen = torch.Generator(device=dev).manual_seed(0)
    G = 50
    acts = torch.randint(0, 15, (G, E, A), generator=gen, device=dev, dtype=torch.int32).to(torch.uint8)
    out = {}
    bufs = None
    if cfg in ("3", "3b"):
        bufs = env.obs_buffers()
    for k in range(warmup):
        env.step(acts[k % G])
    step_eager_us = timed(lambda k: env.step(acts[k % G]), steps)
    r = torch.zeros(E, dtype=torch.float64, device=dev)
    sh = torch.zeros(E, dtype=torch.float32, device=dev)
    dn = torch.zeros(E, dtype=torch.uint8, device=dev)
    step_us = graph_timed(lambda k: env.step(acts[k % G], out=(r, sh, dn)), G, max(1, steps // G))
    out["step_us"] = step_us          # hipGraph-replayed steps (the kernel path)
    out["step_eager_us"] = step_eager_us
    out["agent_steps_per_s_step_only"] = E * A / (step_us * 1e-6)
    step_bytes = (9 * A + 10 * P + 41) * E
    out["step_roofline"] = {"achieved_GBs": step_bytes / (step_us * 1e-6) / 1e9, "frac": step_bytes / (step_us * 1e-6) / 1e9 / HBM}
    if bufs is not None:
        for k in range(3):
            env.build_obs(out=bufs)
        obs_us = timed(lambda k: env.build_obs(out=bufs), max(20, steps // 5))
        H = W = 10
        obs_bytes = E * 4 * (A * 6 * H * W + A * env.actor_vec_dim + 4 * H * W + env.critic_vec_dim)
        out["obs_us"] = obs_us
        out["obs_write_bytes"] = obs_bytes
        out["obs_roofline"] = {"achieved_GBs": obs_bytes / (obs_us * 1e-6) / 1e9,
                               "frac": obs_bytes / (obs_us * 1e-6) / 1e9 / HBM}
        both = timed(lambda k: (env.step(acts[k % G]), env.build_obs(out=bufs)), max(20, steps // 5))
        out["step_plus_obs_eager_us"] = both
        # hipGraph-replayed: step + build_obs as two launches, and mdl_step_obs (one launch)
        both_g = graph_timed(lambda k: (env.step(acts[k % G], out=(r, sh, dn)), env.build_obs(out=bufs)), 10,
                             max(1, steps // 50))
        try:
            fused_g = graph_timed(lambda k: env.step_obs(acts[k % G], out=(r, sh, dn), obs_out=bufs), 10,
                                  max(1, steps // 50))
        except AttributeError:   # an older profiling build without mdl_step_obs (same-box A/B)
            fused_g = float("nan")
        out["step_plus_obs_us"] = both_g
        out["step_obs_fused_us"] = fused_g
        out["agent_steps_per_s_with_obs"] = E * A / (fused_g * 1e-6)
        out["step_obs_roofline"] = {"achieved_GBs": (obs_bytes + step_bytes) / (fused_g * 1e-6) / 1e9,
                                    "frac": (obs_bytes + step_bytes) / (fused_g * 1e-6) / 1e9 / HBM}
    if cfg == "5":
        # the full observations (actor 6 x 64 x 64 maps for 16 agents, vectors
        # MO = 15 / MP = 20, critic map + MR = 16 / MPs = 100 vector) are 1.65 MB per env-step, so they
        # are built and reported per chunk of envs (general k_obs builder: A > 8, P > 64)
        H = W = 64
        chunk = int(os.environ.get("MDL_OBS_CHUNK", "4096"))
        cb = env.obs_buffers(chunk, H, W)
        per_env = 4 * (A * 6 * H * W + A * env.actor_vec_dim + 4 * H * W + env.critic_vec_dim)
        for k in range(2):
            env.build_obs(0, chunk, out=cb)
        nchunks = E // chunk
        reps = 2
        chunk_us = timed(lambda k: env.build_obs((k % nchunks) * chunk, chunk, out=cb), nchunks * reps)
        out["obs_chunk_envs"] = chunk
        out["obs_chunk_us"] = chunk_us
        out["obs_bytes_per_env_step"] = per_env
        out["obs_chunk_roofline"] = {"achieved_GBs": per_env * chunk / (chunk_us * 1e-6) / 1e9,
                                     "frac": per_env * chunk / (chunk_us * 1e-6) / 1e9 / HBM}
        out["obs_all_envs_us"] = chunk_us * nchunks
        out["agent_steps_per_s_step_plus_obs"] = E * A / ((step_us + chunk_us * nchunks) * 1e-6)
        del cb
    out.update(config=cfg, envs=E, agents=A, packages=P, T=T, groups=groups)
    print(json.dumps(out), flush=True)
    env.close()


def run_rollout(steps, graph=False):
    """MAPPO rollout on the device: 4096 envs, map1, A=5, the
    trainer's featurizer sizes, a linear actor on the 52-dim vector and a linear
    critic on the 1301-dim vector; sampling, step, obs into the buffers and GAE
    all on the device.  Reports env agent-steps/s of whole rollouts."""
    import marl_gpu
    import marl_gpu.rollout as R
    from marl_gpu.maps import grid_array, load_map, map_path
    E, A, P, T = 4096, 5, 50, 500
    env = marl_gpu.BatchedEnv(grid_array(load_map(map_path("map1.txt"))), E, A, P, T, seed=42, tracker="mappo",
                              max_other_robots=A - 1, max_packages_obs=5)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    wa = torch.randn(env.actor_vec_dim, 15, device="cuda", generator=g) * 0.1
    wc = torch.randn(env.critic_vec_dim, device="cuda", generator=g) * 0.01
    actor = lambda obs, vec: vec @ wa  # noqa: E731
    critic = lambda gmap, gvec: gvec @ wc  # noqa: E731
    Tr = 128
    ro = R.MappoRollout(env, Tr, seed=1)
    ro.collect(actor, critic, graph=graph)   # (graph: this call runs eagerly and captures)
    torch.cuda.synchronize()
    n = max(1, steps // Tr)
    t0 = time.perf_counter()
    for _ in range(n):
        ro.collect(actor, critic, graph=graph)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out = {"config": "rollout_graph" if graph else "rollout", "envs": E, "agents": A, "rollout_steps": Tr, "rollouts": n,
           "us_per_env_step": dt / (n * Tr) * 1e6, "agent_steps_per_s": E * A * n * Tr / dt,
           "note": "MappoRollout.collect: linear actor/critic (torch), on-device sampling, mdl_step_obs (step + "
                   "next observations in one launch) into the rollout buffers, GAE kernel"}
    print(json.dumps(out))


def run_alt(steps):
    """IDQ/qmix featurizers on 4096 map1 envs, A=5: convert_state for every
    agent (6 x H x W) and convert_global_state_to_tensor (7 x H x W), written by one kernel."""
    import marl_gpu
    from marl_gpu.maps import grid_array, load_map, map_path
    E, A, P, T, H, W = 4096, 5, 50, 500, 10, 10
    env = marl_gpu.BatchedEnv(grid_array(load_map(map_path("map1.txt"))), E, A, P, T, seed=42, tracker="fresh")
    env.reset()
    gen = torch.Generator(device="cuda").manual_seed(0)
    for k in range(60):
        env.step(torch.randint(0, 15, (E, A), generator=gen, device="cuda", dtype=torch.int32).to(torch.uint8))
    out = env.build_obs_alt()
    us = timed(lambda k: env.build_obs_alt(out=out), max(20, steps // 5))
    nbytes = E * 4 * (A * 6 * H * W + 7 * H * W)
    print(json.dumps({"config": "alt_featurizers", "envs": E, "agents": A, "us_per_call": us, "write_bytes": nbytes,
                      "roofline": {"achieved_GBs": nbytes / (us * 1e-6) / 1e9, "frac": nbytes / (us * 1e-6) / 1e9 / HBM},
                      "note": "mdl_build_obs_alt: IDQ convert_state x A + qmix convert_global_state_to_tensor"}),
          flush=True)
    env.close()


def run_greedy(steps):
    """Batched greedy baseline: 4096 map1 envs, A=5, one greedyagent.py
    get_actions per env plus the step, per env-step (one episode, no resets)."""
    import marl_gpu
    from marl_gpu.maps import grid_array, load_map, map_path
    E, A, P, T = 4096, 5, 50, 500
    env = marl_gpu.BatchedEnv(grid_array(load_map(map_path("map1.txt"))), E, A, P, T, seed=42, tracker="fresh")
    env.reset()
    env.greedy_init()
    acts = torch.empty((E, A), dtype=torch.uint8, device="cuda")
    n = min(steps, T - 20)

    def one(k):
        env.greedy_actions(out=acts)
        env.step(acts, auto_reset=False, action_format="codes")

    for k in range(10):
        one(k)
    us = timed(one, n)
    g_us = timed(lambda k: env.greedy_actions(out=acts), 20)
    print(json.dumps({"config": "greedy", "envs": E, "agents": A, "us_per_env_step": us,
                      "agent_steps_per_s": E * A / (us * 1e-6), "greedy_actions_us": g_us,
                      "note": "greedy_actions (BFS distance tables precomputed per map) + mdl_step per env-step"}),
          flush=True)
    env.close()


def run_config1(seconds=5.0):
    """BASELINE.json configs[0]: map1, 5 agents, ONE env, a random agent driving the dict
    API (randomagent.py: np.random.choice over moves and ops per robot) -- plumbing, not a
    throughput path.  Here the env is marl_gpu.compat.Environment (every step a kernel
    launch plus the dict snapshot back to the host); reference on CPU: 62,184 agent-steps/s
    with the agent's time, 243,360 env time only (measured in the build
    container).  Settings of SURVEY.md 8(d) row 1: np.random.seed(2025), env seed 2025,
    P = 50, T = 500, reset on done."""
    from marl_gpu.compat import Environment
    env = Environment("map1.txt", max_time_steps=500, n_robots=5, n_packages=50, seed=2025)
    env.reset()
    np.random.seed(2025)
    moves, ops = ["U", "D", "L", "R", "S"], ["0", "1", "2"]
    n, t_env, t0 = 0, 0.0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        acts = [(np.random.choice(moves), np.random.choice(ops)) for _ in range(5)]
        t1 = time.perf_counter()
        _, _, done, _ = env.step(acts)
        if done:
            env.reset()
        t_env += time.perf_counter() - t1
        n += 1
    wall = time.perf_counter() - t0
    print(json.dumps({"config": "1", "envs": 1, "agents": 5, "steps": n,
                      "agent_steps_per_s_with_agent": 5 * n / wall, "agent_steps_per_s_env_only": 5 * n / t_env,
                      "us_per_step_env": t_env / n * 1e6,
                      "note": "compat.Environment (GPU engine, one env) + the reference random agent's action "
                              "draws; reference on CPU: 62,184 / 243,360 agent-steps/s (BASELINE.md)"}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="3,3b,4,5")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    for c in a.config.split(","):
        if c == "1":
            run_config1()
        elif c in ("rollout", "rollout_graph"):
            run_rollout(a.steps, graph=c == "rollout_graph")
        elif c == "alt":
            run_alt(a.steps)
        elif c == "greedy":
            run_greedy(a.steps)
        else:
            run(c, a.steps, a.warmup)


if __name__ == "__main__":
    main()
