"""Experiment (profiling only): per-call cost of the dict API -- compat.Environment.step and
compat.VectorizedEnv.step (all envs, and an `indices=` subset) -- on map1, 5 robots, 20
packages, random string actions drawn up front (the reference's randomagent.py action set)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "marl-delivery_amd"))
from marl_gpu import compat  # noqa: E402

rs = np.random.RandomState(0)
moves, ops = ["S", "L", "R", "U", "D"], ["0", "1", "2"]


def draw(n_envs, k):
    return [[[(moves[rs.randint(5)], ops[rs.randint(3)]) for _ in range(5)] for _ in range(n_envs)] for _ in range(k)]


def timeit(fn, acts):
    for a in acts[:20]:
        fn(a)
    t0 = time.perf_counter()
    for a in acts[20:]:
        fn(a)
    return (time.perf_counter() - t0) / (len(acts) - 20) * 1e6


K = 2000
env = compat.Environment("map1.txt", 100, 5, 20, seed=1)
env.reset()
print(f"Environment.step                 {timeit(lambda a: env.step(a[0]), draw(1, K)):8.1f} us per call")
for n in (8, 64):
    v = compat.VectorizedEnv(None, n, map_file="map1.txt", max_time_steps=100, n_robots=5, n_packages=20, seed=3)
    v.reset()
    us = timeit(lambda a: v.step(a), draw(n, K // 4))
    print(f"VectorizedEnv({n:2d}).step             {us:8.1f} us per call, {us / n:6.2f} us per env")
    idx = list(range(0, n, 2))
    us = timeit(lambda a: v.step(a[:len(idx)], indices=idx), draw(n, K // 4))
    print(f"VectorizedEnv({n:2d}).step(indices) {us:8.1f} us per call ({len(idx)} envs)")
