"""Experiment (profiling only): per-call cost of the helper-compatible functions on a
map1 state dict (5 robots, 20 tracker entries) -- the reference's CPU costs are in
SURVEY.md section 6 (19.5 / 27.7 / 80.7 / 114.9 / 13.0 us)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "marl-delivery_amd"))
from marl_gpu import helper as Hh  # noqa: E402
from marl_gpu.maps import load_map, map_path  # noqa: E402

grid = load_map(map_path("map1.txt"))
rs = np.random.RandomState(0)
free = [(r, c) for r in range(10) for c in range(10) if grid[r][c] == 0]
robots = [(free[i][0] + 1, free[i][1] + 1, 0) for i in range(5)]
trk = {}
for j in range(20):
    s_, t_ = free[rs.randint(len(free))], free[rs.randint(len(free))]
    trk[j + 1] = dict(id=j + 1, start_pos=s_, target_pos=t_, start_time=0, deadline=50 + j,
                      status="waiting" if j % 3 else "in_transit")
state = dict(time_step=10, map=grid, robots=robots, packages=[])
cur = dict(time_step=11, map=grid, robots=robots, packages=[])
acts = [("S", "0")] * 5
calls = {
    "convert_observation": lambda: Hh.convert_observation(state, trk, 0),
    "generate_vector_features(4,5)": lambda: Hh.generate_vector_features(state, trk, 0, 500, 4, 5),
    "generate_vector_features(100,100)": lambda: Hh.generate_vector_features(state, trk, 0, 500),
    "convert_global_state": lambda: Hh.convert_global_state(state, trk, 500),
    "compute_shaped_rewards": lambda: Hh.compute_shaped_rewards(0.0, state, cur, acts, trk, 5),
}
for name, fn in calls.items():
    for _ in range(20):
        fn()
    t0 = time.perf_counter()
    n = 500
    for _ in range(n):
        fn()
    print(f"{name:36s} {(time.perf_counter() - t0) / n * 1e6:8.1f} us per call")
