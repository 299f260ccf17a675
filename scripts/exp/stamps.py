"""Per-section cycle costs of k_step from the MDL_STAMPS diagnostic build (profiling only).

Run with MDL_PROFILING=1 MDL_LIB_PATH=marl-delivery_amd/build/stamps/libmdl.so."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "marl-delivery_amd"))
import marl_gpu  # noqa: E402
from marl_gpu import _lib  # noqa: E402
from marl_gpu.maps import grid_array, load_map, map_path  # noqa: E402

names = ["kernarg", "w_map", "loads_decode", "move", "pkgs", "term", "shape_pre", "agent_loops", "shape_sum",
         "tracker", "write"]
res = {}
for E in [int(x) for x in (sys.argv[1:] or ["1024", "4096"])]:
    env = marl_gpu.BatchedEnv(grid_array(load_map(map_path("map1.txt"))), E, 5, 50, 500, seed=42, tracker="mappo")
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(1)
    acts = torch.randint(0, 15, (300, E, 5), dtype=torch.uint8, device="cuda", generator=g)
    if os.environ.get("FUSED"):
        env.step_fused(acts[:250])
        env.step_fused(acts[250:])   # stamps of steps 2..8 = the last fused step
    else:
        for k in range(300):
            env.step(acts[k])
    torch.cuda.synchronize()
    buf = np.zeros((65536, 16), np.uint64)
    assert _lib.lib().mdl_debug_stamps(C.c_void_p(buf.ctypes.data), C.c_size_t(buf.nbytes)) == 0
    st = buf[:E, :12].astype(np.int64)
    d = np.diff(st, axis=1)
    mv = buf[:E, [3, 12, 13, 14, 15, 4]].astype(np.int64)
    if os.environ.get("MOVE_DETAIL"):
        md = np.diff(mv, axis=1)
        ok = (mv[:, 1:5] != 0).all(1)   # envs that had movers (inner stamps ran)
        print("move detail (prop, movers loop, occ loop, fixed point, tail):",
              [float(np.median(md[ok, i])) for i in range(5)], "envs", int(ok.sum()), file=sys.stderr)
    res[E] = {
        "median_cycles": {n: float(np.median(d[:, i])) for i, n in enumerate(names)},
        "p90_cycles": {n: float(np.percentile(d[:, i], 90)) for i, n in enumerate(names)},
        "wave_total_median": float(np.median(st[:, 11] - st[:, 0])),
    }
print(json.dumps(res, indent=1))
