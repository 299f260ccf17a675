"""v_readlane issue-cost probe (profiling only)."""
import ctypes as C
import json
import os

import torch

L = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libexp.so"))
s = torch.cuda.Stream()
out = torch.empty(1 << 16, dtype=torch.int32, device="cuda")
res = {}
for E in (1024, 4096):
    for which, name in ((0, "readlane64"), (1, "vadd64")):
        for reps in (1, 9):
            fn = lambda: L.exp_rl(which, C.c_void_p(out.data_ptr()), E, reps, C.c_void_p(s.cuda_stream))  # noqa
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(s):
                fn()
                torch.cuda.synchronize()
                with torch.cuda.graph(g, stream=s):
                    for _ in range(50):
                        fn()
            g.replay()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10):
                g.replay()
            b.record()
            torch.cuda.synchronize()
            res[f"{name}_x{reps}_E{E}_us"] = round(a.elapsed_time(b) / 500 * 1e3, 3)
# per readlane: (t(x9) - t(x1)) / (8*64)
for E in (1024, 4096):
    for name in ("readlane64", "vadd64"):
        d = res[f"{name}_x9_E{E}_us"] - res[f"{name}_x1_E{E}_us"]
        res[f"{name}_E{E}_ns_per_instr"] = round(d * 1e3 / (8 * 64), 3)
print(json.dumps(res))
