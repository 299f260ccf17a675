"""Per-launch floor of graph-replayed kernels at the bench's grid (profiling only)."""
import ctypes as C
import json
import os
import sys

import torch

here = os.path.dirname(os.path.abspath(__file__))
L = C.CDLL(os.path.join(here, "libexp.so"))
dev = torch.device("cuda", 0)
s = torch.cuda.Stream()
out = {}
for E in (1024, 4096):
    A, P = 5, 50
    rob = torch.randint(0, 1 << 20, (E * A,), dtype=torch.int32, device=dev)
    pkg = torch.randint(0, 1 << 30, (E * P,), dtype=torch.int64, device=dev)
    tab = torch.randint(0, 200, (256,), dtype=torch.uint8, device=dev)
    ro = torch.empty_like(rob)
    calls = {
        "empty": lambda: L.exp_empty(E, C.c_void_p(s.cuda_stream)),
        "rt1": lambda: L.exp_rt1(C.c_void_p(rob.data_ptr()), C.c_void_p(pkg.data_ptr()), C.c_void_p(ro.data_ptr()), E, A, P, C.c_void_p(s.cuda_stream)),
        "rt1_big": lambda: L.exp_rt1_big(C.c_void_p(rob.data_ptr()), C.c_void_p(pkg.data_ptr()), C.c_void_p(ro.data_ptr()), E, A, P, C.c_void_p(s.cuda_stream)),
        "icache_line": lambda: L.exp_icache(0, C.c_void_p(ro.data_ptr()), E, C.c_void_p(s.cuda_stream)),
        "icache_loop": lambda: L.exp_icache(1, C.c_void_p(ro.data_ptr()), E, C.c_void_p(s.cuda_stream)),
        "salu2048": lambda: L.exp_salu(0, C.c_void_p(ro.data_ptr()), E, C.c_void_p(s.cuda_stream)),
        "mixed1024x2": lambda: L.exp_salu(1, C.c_void_p(ro.data_ptr()), E, C.c_void_p(s.cuda_stream)),
        "klines1": lambda: L.exp_klines(1, C.c_void_p(rob.data_ptr()), C.c_void_p(ro.data_ptr()), E, C.c_void_p(s.cuda_stream)),
        "klines3": lambda: L.exp_klines(3, C.c_void_p(rob.data_ptr()), C.c_void_p(ro.data_ptr()), E, C.c_void_p(s.cuda_stream)),
        "klines6": lambda: L.exp_klines(6, C.c_void_p(rob.data_ptr()), C.c_void_p(ro.data_ptr()), E, C.c_void_p(s.cuda_stream)),
        "klines9": lambda: L.exp_klines(9, C.c_void_p(rob.data_ptr()), C.c_void_p(ro.data_ptr()), E, C.c_void_p(s.cuda_stream)),
        "klchain1": lambda: L.exp_klines_chain(1, C.c_void_p(rob.data_ptr()), C.c_void_p(ro.data_ptr()), E, C.c_void_p(s.cuda_stream)),
        "klchain9": lambda: L.exp_klines_chain(9, C.c_void_p(rob.data_ptr()), C.c_void_p(ro.data_ptr()), E, C.c_void_p(s.cuda_stream)),
        "rt2": lambda: L.exp_rt2(C.c_void_p(rob.data_ptr()), C.c_void_p(pkg.data_ptr()), C.c_void_p(tab.data_ptr()), C.c_void_p(ro.data_ptr()), E, A, P, C.c_void_p(s.cuda_stream)),
    }
    for name, fn in calls.items():
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            fn()
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=s):
                for _ in range(100):
                    fn()
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        out[f"{name}_E{E}_us"] = round(e0.elapsed_time(e1) / 1000 * 1e3, 3)
print(json.dumps(out))
