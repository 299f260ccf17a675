"""Dependency-latency probes (profiling only): ns per chained instruction pair."""
import ctypes as C
import json
import os

import torch

print("torch up", flush=True)

L = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libexp.so"))
s = torch.cuda.Stream()
out = torch.empty(1 << 16, dtype=torch.int32, device="cuda")
names = {1: "readlane->salu", 2: "readlane->valu", 3: "salu->valu", 4: "valu->valu", 5: "salu->salu",
         6: "dpp chain (+2 nops)"}


def t(which, E, reps):
    fn = lambda: L.exp_probe(which, C.c_void_p(out.data_ptr()), E, reps, C.c_void_p(s.cuda_stream))  # noqa
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
    return a.elapsed_time(b) / 500 * 1e3


res = {}
for w, nm in names.items():
    for E in (1024, 4096):
        d = t(w, E, 9) - t(w, E, 1)
        res[f"{nm} E{E}"] = round(d * 1e3 / (8 * 64), 2)   # ns per pair
        print(nm, E, res[f"{nm} E{E}"], flush=True)
print(json.dumps(res, indent=0))
