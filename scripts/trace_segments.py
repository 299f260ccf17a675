"""Split a rocprofv3 kernel trace of bench.py into its phases (eager warmup,
graph replay, eager, isolated launches) and report per-phase kernel durations,
so the rocprof average can be set beside bench.py's event-timed kernel_us.
usage: trace_segments.py <run_kernel_trace.csv> <kernel-substring> <warmup> <steps>"""
import csv
import json
import sys

import numpy as np

path, kern, W, K = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
rows = [r for r in csv.DictReader(open(path)) if kern in r["Kernel_Name"]]
s = np.array([int(r["Start_Timestamp"]) for r in rows])
e = np.array([int(r["End_Timestamp"]) for r in rows])
o = np.argsort(s)
s, e = s[o], e[o]
d = e - s
# bench.py order: W eager warmup, 1 priming launch, the captured graph replayed
# K/G times (K launches), K eager launches, then <=200 isolated launches
seg = {"warmup_eager": (0, W), "graph_replay": (W + 1, W + 1 + K), "eager": (W + 1 + K, W + 1 + 2 * K),
       "isolated": (W + 1 + 2 * K, len(d))}
out = {"kernel": rows[0]["Kernel_Name"], "dispatches": len(d)}
for k, (a, b) in seg.items():
    b = min(b, len(d))
    if b > a:
        out[k] = {"n": int(b - a), "mean_ns": float(d[a:b].mean()), "median_ns": float(np.median(d[a:b])),
                  "mean_start_to_start_ns": float(np.mean(np.diff(s[a:b]))) if b - a > 1 else None}
print(json.dumps(out, indent=1))
