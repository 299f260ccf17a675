"""Summarise rocprofv3 CSVs under gpurun_out/prof_<tag>: median per counter for one kernel."""
import collections
import csv
import glob
import json
import sys

tag, kern = sys.argv[1], sys.argv[2]
out = {}
for f in glob.glob(f"gpurun_out/prof_{tag}/*/run_counter_collection.csv"):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            d[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in d.items():
        v.sort()
        out[k] = {"median": v[len(v) // 2], "mean": sum(v) / len(v), "dispatches": len(v)}
for f in glob.glob(f"gpurun_out/prof_{tag}/trace/run_kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        if kern in r["Name"]:
            out.setdefault("kernel_stats", []).append({k: r[k] for k in ("Name", "Calls", "AverageNs", "MinNs", "MaxNs")})
print(json.dumps(out, indent=1))
