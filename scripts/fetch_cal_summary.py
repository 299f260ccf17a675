"""Summarise the FETCH_SIZE / WRITE_SIZE calibration passes (scripts/fetch_cal.sh).

Per kernel of scripts/exp/fetch_cal.hip the dispatches come in the order the program
prints them (per shape: `reps` "hot" launches, then `reps` "cold" ones).  Counter values
are KB (x1024).  Output: per shape and placement the median counted bytes per dispatch
and their ratio to the algorithmic read bytes."""
import collections
import csv
import glob
import json
import os
import sys

O = sys.argv[1]
plan = [json.loads(ln) for ln in open(os.path.join(O, "plain.jsonl")) if ln.startswith("{")]


def load(counter):
    per = collections.defaultdict(list)   # kernel base name -> [(dispatch id, value)]
    for f in glob.glob(os.path.join(O, counter.split("_")[0].lower(), "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"]
            key = "k_stream16" if "k_stream16" in name else \
                "k_rows<%s>" % name.split("k_rows<")[1].split(">")[0] if "k_rows<" in name else None
            if key:
                per[key].append((int(r["Dispatch_Id"]), float(r["Counter_Value"]) * 1024.0))
    return {k: [v for _, v in sorted(x)] for k, x in per.items()}


fetch, write = load("FETCH_SIZE"), load("WRITE_SIZE")
used = collections.Counter()
rows = []
for p in plan:
    k = p["kernel"]
    n = p["dispatches"]
    i0 = used[k]
    used[k] += n
    f = sorted(fetch.get(k, [])[i0:i0 + n])
    w = sorted(write.get(k, [])[i0:i0 + n])
    fm = f[len(f) // 2] if f else None
    wm = w[len(w) // 2] if w else None
    rows.append(dict(shape=p["shape"], kernel=k, placement=p["placement"], dispatches=len(f),
                     algorithmic_read_bytes=p["algorithmic_read_bytes"], fetch_size_bytes_median=fm,
                     fetch_over_algorithmic=None if fm is None else fm / p["algorithmic_read_bytes"],
                     write_size_bytes_median=wm, write_bytes=p["write_bytes"]))
print(json.dumps({"units": "bytes per dispatch (counter KB x 1024), medians", "rows": rows}, indent=1))
