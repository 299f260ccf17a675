"""Per-subset medians of k_obs counters from profile_obs.sh (dispatch order:
obs_parts.py's 5 subsets x 23 launches; the first 3 of each are warmup)."""
import collections
import csv
import glob
import json
import sys

NAMES = ["actor_map", "actor_vec", "critic_map", "critic_vec", "all"]
out = collections.defaultdict(dict)
for f in glob.glob(sys.argv[1] + "/*/run_counter_collection.csv"):
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if "k_obs" in r["Kernel_Name"]:
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] = per[int(r["Dispatch_Id"])].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = sorted(per)
    for g, name in enumerate(NAMES):
        grp = ids[g * 23 + 3:(g + 1) * 23]
        for cn in per[ids[0]]:
            v = sorted(per[i][cn] for i in grp)
            out[name][cn] = v[len(v) // 2]
res = {}
for name, d in out.items():
    w = d.get("SQ_WAVES", 16384) or 16384
    res[name] = {k: (v / w if k.startswith("SQ_INSTS") or k in ("SQ_WAVE_CYCLES", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY",
                                                                 "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU") else v)
                 for k, v in d.items()}
print(json.dumps(res, indent=1))
