"""Copy the round-4 profile pass (gpurun_out/prof_r04, scripts/profile_r04.sh) into profiles/r04/:
kernel stats CSVs, the per-dispatch PMC rows of k_step (FETCH_SIZE, WRITE_SIZE, the SQ set) trimmed to
(Dispatch_Id, Kernel_Name, Counter_Name, Counter_Value), the bench JSON lines, SQ per-wave summaries; then
regenerate profiles/traffic.json from the committed PMC rows (scripts/traffic_json.py), so that bench.py's
roofline.traffic can be recomputed from files under profiles/ alone."""
import collections
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "gpurun_out", "prof_r04")
DST = os.path.join(REPO, "profiles", "r04")


def one(pattern):
    fs = sorted(glob.glob(os.path.join(SRC, pattern), recursive=True))
    if not fs:
        raise SystemExit(f"missing {pattern} under {SRC}")
    return fs[0]


def trim_pmc(src_dir, dst_file):
    rows = []
    for f in glob.glob(os.path.join(src_dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_step" in r["Kernel_Name"]:
                rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], r["Counter_Name"], r["Counter_Value"]))
    rows.sort()
    os.makedirs(os.path.dirname(dst_file), exist_ok=True)
    with open(dst_file, "w", newline="") as fo:
        w = csv.writer(fo)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writerows(rows)
    return rows


def main():
    os.makedirs(DST, exist_ok=True)
    shutil.copy(one("driver/**/run_kernel_stats.csv"), os.path.join(DST, "driver_command_kernel_stats.csv"))
    shutil.copy(one("trace/**/run_kernel_stats.csv"), os.path.join(DST, "config2_bench2000_kernel_stats.csv"))
    shutil.copy(one("configs/**/run_kernel_stats.csv"), os.path.join(DST, "configs_3_3b_4_5_kernel_stats.csv"))
    for name in ("driver_bench.json", "trace_bench.json", "configs.jsonl"):
        shutil.copy(os.path.join(SRC, name), os.path.join(DST, name))
    summary = []
    for cfg in ("c2", "c5"):
        for kind in ("fetch", "write", "sq"):
            rows = trim_pmc(os.path.join(SRC, cfg, kind), os.path.join(DST, "pmc", cfg, kind, "run_counter_collection.csv"))
            if kind == "sq":
                agg = collections.defaultdict(list)
                for _, _, n, v in rows:
                    agg[n].append(float(v))
                m = {n: sorted(v)[len(v) // 2] for n, v in agg.items()}
                wv = m.get("SQ_WAVES", 1.0)
                summary.append(f"{cfg} k_step per wave (medians over dispatches): " +
                               json.dumps({n: round(v / wv, 1) for n, v in sorted(m.items())}))
    for f in ("config2_bench2000_kernel_stats.csv", "driver_command_kernel_stats.csv", "configs_3_3b_4_5_kernel_stats.csv"):
        for r in csv.DictReader(open(os.path.join(DST, f))):
            if r["Name"].startswith("void mdl::") or r["Name"].startswith("mdl::"):
                summary.append(f"{f}: {r['Name'][:70]} calls {r['Calls']} avg {float(r['AverageNs']) / 1e3:.3f} us")
    open(os.path.join(DST, "profile_summary.txt"), "w").write("\n".join(summary) + "\n")
    subprocess.check_call([sys.executable, os.path.join(REPO, "scripts", "traffic_json.py"),
                           os.path.join(REPO, "profiles", "traffic.json"),
                           os.path.join(REPO, "profiles", "r03", "fetch_calibration.json"),
                           "c2=" + os.path.join(DST, "pmc", "c2"),
                           "c5=" + os.path.join(DST, "pmc", "c5") + ":16384,16,100,synthetic64.txt"],
                          stdout=open(os.path.join(DST, "traffic.log"), "w"))
    print("\n".join(summary))


if __name__ == "__main__":
    main()
