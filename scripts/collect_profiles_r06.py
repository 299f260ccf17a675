"""Copy the round-6 profile pass (gpurun_out/prof_r06, scripts/profile_r06.sh) into profiles/r06/final/: kernel
stats CSVs of the driver's bench command, the 2000-step config-2 bench and the config-3 / config-5 bench
lines, the bench JSON lines, the per-dispatch PMC rows (FETCH_SIZE, WRITE_SIZE, the SQ set) trimmed to
(Dispatch_Id, Kernel_Name, Counter_Name, Counter_Value), SQ per-wave summaries; then regenerate
profiles/traffic.json from the committed PMC rows (scripts/traffic_json.py), so that bench.py's
roofline.traffic can be recomputed from files under profiles/ alone (tests/test_host_cpu.py)."""
import collections
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "gpurun_out", "prof_r06")
DST = os.path.join(REPO, "profiles", "r06", "final")
# PMC directory -> (kernel-name substring kept, traffic.json spec suffix); the c5full kernel is whichever
# layout AUTO took (k_step_halves or k_step), read from the pass itself
C4MAPS = "+".join(f"map{i}.txt" for i in range(1, 6))
PMC = {"c2": ("k_step<", ":4096,5,50,map1.txt:k_step<:0"),
       "c3": ("k_step_obs", ":16384,5,50,map1.txt:k_step_obs:1"),
       "c4": ("k_step_rows<", ":65536,5,50," + C4MAPS + ":k_step_rows<:0"),
       "c5full": (None, ":131072,16,100,synthetic64.txt:{k}:0")}
PMC_FULL = {}


def c5_kernel():
    for f in glob.glob(os.path.join(SRC, "c5full", "fetch", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            return "k_step_halves<" if "k_step_halves" in r["Kernel_Name"] else "k_step<"
    raise SystemExit("no c5full PMC rows")


def one(pattern):
    fs = sorted(glob.glob(os.path.join(SRC, pattern), recursive=True))
    if not fs:
        raise SystemExit(f"missing {pattern} under {SRC}")
    return fs[0]


def trim_pmc(src_dir, dst_file, kern):
    rows = []
    for f in glob.glob(os.path.join(src_dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
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
    k5 = c5_kernel()
    PMC["c5full"] = (k5, PMC["c5full"][1].format(k=k5))
    stats = {"driver": "driver_command_kernel_stats.csv", "trace": "config2_bench2000_kernel_stats.csv",
             "c3trace": "config3_bench_kernel_stats.csv", "c4trace": "config4_bench_kernel_stats.csv",
             "c5trace": "config5_bench_kernel_stats.csv"}
    for d, name in stats.items():
        shutil.copy(one(f"{d}/**/run_kernel_stats.csv"), os.path.join(DST, name))
    for name in ("driver_bench", "trace_bench", "c3_bench", "c4_bench", "c5_bench"):
        shutil.copy(os.path.join(SRC, name + ".json"), os.path.join(DST, name + ".json"))
    summary = []
    for cfg, (kern, _) in PMC.items():
        for kind in ("fetch", "write", "sq"):
            rows = trim_pmc(os.path.join(SRC, cfg, kind), os.path.join(DST, "pmc", cfg, kind, "run_counter_collection.csv"),
                            kern)
            if not rows:
                raise SystemExit(f"no {kern} rows in {cfg}/{kind}")
            if kind == "sq":
                agg = collections.defaultdict(list)
                for _, _, n, v in rows:
                    agg[n].append(float(v))
                m = {n: sorted(v)[len(v) // 2] for n, v in agg.items()}
                wv = m.get("SQ_WAVES", 1.0)
                summary.append(f"{cfg} {kern} per wave (medians over dispatches): " +
                               json.dumps({n: round(v / wv, 1) for n, v in sorted(m.items())}))
    for cfg, (kern, _) in PMC_FULL.items():
        for kind in ("fetch", "write"):
            if not trim_pmc(os.path.join(SRC, cfg, kind), os.path.join(DST, "pmc", cfg, kind, "run_counter_collection.csv"),
                            kern):
                raise SystemExit(f"no {kern} rows in {cfg}/{kind}")
    for f in stats.values():
        for r in csv.DictReader(open(os.path.join(DST, f))):
            if r["Name"].startswith("void mdl::") or r["Name"].startswith("mdl::"):
                summary.append(f"{f}: {r['Name'][:70]} calls {r['Calls']} avg {float(r['AverageNs']) / 1e3:.3f} us")
    for name in ("driver_bench", "trace_bench", "c3_bench", "c4_bench", "c5_bench"):
        d = json.loads(open(os.path.join(DST, name + ".json")).read().strip().splitlines()[-1])
        summary.append(f"{name}: value {d['value']:.4e} ms_per_step {d['ms_per_step']:.6f} kernel_us "
                       f"{d['roofline']['kernel_us']:.3f} frac {d['roofline']['frac']:.4f} "
                       f"launch_floor_ms_per_step {d.get('launch_floor_ms_per_step')}")
    open(os.path.join(DST, "profile_summary.txt"), "w").write("\n".join(summary) + "\n")
    specs = [f"{cfg}=" + os.path.join(DST, "pmc", cfg) + suffix for cfg, (_, suffix) in {**PMC, **PMC_FULL}.items()]
    subprocess.check_call([sys.executable, os.path.join(REPO, "scripts", "traffic_json.py"),
                           os.path.join(REPO, "profiles", "traffic.json"),
                           os.path.join(REPO, "profiles", "r03", "fetch_calibration.json")] + specs,
                          stdout=open(os.path.join(DST, "traffic.log"), "w"))
    print("\n".join(summary))


if __name__ == "__main__":
    main()
