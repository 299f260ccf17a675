mkdir -p gpurun_out/r03ap
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03ap/prof -o driver -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/r03ap/driver.json 2> gpurun_out/r03ap/driver.err || exit $?
python3 - <<'PY'
import csv, glob, json, statistics
t = glob.glob("gpurun_out/r03ap/prof/**/driver_kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(t)) if "k_step<true, 1, false, 5>" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
print("k_step dispatches", len(d), "mean us %.2f" % statistics.mean(d))
# the timed region: the 20 dispatches of the second replay of the 20-node graph (after the upload replay and the
# 5-step warmup graph): find runs of 20 back-to-back dispatches (gaps < 3 us)
runs, cur = [], [0]
for i in range(1, len(rows)):
    gap = (int(rows[i]["Start_Timestamp"]) - int(rows[i - 1]["End_Timestamp"])) / 1e3
    if gap < 3.0: cur.append(i)
    else: runs.append(cur); cur = [i]
runs.append(cur)
for r in runs:
    if len(r) >= 5:
        print("run of", len(r), "dispatches: mean duration us %.2f" % statistics.mean(d[i] for i in r),
              "span us %.1f" % ((int(rows[r[-1]]["End_Timestamp"]) - int(rows[r[0]]["Start_Timestamp"])) / 1e3))
b = json.loads(open("gpurun_out/r03ap/driver.json").read().strip().splitlines()[-1])
print("bench kernel_us %.2f" % b["roofline"]["kernel_us"], "value %.3e" % b["value"])
PY
