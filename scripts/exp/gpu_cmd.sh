mkdir -p gpurun_out/r03aa
export TMPDIR=/tmp
for MM in 100,100 4,5; do
OBS_WHICH=all OBS_MO_MP=$MM timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_obs_small -d gpurun_out/r03aa/w_$MM -o run --output-format csv -- python3 scripts/exp/obs_parts.py > gpurun_out/r03aa/w_$MM.log 2>&1 || exit $?
done
python3 - <<'PY'
import csv, glob, statistics
for mm in ("100,100", "4,5"):
    v = [float(r["Counter_Value"]) for f in glob.glob(f"gpurun_out/r03aa/w_{mm}/**/run_counter_collection.csv", recursive=True) for r in csv.DictReader(open(f)) if r["Counter_Name"] == "WRITE_SIZE"]
    print(mm, "launches", len(v), "WRITE_SIZE median (KB)", statistics.median(v))
PY
