"""Write profiles/traffic.json (the roofline.traffic source bench.py reads) from rocprofv3 PMC
passes of the current build, corrected by the committed FETCH_SIZE calibration.

Usage: python scripts/traffic_json.py OUT.json CAL.json NAME=DIR[:config[:kernel[:obs]]] ...
  DIR holds fetch/ and write/ rocprofv3 CSV passes (run_counter_collection.csv) of the kernel;
  config = envs,agents,packages,map1+map2... (default 4096,5,50,map1.txt); kernel = the kernel-name
  substring (default k_step); obs = 1 for a step + observation launch (bench.py --config 3), whose
  reads are the step's (the same calibrated access shapes) and whose writes are mostly observations.
Counter values are KB (x1024).  HBM bytes per launch = FETCH_SIZE x (1 / the calibrated
counted-over-read ratio of the step's access shape) + WRITE_SIZE (exact for the writes, per
the calibration's write column)."""
import collections
import csv
import glob
import json
import os
import sys


def median_counter(d, counter, kern):
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and kern in r["Kernel_Name"]:
                vals.append(float(r["Counter_Value"]) * 1024.0)
    vals.sort()
    return (vals[len(vals) // 2], len(vals)) if vals else (None, 0)


REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rel(path):
    """Repo-relative form of a path, so the record reads the same on any box."""
    return os.path.relpath(os.path.abspath(path), REPO)


def main():
    out, cal_path = sys.argv[1], sys.argv[2]
    cal = json.load(open(cal_path))
    step_row = [r for r in cal["rows"] if r["shape"].startswith("step_shape") and r["placement"] == "hot"][0]
    ratio = step_row["fetch_over_algorithmic"]          # counted / read bytes for the step's loads
    recs = []
    for spec in sys.argv[3:]:
        name, rest = spec.split("=", 1)
        d, _, more = rest.partition(":")
        cfg, _, more = more.partition(":")
        kern, _, obs = more.partition(":")
        kern = kern or "k_step"
        E, A, P, maps = (cfg or "4096,5,50,map1.txt").split(",")
        fetch, nf = median_counter(os.path.join(d, "fetch"), "FETCH_SIZE", kern)
        write, nw = median_counter(os.path.join(d, "write"), "WRITE_SIZE", kern)
        if fetch is None or write is None:
            raise SystemExit(f"{name}: no FETCH_SIZE / WRITE_SIZE rows for {kern} under {d}")
        read_bytes = fetch / ratio
        recs.append({
            "name": name,
            "config": {"envs": int(E), "agents": int(A), "packages": int(P), "maps": maps.split("+")},
            "kernel": "mdl::" + kern,
            "obs": obs == "1",
            "hbm_bytes_per_launch": read_bytes + write,
            "fetch_size_bytes_median": fetch, "fetch_dispatches": nf,
            "read_bytes_corrected": read_bytes,
            "write_bytes": write, "write_dispatches": nw,
            "source": f"{rel(d)} (rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, eager launches, medians; "
                      f"KB x1024); FETCH_SIZE / {ratio:.4f}: the counted-over-read ratio measured for the step's own "
                      f"access shapes by scripts/exp/fetch_cal.hip ({rel(cal_path)}, row 'step_shape', hot)",
        })
    json.dump({"calibration": rel(cal_path), "fetch_ratio": ratio, "records": recs}, open(out, "w"), indent=1)
    print(json.dumps(recs, indent=1))


if __name__ == "__main__":
    main()
