#!/bin/bash
# SQ counters of the config-3 fused step + observation kernel (k_step_obs) and builder (k_obs_small)
# per variant (VARIANTS: main or build/ab names), one rocprofv3 --pmc pass per counter group.
set -u
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/c3sq
mkdir -p $O
for V in ${VARIANTS:-main}; do
  if [ "$V" = main ]; then L=$R/marl-delivery_amd/marl_gpu/libmdl.so; else L=$R/marl-delivery_amd/build/ab/libmdl_$V.so; fi
  for G in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
    tag=$(echo $G | cut -d' ' -f2)
    MDL_PROFILING=1 MDL_LIB_PATH=$L C3_R=3 timeout -s KILL 120 rocprofv3 --pmc $G --kernel-include-regex "k_step_obs|k_obs_small" \
        -d $O/${V}_$tag -o run --output-format csv -- python3 $R/scripts/exp/c3_time.py > $O/${V}_$tag.log 2>&1 || exit $?
  done
  python3 - $O $V <<'PY'
import csv, glob, collections, json, sys
O, V = sys.argv[1], sys.argv[2]
for kern in ("k_step_obs", "k_obs_small"):
    agg = collections.defaultdict(list)
    for f in glob.glob(f"{O}/{V}_*/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {n: sorted(v)[len(v) // 2] for n, v in agg.items()}
    w = m.get("SQ_WAVES", 1)
    per = {n.replace("SQ_", ""): round(v / w, 1) for n, v in sorted(m.items()) if n.startswith("SQ_") and n != "SQ_WAVES"}
    per["GRBM_GUI_ACTIVE"] = m.get("GRBM_GUI_ACTIVE")
    print(V, kern, json.dumps(per))
PY
done
