#!/bin/bash
# Same-box A/B of k_step_rows builds (VARIANTS, build/ab/libmdl_<v>.so) on config 4 and config-2-shaped
# batches of ENVS envs, against the one-wave-per-env layout of the main build; interleaved REPS times.
set -u
R=$(pwd)
O=$R/gpurun_out/abrows; mkdir -p $O
run() {  # tag lib layout args...
  local t=$1 L=$2 lay=$3; shift 3
  MDL_PROFILING=1 MDL_LIB_PATH=$L timeout -k 10 200 python3 $R/bench.py --step-layout $lay --cpu-seconds 0 --fused-k 0 \
      --no-floor --graph-only "$@" > $O/$t.json 2> $O/$t.err || { tail -5 $O/$t.err; exit 1; }
  python3 -c "
import json
d = json.loads(open('$O/$t.json').read().strip().splitlines()[-1])
print('$t', 'us/step %.3f' % (d['ms_per_step'] * 1e3))"
}
for rep in $(seq 1 ${REPS:-2}); do
  [ "${NOWAVE:-0}" = 1 ] || run wave_c4_$rep $R/marl-delivery_amd/marl_gpu/libmdl.so wave --config 4 --steps 300 --warmup 30 || exit 1
  for V in ${VARIANTS:-w5 w6 w7}; do
    run ${V}_c4_$rep $R/marl-delivery_amd/build/ab/libmdl_$V.so rows --config 4 --steps 300 --warmup 30 || exit 1
  done
  for E in ${ENVS:-4096 8192 12288 16384}; do
    [ "${NOWAVE:-0}" = 1 ] || run wave_e${E}_$rep $R/marl-delivery_amd/marl_gpu/libmdl.so wave --envs $E --steps 1000 --warmup 100 || exit 1
    for V in ${VARIANTS:-w5 w6 w7}; do
      run ${V}_e${E}_$rep $R/marl-delivery_amd/build/ab/libmdl_$V.so rows --envs $E --steps 1000 --warmup 100 || exit 1
    done
  done
done
