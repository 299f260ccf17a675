#!/bin/bash
# Observation builder per output subset, config 3b (MO = MP = 100), builds A and B interleaved.
set -u
for rep in 1 2; do
  for V in A B; do
    echo -n "$V $rep "
    OBS_MO_MP=100,100 MDL_PROFILING=1 MDL_LIB_PATH=marl-delivery_amd/build/ablate/libmdl_$V.so timeout -k 10 200 python scripts/exp/obs_parts.py 2>/dev/null || exit 1
  done
done
