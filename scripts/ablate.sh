#!/bin/bash
# Build ablation variants of libmdl.so (profiling only) into build/ablate/.
set -e
cd "$(dirname "$0")/../marl-delivery_amd"
mkdir -p build/ablate
for A in ${VARIANTS:-0 1 2 3 4 8 15}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt -DMDL_ABLATE=$A \
     -I../include -Icsrc -shared csrc/mdl_kernels.hip csrc/mdl_engine.hip csrc/mdl_rollout.hip csrc/mdl_greedy.hip -o build/ablate/libmdl_$A.so &
done
wait
ls build/ablate
