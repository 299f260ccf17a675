#!/bin/bash
# As ab_build.sh, but mdl_engine.hip is compiled with the same $DEFS too (variants whose host
# side differs).  Usage: DEFS=... scripts/ab_build2.sh <name>
set -e
N=${1:?name}
cd "$(dirname "$0")/../marl-delivery_amd"
mkdir -p build/ab
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt"
/opt/rocm/bin/hipcc $F -mllvm -amdgpu-kernarg-preload-count=14 -mllvm -amdgpu-sched-strategy=max-ilp -DMDL_PROFILING_BUILD ${DEFS:-} -I../include -Icsrc -c csrc/mdl_kernels.hip \
    -o build/ab/k_$N.o &
/opt/rocm/bin/hipcc $F -DMDL_PROFILING_BUILD ${DEFS:-} -I../include -Icsrc -c csrc/mdl_engine.hip -o build/ab/e_$N.o
wait
/opt/rocm/bin/hipcc $F -shared -o build/ab/libmdl_$N.so build/ab/k_$N.o build/ab/e_$N.o build/mdl_rollout.o \
    build/mdl_greedy.o
ls -la build/ab/libmdl_$N.so
