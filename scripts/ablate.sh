#!/bin/bash
# Build ablation variants of libmdl.so (profiling only) into marl-delivery_amd/build/ablate/:
# mdl_kernels.hip recompiled with -DMDL_ABLATE=<bits> (each bit removes one section of the
# step, see mdl_kernels.hip) and the production flags (incl. kernarg preloading), linked with
# the production objects of the other files (run `make -C marl-delivery_amd` first).
set -e
cd "$(dirname "$0")/../marl-delivery_amd"
mkdir -p build/ablate
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt"
for A in ${VARIANTS:-0 1 2 4 8 16 32 64}; do
  ( /opt/rocm/bin/hipcc $F -mllvm -amdgpu-kernarg-preload-count=14 -mllvm -amdgpu-sched-strategy=max-ilp -DMDL_PROFILING_BUILD -DMDL_ABLATE=$A -I../include -Icsrc \
        -c csrc/mdl_kernels.hip -o build/ablate/k_$A.o &&
    /opt/rocm/bin/hipcc $F -shared -o build/ablate/libmdl_$A.so build/ablate/k_$A.o build/mdl_engine.o \
        build/mdl_rollout.o build/mdl_greedy.o ) &
done
wait
ls build/ablate
