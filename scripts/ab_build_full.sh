#!/bin/bash
# Build an A/B variant of libmdl.so (profiling only) from ALL current sources with extra -D flags
# ($DEFS) into marl-delivery_amd/build/ab/libmdl_<name>.so (host and device code both see DEFS).
set -e
N=${1:?name}
cd "$(dirname "$0")/../marl-delivery_amd"
D=build/abf/$N
mkdir -p $D build/ab
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt -DMDL_PROFILING_BUILD ${DEFS:-}"
/opt/rocm/bin/hipcc $F -mllvm -amdgpu-kernarg-preload-count=14 -mllvm -amdgpu-sched-strategy=max-ilp -I../include -Icsrc -c csrc/mdl_kernels.hip -o $D/k.o &
for f in mdl_engine mdl_rollout mdl_greedy; do /opt/rocm/bin/hipcc $F -I../include -Icsrc -c csrc/$f.hip -o $D/$f.o & done
wait
/opt/rocm/bin/hipcc $F -shared -o build/ab/libmdl_$N.so $D/k.o $D/mdl_engine.o $D/mdl_rollout.o $D/mdl_greedy.o
ls -la build/ab/libmdl_$N.so
