#!/bin/bash
# Same-box A/B of builder variants on configs 3 and 3b (scripts/exp/ab_obs.sh per config), the
# variants interleaved REPS times.  VARIANTS: "main" (the in-tree libmdl.so) and names of
# marl-delivery_amd/build/ab/libmdl_<name>.so builds.
set -u
for C in ${CONFIGS:-3 3b}; do
  CONFIG=$C REPS=${REPS:-3} VARIANTS="${VARIANTS:-base main}" bash scripts/exp/ab_obs.sh || exit $?
done
