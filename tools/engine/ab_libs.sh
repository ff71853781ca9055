#!/bin/bash
# Same-box A/B of engine builds: neural_amd/libneural_amd_base.so (a baseline build, made by hand) vs the tree's
# library, and the tree's library with each extra environment given as arguments (e.g. NAD_ENGINE_X8=1).
# Runs tools/engine_ab.py (cut / whole / indep tokens per second) for each, alternating, REPS times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in $(seq ${REPS:-2}); do
  for L in base new "$@"; do
    echo "== $L"
    if [ "$L" = base ]; then
      NAD_LIB_PATH=$PWD/neural_amd/libneural_amd_base.so ENGINE_AB_INDEP=1 timeout -k 10 200 python -u tools/engine_ab.py 2>&1 | grep -v amdgpu.ids || exit 4
    elif [ "$L" = new ]; then
      ENGINE_AB_INDEP=1 timeout -k 10 200 python -u tools/engine_ab.py 2>&1 | grep -v amdgpu.ids || exit 4
    else
      env "$L" ENGINE_AB_INDEP=1 timeout -k 10 200 python -u tools/engine_ab.py 2>&1 | grep -v amdgpu.ids || exit 4
    fi
  done
done
