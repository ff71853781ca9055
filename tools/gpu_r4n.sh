#!/bin/bash
# Same-box A/B of the M = 1 GEMV: base library (neural_amd/libneural_amd_base.so) vs the tree's (branch-free stage
# loads), each with the default and NAD_GEMV_PRE=3 (whole register ring issued before the activation staging).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do
  echo "#### round $i: base library"
  NAD_LIB_PATH=$PWD/neural_amd/libneural_amd_base.so timeout -k 10 150 python -u tools/gemv_sweep.py base NAD_GEMV_PRE=3 2>&1 | grep -v amdgpu.ids || exit 4
  echo "#### round $i: tree library"
  timeout -k 10 150 python -u tools/gemv_sweep.py base NAD_GEMV_PRE=3 2>&1 | grep -v amdgpu.ids || exit 4
done
echo "#### traced (tree sources, phase-trace build): default vs NAD_GEMV_PRE=3"
NAD_LIB_PATH=$PWD/neural_amd/libneural_amd_tr.so timeout -k 10 150 python -u tools/gemv_sweep.py --trace --shapes qkv,o,gate_up,down base NAD_GEMV_PRE=3 2>&1 | grep -v amdgpu.ids || exit 4
