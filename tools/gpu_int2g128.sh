#!/bin/bash
# gemm4 int2 / int8 at groups of 128: unfolded (the default), unfolded + wave stagger, scale fold on every block size
# (NAD_GEMM4_FOLD_ALL=1, which also turns the int2 stagger on).  M = 2048, fp16 A.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for run in 1 2; do
  for spec in "2" "8"; do
    for cfg in "NAD_GEMM4_FOLD_ALL=0 NAD_GEMM4_STAGGER2=0" "NAD_GEMM4_FOLD_ALL=0 NAD_GEMM4_STAGGER2=1" "NAD_GEMM4_FOLD_ALL=1 NAD_GEMM4_STAGGER2=0"; do
      echo "## run $run bits $spec g128 $cfg"
      env $cfg timeout -k 10 200 python -u tools/gemm_sweep.py --m 2048 --act fp16 --kernels 4s --shapes o,gate,down --bits $spec --group 128 2>&1 | grep -v amdgpu || exit 5
    done
  done
done
