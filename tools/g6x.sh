#!/bin/bash
# gemm6/7 experiment builds (neural_amd/libneural_amd_g6*.so, make g6x) against the tree's library, same box
cd $GRAFT_REPO_ROOT
for L in "" $LIBS; do
  echo "== lib ${L:-main}"
  if [ -n "$L" ]; then export NAD_LIB_PATH=$PWD/neural_amd/libneural_amd_$L.so; else unset NAD_LIB_PATH; fi
  timeout -k 10 120 python -u tools/gemm_sweep.py --m ${PM:-2048,4096} --act fp16 --shapes ${SHAPES:-o} --kernels ${KERN:-6} --reps 20 2>&1 | grep gemm || exit 3
done
