#!/bin/bash
# round-4: full GPU suite with the gemm4 g128 fold on (NAD_GEMM4_FOLD_ALL=1); gemm3 prefill PMC; gemm4 g32 sweep
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== suite, FOLD_ALL=1"; date
NAD_GEMM4_FOLD_ALL=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04f_suite_foldall.log 2>&1; rc=$?
tail -3 gpurun_out/r04f_suite_foldall.log; echo "suite rc=$rc"; [ $rc -ge 124 ] && exit $rc
echo "== gemm3 PMC"; date
TAG=g3s KERN=3s SHAPES=o PM=4096 timeout -k 10 400 bash tools/pmc_prefill.sh; rc=$?; [ $rc -ge 124 ] && exit $rc
echo "== gemm4 g32 sweep"; date
for cfg in "--bits 4 --group 32" "--bits 4 --group 32 --asym" "--bits 8 --group 32"; do
  timeout -k 10 200 python tools/gemm_sweep.py --m 2048 --act fp16 --shapes o,gate,down --kernels 4s $cfg >> gpurun_out/r04f_g32_sweep.txt 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "sweep rc=$rc"; exit $rc; }
done
grep -v amdgpu.ids gpurun_out/r04f_g32_sweep.txt
echo "== done"; date
