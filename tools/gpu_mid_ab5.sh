#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mid_gpu.py tests/test_gemm2_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_mid5.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_mid5.log; [ $rc -eq 0 ] || exit $rc
out=gpurun_out/mid_ab5.txt; : > $out
for mm in 17 1; do for act in fp16 fp32; do
  echo "== NAD_MID_MIN_M=$mm act $act" >> $out
  NAD_MID_MIN_M=$mm timeout -k 10 120 python -u tools/m_sweep.py --m 1,2,4,8,12,16,17,32,64 --act $act --reps 64 2>&1 | grep "M=" >> $out || exit 1
done; done
cat $out
