#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm2_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm9" > gpurun_out/pytest_g9.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_g9.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/gemm_sweep.py --kernels 7,9 --act fp16 ${SW:-} > gpurun_out/sweep_g9.txt 2>&1; rc=$?
cat gpurun_out/sweep_g9.txt; exit $rc
