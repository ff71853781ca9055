#!/bin/bash
# round-4: gemm3 on 32x32x16 MFMAs (NAD_GEMM3_MF32): parity, then sweep vs the 16x16x32 form
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== gemm parity"; date
timeout -k 10 300 python -u -m pytest tests/test_gemm2_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "test_gemm_parity" > gpurun_out/r04g_parity.log 2>&1; rc=$?
tail -5 gpurun_out/r04g_parity.log; [ $rc -ne 0 ] && exit $rc
echo "== sweep"; date
timeout -k 10 300 python tools/gemm_sweep.py --m 2048,4096 --act fp16,fp32 --kernels 3s,3sm > gpurun_out/r04g_sweep.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r04g_sweep.txt; exit $rc
