#!/bin/bash
# gemm7 int2 asym re-check after the constant change (development tool)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm2_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm7_small_groups" > gpurun_out/pytest_g7hs2.log 2>&1 || { tail -40 gpurun_out/pytest_g7hs2.log; exit 1; }
tail -2 gpurun_out/pytest_g7hs2.log
timeout -k 10 200 python -u tools/gemm_sweep.py --m 2048,4096 --act fp16 --shapes o,gate,down --kernels 7,4j --bits 2 --group 64 --asym 2>&1 | grep -v "amdgpu.ids\|Radeon" > gpurun_out/sweep_g7hs2.txt
cat gpurun_out/sweep_g7hs2.txt
