#!/bin/bash
# gemm7 with scale / zero-point DMAs from the owning waves only: parity, then the sweeps of the earlier round-5 files
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm2_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm7 or splitk or mid_m or ffn" > gpurun_out/pytest_g7sw.log 2>&1 || { tail -30 gpurun_out/pytest_g7sw.log; exit 1; }
tail -2 gpurun_out/pytest_g7sw.log
out=gpurun_out/sweep_g7sw.txt; : > $out
for cfg in "4 128" "4 128 --asym" "4 32" "4 32 --asym" "8 32 --asym" "2 64 --asym" "2 64"; do set -- $cfg
  timeout -k 10 200 python -u tools/gemm_sweep.py --m 2048,4096 --act fp16 --shapes o,gate,down --kernels 7 --bits $1 --group $2 $3 2>&1 | grep -v "amdgpu.ids\|Radeon" >> $out || exit 1
done
cat $out
