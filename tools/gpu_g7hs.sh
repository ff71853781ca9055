#!/bin/bash
# gemm7 half-step mode (int2 / int8): parity tests, then the M = 2048 / 4096 sweep against gemm4 (development tool)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gemm2_gpu.py tests/test_gguf_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_g7hs.log 2>&1 || { tail -40 gpurun_out/pytest_g7hs.log; exit 1; }
tail -3 gpurun_out/pytest_g7hs.log
out=gpurun_out/sweep_g7hs.txt; : > $out
for cfg in "2 64" "2 64 --asym" "8 32" "8 32 --asym" "8 128"; do set -- $cfg
  timeout -k 10 200 python -u tools/gemm_sweep.py --m 2048,4096 --act fp16 --shapes o,gate,down --kernels 7,4j --bits $1 --group $2 $3 2>&1 | grep -v "amdgpu.ids\|Radeon" >> $out || exit 1
done
cat $out
