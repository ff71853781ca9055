#!/bin/bash
# gemm7 at int4 g32 / g64: parity tests, then the M = 2048 / 4096 sweep against gemm4 (development tool)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm2_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "gemm7_small_groups or gemm4_parity or scale_fold or gemm4_splitk or ffn_prefill or mid_m" > gpurun_out/pytest_g7groups.log 2>&1 || { tail -30 gpurun_out/pytest_g7groups.log; exit 1; }
tail -3 gpurun_out/pytest_g7groups.log
out=gpurun_out/sweep_g7groups.txt; : > $out
for g in 32 64; do for a in "" "--asym"; do
  timeout -k 10 200 python -u tools/gemm_sweep.py --m 2048,4096 --act fp16 --shapes o,gate,down --kernels 7,4j --group $g $a 2>&1 | sed "s/^/g$g$a /" >> $out || exit 1
done; done
cat $out
