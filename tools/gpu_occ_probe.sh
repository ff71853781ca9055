#!/bin/bash
# occupancy probe (development tool): gemm7 64 / 32-row tiles with a 2-slot A ring (several workgroups per CU) against
# the 256-row default, int4 g128, M = 2048 / 4096
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/occ_probe.txt; : > $out
timeout -k 10 200 python -u -m pytest tests/test_gemm2_gpu.py -x -q --timeout 120 --timeout-method thread -k "mid_m or gemm7_small" > gpurun_out/pytest_occ.log 2>&1 || { tail -30 gpurun_out/pytest_occ.log; exit 1; }
tail -1 gpurun_out/pytest_occ.log >> $out
for bm in 256 64 32; do
  echo "== NAD_GEMM7_BM=$bm" >> $out
  NAD_GEMM7_BM=$bm timeout -k 10 200 python -u tools/gemm_sweep.py --m 2048,4096 --act fp16 --shapes o,gate,down --kernels 7 --group 128 2>&1 | grep "gemm7" >> $out || exit 1
done
cat $out
