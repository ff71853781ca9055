#!/bin/bash
# round-4: gemm tests after gemm5 removal + g128 fold default; gemm4 KSW A/B; bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== gemm tests"; date
timeout -k 10 400 python -u -m pytest tests/test_gemm2_gpu.py tests/test_model_shapes_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04h_gemm_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r04h_gemm_tests.log; [ $rc -ne 0 ] && exit $rc
echo "== KSW A/B"; date
for cfg in "--bits 4 --group 32" "--bits 4 --group 32 --asym" "--bits 8 --group 32" "--bits 2 --group 64" "--bits 8 --group 128"; do
  timeout -k 10 200 python tools/gemm_sweep.py --m 2048 --act fp16 --shapes o,gate,down --kernels 4s,4sk $cfg >> gpurun_out/r04h_ksw.txt 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "sweep rc=$rc"; exit $rc; }
done
grep -v amdgpu.ids gpurun_out/r04h_ksw.txt
echo "== bench"; date
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r04h_bench.json 2> gpurun_out/r04h_bench.err; rc=$?
tail -2 gpurun_out/r04h_bench.err; echo "bench rc=$rc"; date; exit $rc
