#!/bin/bash
# round-4: gemm4 KSW auto choice; int4 g128 on gemm4 (fold + KSW) vs gemm3; gemm tests; bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== gemm tests"; date
timeout -k 10 400 python -u -m pytest tests/test_gemm2_gpu.py tests/test_model_shapes_gpu.py tests/test_capi_fused_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04i_gemm_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r04i_gemm_tests.log; [ $rc -ne 0 ] && exit $rc
echo "== sweeps"; date
timeout -k 10 300 python tools/gemm_sweep.py --m 2048,4096 --act fp16 --kernels 4s,4sk,4sj --bits 4 --group 32 > gpurun_out/r04i_ksw_auto.txt 2>&1 || exit $?
timeout -k 10 300 python tools/gemm_sweep.py --m 2048,4096 --act fp16 --kernels 3s,4saj,4sak > gpurun_out/r04i_g128_gemm4.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r04i_ksw_auto.txt gpurun_out/r04i_g128_gemm4.txt
echo "== bench"; date
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r04i_bench.json 2> gpurun_out/r04i_bench.err; rc=$?
tail -2 gpurun_out/r04i_bench.err; echo "bench rc=$rc"; date; exit $rc
