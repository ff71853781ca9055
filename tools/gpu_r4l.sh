#!/bin/bash
# round-4: dual-format decode QKV (NAD_GEMV_DUAL): parity; Llama per-op base vs tree (m1 body refactor); Mistral bench A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== tests"; date
timeout -k 10 400 python -u -m pytest tests/test_batch_gpu.py tests/test_model_shapes_gpu.py tests/test_gpu_parity.py tests/test_capi_fused_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04l_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r04l_tests.log; [ $rc -ne 0 ] && exit $rc
echo "== per-op A/B"; date
REPS=1 timeout -k 10 400 bash tools/ab_libs.sh > gpurun_out/r04l_ab.txt 2>&1; rc=$?
grep -v amdgpu gpurun_out/r04l_ab.txt; [ $rc -ne 0 ] && exit $rc
echo "== bench dual 0 / 1"; date
for d in 0 1; do
  NAD_GEMV_DUAL=$d timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-synthetic > gpurun_out/r04l_bench_dual$d.json 2> gpurun_out/r04l_bench_dual$d.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/r04l_bench_dual$d.json')); m=d['workloads']['mistral_7b_int2_g64_policy']; print('dual $d', d['value'], m['tokens_per_s'], m['per_op_tokens_per_s'], m['engine_cut_tokens_per_s'], m['launches_per_token'])"
done
date
