#!/bin/bash
# round-4: batched M = 1 GEMV (nad_batch_*): parity, then bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== batch tests"; date
timeout -k 10 300 python -u -m pytest tests/test_batch_gpu.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04k_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r04k_tests.log; [ $rc -ne 0 ] && exit $rc
echo "== bench"; date
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r04k_bench.json 2> gpurun_out/r04k_bench.err; rc=$?
tail -2 gpurun_out/r04k_bench.err; echo "bench rc=$rc"
python -c "import json; d=json.load(open('gpurun_out/r04k_bench.json')); s=d['synthetic']; print(json.dumps(s['config2_m1_batched'])); print(json.dumps(s['config2_m1_batched_engine'])); print(d['value'], d['prefill_tflops'])"
date; exit $rc
