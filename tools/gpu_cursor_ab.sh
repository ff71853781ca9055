#!/bin/bash
# A/B (development tool): weight buffer resources rebuilt only when the weight changes (libneural_amd.so) vs every stripe
# form (libneural_amd_xold.so), Llama int4 and Mistral int2 decode tokens, interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_capi_fused_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_sab.log 2>&1 || { tail -30 gpurun_out/pytest_sab.log; exit 1; }
tail -1 gpurun_out/pytest_sab.log
out=gpurun_out/cursor_ab.txt; : > $out
for r in 1 2; do for lib in libneural_amd.so libneural_amd_xold.so; do for m in llama llama_asym mistral; do
  NAD_LIB_PATH=$PWD/neural_amd/$lib timeout -k 10 200 python -u tools/mistral_decode.py $m 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', '$m', d['tokens_per_s'], d['per_op_per_shape_us'])" >> $out || exit 1
done; done; done
cat $out
