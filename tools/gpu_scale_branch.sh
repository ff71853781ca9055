#!/bin/bash
# M = 1 GEMV with the stage's group scales converted once per stage behind a uniform branch: parity, int2 / int4 decode
# shapes, the Mistral and Llama tokens (development tool)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_capi_fused_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_sb.log 2>&1 || { tail -30 gpurun_out/pytest_sb.log; exit 1; }
tail -1 gpurun_out/pytest_sb.log
SWEEP_BITS=2 SWEEP_GROUP=64 timeout -k 10 300 python -u tools/gemv_sweep.py --shapes o,gate_up,lm_head base > gpurun_out/sb_int2.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/gemv_sweep.py base > gpurun_out/sb_int4.txt 2>&1 || exit 1
grep -v "amdgpu.ids\|Radeon\|^\s*$" gpurun_out/sb_int2.txt gpurun_out/sb_int4.txt
for r in 1 2; do timeout -k 10 200 python -u tools/mistral_decode.py mistral 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('mistral', d['tokens_per_s'], d['per_op_per_shape_us'])" || exit 1; done
