#!/bin/bash
# int2 dequantization with one v_and_or_b32 per crumb pair: parity, the int2 decode shapes, the Mistral token
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_mid_gpu.py tests/test_gemm2_gpu.py tests/test_capi_fused_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_andor.log 2>&1 || { tail -30 gpurun_out/pytest_andor.log; exit 1; }
tail -1 gpurun_out/pytest_andor.log
SWEEP_BITS=2 SWEEP_GROUP=64 timeout -k 10 300 python -u tools/gemv_sweep.py --shapes o,gate_up,lm_head base > gpurun_out/int2_andor.txt 2>&1 || exit 1
grep -v "amdgpu.ids\|Radeon\|^\s*$" gpurun_out/int2_andor.txt
for r in 1 2; do timeout -k 10 200 python -u tools/mistral_decode.py mistral 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['tokens_per_s'], d['per_op_per_shape_us'])" || exit 1; done
