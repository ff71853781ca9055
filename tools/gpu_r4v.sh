#!/bin/bash
# long K on 2-tile slices (NAD_GEMV_LK=1) vs the 4-tile split, both orders: Llama down (int4 g128 K = 11008), Mistral
# int2 policy token (its down: int4 g64 K = 14336); then the GEMV parity files with LK=1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 200 python -u tools/gemv_sweep.py --shapes down NAD_GEMV_LK=1 base NAD_GEMV_LK=1 base 2>&1 | grep -E "==|base|LK" || exit 4
SWEEP_GROUP=64 timeout -k 10 200 python -u tools/gemv_sweep.py --shapes down NAD_GEMV_LK=1 base NAD_GEMV_LK=1 base 2>&1 | grep -E "==|base|LK" || exit 4
for c in NAD_GEMV_LK=1 base NAD_GEMV_LK=1 base; do
  if [ $c = base ]; then E=""; else E=$c; fi
  env $E timeout -k 10 200 python tools/mistral_decode.py mistral 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('$c mistral per-op tok/s', d['tokens_per_s'], d['per_op_per_shape_us'])" || exit 4
done
NAD_GEMV_LK=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_model_shapes_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pt_lk.log 2>&1; rc=$?; tail -3 gpurun_out/pt_lk.log; exit $rc
