#!/bin/bash
# two workgroups per CU for the M = 1 launches (NAD_GEMV_WPC=2), both orders; int4 g128 and int2 g64 shapes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 250 python -u tools/gemv_sweep.py NAD_GEMV_WPC=2 base NAD_GEMV_WPC=2 base 2>&1 | grep -E "==|base|WPC" || exit 4
SWEEP_BITS=2 SWEEP_GROUP=64 timeout -k 10 250 python -u tools/gemv_sweep.py --shapes o,gate_up,lm_head NAD_GEMV_WPC=2 base NAD_GEMV_WPC=2 base 2>&1 | grep -E "==|base|WPC" || exit 4
for c in NAD_GEMV_WPC=2 base NAD_GEMV_WPC=2 base; do
  if [ $c = base ]; then E=""; else E=$c; fi
  env $E timeout -k 10 200 python tools/mistral_decode.py mistral 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('$c mistral per-op tok/s', d['tokens_per_s'], d['per_op_per_shape_us'])" || exit 4
done
