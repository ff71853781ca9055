#!/bin/bash
# xt (previous build) vs tree (narrow-slice launches stage one activation slice per wave)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2; do
  for L in xt tree; do
    if [ $L = tree ]; then P=$PWD/neural_amd/libneural_amd.so; else P=$PWD/neural_amd/libneural_amd_$L.so; fi
    echo "#### round $i: $L"
    NAD_LIB_PATH=$P timeout -k 10 150 python -u tools/gemv_sweep.py base 2>&1 | grep -E "==|base" || exit 4
    NAD_LIB_PATH=$P timeout -k 10 200 python tools/mistral_decode.py mistral 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('mistral per-op tok/s', d['tokens_per_s'], d['per_op_per_shape_us'])" || exit 4
    NAD_LIB_PATH=$P timeout -k 10 200 python tools/msmall_probe.py 2>/dev/null || exit 4
  done
done
