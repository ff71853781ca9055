#!/bin/bash
# M = 1 register ring depth A/B: xa = 3 stages everywhere (the round-4 kernel), tree = int2 1-tile slices 6 stages,
# xb = int2 6 + int4 6.  Mistral int2-policy decode token (per-op) and int2 / int4 per-shape sweeps, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do
  for L in xc xd xe; do
    if [ $L = tree ]; then P=$PWD/neural_amd/libneural_amd.so; else P=$PWD/neural_amd/libneural_amd_$L.so; fi
    echo "#### round $i: $L"
    NAD_LIB_PATH=$P timeout -k 10 200 python tools/mistral_decode.py mistral 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('mistral per-op tok/s', d['tokens_per_s'], d['per_op_per_shape_us'])" || exit 4
    NAD_LIB_PATH=$P SWEEP_BITS=2 SWEEP_GROUP=64 timeout -k 10 150 python -u tools/gemv_sweep.py --shapes o,gate_up,qkv base 2>&1 | grep -E "==|base" || exit 4
    NAD_LIB_PATH=$P timeout -k 10 150 python -u tools/gemv_sweep.py base 2>&1 | grep -E "==|base" || exit 4
  done
done
