#!/bin/bash
# M = 1 register stages per wave: xa = 3 everywhere (round-4 kernel), tree = auto (1 where a wave streams <= 2 stages,
# else 2; batch / dual 2), xf = tree with batch / dual at 3.  Llama int4 per-shape, Mistral int2 token, config-2 batch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do
  for L in xa tree xf; do
    if [ $L = tree ]; then P=$PWD/neural_amd/libneural_amd.so; else P=$PWD/neural_amd/libneural_amd_$L.so; fi
    echo "#### round $i: $L"
    if [ $L = tree ]; then C="base NAD_GEMV_NST=1 NAD_GEMV_NST=2"; else C=base; fi
    NAD_LIB_PATH=$P timeout -k 10 150 python -u tools/gemv_sweep.py $C 2>&1 | grep -E "==|base|NST" || exit 4
    NAD_LIB_PATH=$P timeout -k 10 200 python tools/mistral_decode.py mistral 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('mistral per-op tok/s', d['tokens_per_s'], d['per_op_per_shape_us'])" || exit 4
    NAD_LIB_PATH=$P timeout -k 10 200 python tools/batch_probe.py 2>/dev/null || exit 4
  done
done
