#!/bin/bash
# K-slice width of the M = 1 launches, both orders (the first config of a process runs cold): default vs
# NAD_GEMV_KS=4 on int4 g128 Llama shapes, default vs NAD_GEMV_KS=3 on int2 g64
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 250 python -u tools/gemv_sweep.py NAD_GEMV_KS=4 base NAD_GEMV_KS=4 base 2>&1 | grep -E "==|base|KS" || exit 4
SWEEP_BITS=2 SWEEP_GROUP=64 timeout -k 10 250 python -u tools/gemv_sweep.py --shapes o,gate_up,qkv,lm_head NAD_GEMV_KS=3 base NAD_GEMV_KS=3 base 2>&1 | grep -E "==|base|KS" || exit 4
