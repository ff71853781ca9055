#!/bin/bash
# int2 g64 decode GEMV: register stages per wave (NAD_GEMV_NST) on the Llama shapes and the Mistral decode token
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SWEEP_BITS=2 SWEEP_GROUP=64 timeout -k 10 300 python -u tools/gemv_sweep.py --shapes o,gate_up,lm_head base NAD_GEMV_NST=2 NAD_GEMV_NST=3 NAD_GEMV_NST=4 > gpurun_out/int2_nst.txt 2>&1; rc=$?
grep -v "^\s*$" gpurun_out/int2_nst.txt | tail -30; exit $rc
