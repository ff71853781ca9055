#!/bin/bash
# decode GEMV phase trace of the current build (libneural_amd_trace.so): Llama int4 g128 shapes and Mistral int2 g64
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/trace_m1.txt; : > $out
timeout -k 10 300 python -u tools/gemv_sweep.py --trace base >> $out 2>&1 || exit 1
SWEEP_BITS=2 SWEEP_GROUP=64 timeout -k 10 300 python -u tools/gemv_sweep.py --trace --shapes o,gate_up,lm_head base >> $out 2>&1 || exit 1
grep -v "amdgpu.ids" $out | tail -60
