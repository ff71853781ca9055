#!/bin/bash
# Round-3 GPU iteration: engine + decode parity tests, VALU-body A/B, Mistral int2 decode on both paths.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_chain_gpu.py tests/test_gpu_parity.py -q -x -k "chain or valu or two_tile" --timeout 120 --timeout-method thread > gpurun_out/r3_tests.log 2>&1; rc=$?
tail -4 gpurun_out/r3_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/gemv_sweep.py base NAD_GEMV_VALU=1 > gpurun_out/valu_sweep4.txt 2>&1 || exit 5
SWEEP_BITS=2 SWEEP_GROUP=64 timeout -k 10 300 python -u tools/gemv_sweep.py base NAD_GEMV_VALU=1 > gpurun_out/valu_sweep2.txt 2>&1 || exit 6
grep -v amdgpu gpurun_out/valu_sweep4.txt | grep -v "^#"; grep -v amdgpu gpurun_out/valu_sweep2.txt | grep -v "^#"
for v in 0 1; do NAD_GEMV_VALU=$v timeout -k 10 300 python -u tools/mistral_decode.py mistral 2>&1 | grep tokens_per_s | sed "s/^/valu=$v /"; done > gpurun_out/r3_mistral.txt || exit 7
cat gpurun_out/r3_mistral.txt
