#!/bin/bash
# gemm4 at groups of 64: scale fold (NAD_GEMM4_FOLD64=1) vs group-end fp32 scaling, parity then sweep; Mistral prefill.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm2_gpu.py -q -x -k "fold or gemm4" --timeout 200 --timeout-method thread > gpurun_out/fold64_tests.log 2>&1; rc=$?
tail -3 gpurun_out/fold64_tests.log; [ $rc -eq 0 ] || exit $rc
for F in 0 1; do
  for spec in "4 " "4 --asym" "2 " "2 --asym"; do
    set -- $spec
    echo "## NAD_GEMM4_FOLD64=$F bits $1 g64 $2"
    NAD_GEMM4_FOLD64=$F timeout -k 10 200 python -u tools/gemm_sweep.py --m 2048 --act fp16 --kernels 4 --shapes o,gate,down --bits $1 --group 64 $2 2>&1 | grep -v amdgpu || exit 5
  done
done
