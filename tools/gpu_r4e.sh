#!/bin/bash
# round-4: engine pre-dequant (NAD_ENGINE_PD): chain parity tests, then base / tree / tree PD=0 A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== chain tests"; date
timeout -k 10 300 python -u -m pytest tests/test_chain_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04e_chain_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r04e_chain_tests.log; [ $rc -ne 0 ] && exit $rc
echo "== engine A/B"; date
REPS=2 timeout -k 10 700 bash tools/ab_libs.sh NAD_ENGINE_PD=0 > gpurun_out/r04e_engine_ab.txt 2>&1; rc=$?
cat gpurun_out/r04e_engine_ab.txt; exit $rc
