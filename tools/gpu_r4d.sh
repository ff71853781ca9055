#!/bin/bash
# round-4 session c: engine generation tickets (no end-of-launch bump): chain parity tests, then base-vs-tree A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== chain tests"; date
timeout -k 10 300 python -u -m pytest tests/test_chain_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04d_chain_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r04d_chain_tests.log; [ $rc -ne 0 ] && exit $rc
echo "== engine A/B base vs tree"; date
REPS=2 timeout -k 10 600 bash tools/ab_libs.sh > gpurun_out/r04d_engine_ab.txt 2>&1; rc=$?
cat gpurun_out/r04d_engine_ab.txt; exit $rc
