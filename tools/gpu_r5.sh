#!/bin/bash
# Round-5 GPU iteration: parity of the selected tests, then a prefill sweep of the selected kernels.
#   PYTEST_K: -k filter for tests/test_gemm2_gpu.py etc. (TESTS: files), SWEEP: gemm_sweep args
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r5}
if [ -n "$TESTS" ]; then
  echo "== pytest $TESTS ${PYTEST_K:+-k $PYTEST_K}"
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
  tail -15 gpurun_out/pytest_$TAG.log; echo "pytest rc=$rc"
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$SWEEP" ]; then
  echo "== sweep $SWEEP"
  timeout -k 10 600 python -u tools/gemm_sweep.py $SWEEP > gpurun_out/sweep_$TAG.txt 2>&1; rc=$?
  cat gpurun_out/sweep_$TAG.txt; echo "sweep rc=$rc"
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$EXTRA" ]; then
  echo "== $EXTRA"
  timeout -k 10 600 $EXTRA > gpurun_out/extra_$TAG.txt 2>&1; rc=$?
  tail -60 gpurun_out/extra_$TAG.txt; echo "extra rc=$rc"
  exit $rc
fi
