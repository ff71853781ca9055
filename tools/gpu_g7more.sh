#!/bin/bash
# the gemm7 parity cases (development tool)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm2_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm7_small_groups" > gpurun_out/pytest_g7more.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_g7more.log; exit $rc
