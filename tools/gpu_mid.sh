#!/bin/bash
# mid-M kernel: parity, then the K = N = 4096 M sweep, then per-kernel device times of the sweep under rocprofv3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-mid}
timeout -k 10 400 python -u -m pytest tests/test_mid_gpu.py ${EXTRA_TESTS} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/m_sweep.py --m ${M:-1,8,16,17,24,32,48,64,96,128,256} > gpurun_out/msweep_$TAG.txt 2>&1; rc=$?
cat gpurun_out/msweep_$TAG.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_$TAG -o ms -- python3 -u tools/m_sweep.py --m ${PM:-17,32,64} > gpurun_out/prof_$TAG.txt 2>&1; rc=$?
exit $rc
