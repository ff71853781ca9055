#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mid_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_mid4.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_mid4.log; [ $rc -eq 0 ] || exit $rc
out=gpurun_out/mid_ab4.txt; : > $out
timeout -k 10 200 python -u tools/trace_mid.py 17 48 64 > gpurun_out/trace_mid4.txt 2>&1 || exit 1
for v in "1 0" "0 0"; do set -- $v
  echo "== NAD_MID_TICKETS=$1 NAD_MID_KS=$2" >> $out
  NAD_MID_TICKETS=$1 NAD_MID_KS=$2 timeout -k 10 120 python -u tools/m_sweep.py --m ${M:-16,17,24,32,33,48,64} --reps 64 2>&1 | grep "M=" >> $out || exit 1
done
grep -A8 "rep 2" gpurun_out/trace_mid4.txt; cat $out
