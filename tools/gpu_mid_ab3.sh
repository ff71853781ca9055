#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/mid_ab3.txt; : > $out
timeout -k 10 200 python -u tools/trace_mid.py ${TM:-17 64} > gpurun_out/trace_mid3.txt 2>&1 || exit 1
for v in "1 0" "0 0" "1 2" "0 2" "1 8"; do set -- $v
  echo "== NAD_MID_TICKETS=$1 NAD_MID_KS=$2" >> $out
  NAD_MID_TICKETS=$1 NAD_MID_KS=$2 timeout -k 10 120 python -u tools/m_sweep.py --m ${M:-17,32,64} --reps 64 2>&1 | grep "M=" >> $out || exit 1
done
grep -A8 "rep 2" gpurun_out/trace_mid3.txt; cat $out
