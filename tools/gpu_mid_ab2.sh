#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/mid_ab2.txt; : > $out
for dev in 0 1 2 3; do
  echo "== NAD_MID_DEV=$dev tickets 0" >> $out
  NAD_MID_TICKETS=0 NAD_MID_DEV=$dev timeout -k 10 120 python -u tools/m_sweep.py --m 17,64 --reps 64 2>&1 | grep "M=" >> $out || exit 1
done
NAD_MID_TICKETS=0 timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/prof_ab2 -o ms -- python3 -u tools/m_sweep.py --m 17,64 > /dev/null 2>&1 || exit 1
cat $out
