#!/bin/bash
# per-kernel device times of the mid-M sweep points (rocprofv3 kernel trace + stats)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
M=${M:-17,64,256}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ms -o ms -- python3 -u tools/m_sweep.py --m $M > gpurun_out/prof_ms.txt 2>&1; rc=$?
cat gpurun_out/prof_ms.txt | grep -v "^\[" | tail -8
f=$(find gpurun_out/prof_ms -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-8 "$f" | head -20
exit $rc
