#!/bin/bash
# mid-M kernel A/B over its split-K geometry: K runs (NAD_MID_KS) x in-launch combine (NAD_MID_TICKETS)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/mid_ab.txt; : > $out
for t in 1 0; do for ks in 0 1 2 8; do
  echo "== NAD_MID_TICKETS=$t NAD_MID_KS=$ks" >> $out
  NAD_MID_TICKETS=$t NAD_MID_KS=$ks timeout -k 10 120 python -u tools/m_sweep.py --m ${M:-17,32,64} --reps 64 2>&1 | grep "M=" >> $out || exit 1
done; done
cat $out
