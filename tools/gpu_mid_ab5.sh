#!/bin/bash
# mid-M kernel below 17 rows (NAD_MID_MIN_M=1) against the stripe-stream GEMV, fp16 and fp32 activations
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/mid_ab5.txt; : > $out
for n in 4096 11008; do for mm in 17 1; do for act in fp16 fp32; do
  echo "== N=$n NAD_MID_MIN_M=$mm act $act" >> $out
  NAD_MID_MIN_M=$mm timeout -k 10 120 python -u tools/m_sweep.py --n $n --m 2,4,8,12,16 --act $act --reps 64 2>&1 | grep "M=" >> $out || exit 1
done; done; done
cat $out
