#!/bin/bash
# SQ counters of the int2 g64 decode GEMV (gate_up, lm_head) against int4 g128 gate_up (development tool)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for cfg in "2 64 gate_up" "2 64 lm_head" "4 128 gate_up"; do set -- $cfg
  OUT=gpurun_out/pmc_int2/b$1_$3; mkdir -p $OUT; i=0
  for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
             "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_SMEM" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM"; do
    i=$((i+1))
    SWEEP_BITS=$1 SWEEP_GROUP=$2 timeout -s KILL 90 rocprofv3 --pmc $set -d $OUT/p$i -o run --output-format csv -- python tools/gemv_sweep.py --shapes $3 --reps 8 base > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  done
  echo "== bits $1 g$2 $3"; python tools/pmc_summarize.py $OUT $OUT/summary.json | grep -i "gemv"
done
