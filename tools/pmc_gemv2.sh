#!/bin/bash
# SQ counter passes over the lm_head decode GEMV (development tool): where do the waves' cycles go?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc2
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_SMEM" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d gpurun_out/pmc2/p$i -o run --output-format csv -- python tools/gemv_sweep.py --shapes ${SHAPES:-lm_head} --reps 8 base > gpurun_out/pmc2/p$i.log 2>&1 || echo "pass $i failed"
done
python tools/pmc_summarize.py gpurun_out/pmc2 | grep -i "gemv"
