#!/bin/bash
# PMC passes over the O-shape decode GEMV and the same-size pure read (tools/hbm_probe one): development tool.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
i=0
for set in "TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCP_UTCL1_REQUEST" "TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ" "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU" "TCP_PENDING_STALL_CYCLES TCP_TCP_TA_DATA_STALL_CYCLES TA_BUSY_avr"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $set -d gpurun_out/pmc/g$i -o run --output-format csv -- python tools/gemv_sweep.py --shapes ${SHAPES:-o} --reps 8 base > /dev/null 2>&1 || echo "gemv pass $i failed"
  timeout -k 10 200 rocprofv3 --pmc $set -d gpurun_out/pmc/p$i -o run --output-format csv -- ./tools/hbm_probe one > /dev/null 2>&1 || echo "probe pass $i failed"
done
echo done
