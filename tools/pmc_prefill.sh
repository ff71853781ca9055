#!/bin/bash
# SQ / TCC counter passes over one prefill GEMM shape (development tool): where do the prefill kernel's cycles go?
# Usage (GPU box): [TAG=x] [SHAPES=o] [PM=4096] [KERN=3] bash tools/pmc_prefill.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_prefill${TAG:+_$TAG}
mkdir -p "$OUT"
ARGS="--shapes ${SHAPES:-o} --m ${PM:-4096} --act fp16 --reps 4 --kernels ${KERN:-3}"
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d "$OUT/p$i" -o run --output-format csv -- python tools/gemm_sweep.py $ARGS > "$OUT/p$i.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "pass $i rc=$rc"; tail -3 "$OUT/p$i.log"
    [ $rc -ge 124 ] && exit $rc
  fi
done
python tools/pmc_summarize.py "$OUT" "$OUT/summary.json" | grep -i gemm
exit 0
