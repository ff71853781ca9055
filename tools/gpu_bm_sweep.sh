#!/bin/bash
# gemm7 tile height for 96 <= M <= 512 (NAD_GEMM7_BM: 0 auto, 64, 128, 256), K = N = 4096 int4 g128 (development tool)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/bm_sweep.txt; : > $out
for bm in 0 64 128 256; do
  echo "== NAD_GEMM7_BM=$bm" >> $out
  NAD_GEMM7_BM=$bm timeout -k 10 200 python -u tools/m_sweep.py --m 65,96,128,192,256,384,512 --act fp16 2>&1 | grep "M=" >> $out || exit 1
done
cat $out
