#!/bin/bash
# gemm7 tile height, second pass: 32 vs 64 rows at M <= 256, 128 vs 256 at M >= 640, N = 4096 and 11008 (development tool)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/bm_sweep2.txt; : > $out
for n in 4096 11008; do
for bm in 32 64 128 256; do
  case $bm in 32|64) ms=65,96,128,192,256 ;; *) ms=384,512,640,768,1024,1536 ;; esac
  [ $bm = 128 ] && ms=128,192,256,384,512,640,768,1024,1536
  echo "== N=$n NAD_GEMM7_BM=$bm" >> $out
  NAD_GEMM7_BM=$bm timeout -k 10 200 python -u tools/m_sweep.py --n $n --m $ms --act fp16 --mb 300 2>&1 | grep "M=" >> $out || exit 1
done; done
cat $out
