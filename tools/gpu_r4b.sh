#!/bin/bash
# round-4 session b: bench, gemm4 KSW sweep, prefill PMC passes gemm3 vs gemm5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== bench"; date
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r04_bench_b.json 2> gpurun_out/r04_bench_b.err; rc=$?
tail -3 gpurun_out/r04_bench_b.err; echo "bench rc=$rc"; [ $rc -ge 124 ] && exit $rc
echo "== gemm4 KSW sweep"; date
for cfg in "--bits 4 --group 32" "--bits 2 --group 64" "--bits 8 --group 32" "--bits 4 --group 64"; do
  timeout -k 10 200 python tools/gemm_sweep.py --m 2048 --act fp16 --shapes o,gate,down --kernels 4s,4sk $cfg >> gpurun_out/r04_ksw_sweep.txt 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "sweep rc=$rc"; exit $rc; }
done
cat gpurun_out/r04_ksw_sweep.txt | grep -v amdgpu.ids
echo "== gemm5 sweep (no scratch)"; date
timeout -k 10 300 python tools/gemm_sweep.py --m 2048 --act fp16,fp32 --kernels 3s,5s,5 > gpurun_out/r04_gemm5_sweep_b.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r04_gemm5_sweep_b.txt; [ $rc -ge 124 ] && exit $rc
echo "== decode GEMV phase trace"; date
timeout -k 10 300 python tools/trace_skinny.py > gpurun_out/r04_trace_skinny.txt 2>&1; rc=$?
tail -30 gpurun_out/r04_trace_skinny.txt; [ $rc -ge 124 ] && exit $rc
echo "== prefill PMC gemm3 vs gemm5"; date
TAG=g3 KERN=3s SHAPES=o PM=4096 timeout -k 10 400 bash tools/pmc_prefill.sh; rc=$?; [ $rc -ge 124 ] && exit $rc
TAG=g5 KERN=5s SHAPES=o PM=4096 timeout -k 10 400 bash tools/pmc_prefill.sh; rc=$?
echo "== done rc=$rc"; date
