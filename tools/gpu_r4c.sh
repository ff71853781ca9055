#!/bin/bash
# round-4 session c: M = 1 GEMV with every weight stage issued before the activation staging (NAD_GEMV_PRE), then bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== gemv sweep: base lib, tree lib PRE=1 / PRE=3"; date
for r in 1 2; do
  NAD_LIB_PATH=$PWD/neural_amd/libneural_amd_base.so timeout -k 10 200 python -u tools/gemv_sweep.py base >> gpurun_out/r04c_gemv_pre.txt 2>&1 || exit $?
  timeout -k 10 200 python -u tools/gemv_sweep.py NAD_GEMV_PRE=1 NAD_GEMV_PRE=3 >> gpurun_out/r04c_gemv_pre.txt 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/r04c_gemv_pre.txt
echo "== bench"; date
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r04c_bench.json 2> gpurun_out/r04c_bench.err; rc=$?
tail -3 gpurun_out/r04c_bench.err; echo "bench rc=$rc"; date
exit $rc
