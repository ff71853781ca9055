#!/bin/bash
# gemm7 tile height by the cost model (NAD_GEMM7_BM=0): the mid / prefill M sweep at N = 4096 and 11008, then the
# prefill GEMM parity tests (development tool)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/bm_auto.txt; : > $out
for n in 4096 11008; do
  echo "== N=$n auto" >> $out
  timeout -k 10 200 python -u tools/m_sweep.py --n $n --m 65,96,128,192,256,384,512,640,768,1024,1536,2048 --act fp16 --mb 300 2>&1 | grep "M=" >> $out || exit 1
done
cat $out
timeout -k 10 500 python -u -m pytest tests/test_gemm2_gpu.py tests/test_model_shapes_gpu.py tests/test_capi_fused_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_bm_auto.log 2>&1 || { tail -30 gpurun_out/pytest_bm_auto.log; exit 1; }
tail -2 gpurun_out/pytest_bm_auto.log
