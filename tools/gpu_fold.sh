#!/bin/bash
# gemm4 g32 scale folding: parity (gemm / split-K / GGUF / model-shape / int8 tests), then the g32 sweep with it (default)
# and without it (NAD_GEMM4_FOLD=0), alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm2_gpu.py tests/test_gguf_gpu.py tests/test_model_shapes_gpu.py tests/test_int8_compute_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/fold_tests.log 2>&1; rc=$?
tail -4 gpurun_out/fold_tests.log; [ $rc -eq 0 ] || exit $rc
for F in 1 0; do
  for spec in "4 " "4 --asym" "8 " "8 --asym"; do
    set -- $spec
    echo "## NAD_GEMM4_FOLD=$F bits $1 g32 $2"
    NAD_GEMM4_FOLD=$F timeout -k 10 200 python -u tools/gemm_sweep.py --m 2048 --act fp16 --kernels 4 --shapes o,gate,down --bits $1 --group 32 $2 2>&1 | grep -v amdgpu || exit 5
  done
done
