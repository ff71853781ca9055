#!/bin/bash
# round-4: int4 g128 on gemm4 (fold + KSW) vs gemm3; int8 g128 folded KSW A/B; CU count
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
python -c "import torch; print('CUs', torch.cuda.get_device_properties(0).multi_processor_count)"
timeout -k 10 300 python tools/gemm_sweep.py --m 2048,4096 --act fp16,fp32 --kernels 3s,4saj,4sak > gpurun_out/r04j_g128_gemm4.txt 2>&1 || exit $?
timeout -k 10 300 python tools/gemm_sweep.py --m 2048 --act fp16 --shapes o,gate,down --kernels 4s,4sk --bits 8 --group 128 > gpurun_out/r04j_i8g128.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r04j_g128_gemm4.txt gpurun_out/r04j_i8g128.txt
