mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -q -x -k "valu or two_tile" --timeout 120 --timeout-method thread > gpurun_out/valu_test.log 2>&1; rc=$?; tail -3 gpurun_out/valu_test.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/gemv_sweep.py base NAD_GEMV_VALU=1 base NAD_GEMV_VALU=1 > gpurun_out/valu_sweep4.txt 2>&1 || exit 5
SWEEP_BITS=2 SWEEP_GROUP=64 timeout -k 10 300 python -u tools/gemv_sweep.py base NAD_GEMV_VALU=1 > gpurun_out/valu_sweep2.txt 2>&1 || exit 6
for v in 0 1 0 1; do NAD_GEMV_VALU=$v timeout -k 10 200 python -u tools/mistral_decode.py mistral 2>&1 | grep tokens_per_s | sed "s/^/valu=$v /"; done > gpurun_out/valu_mistral.txt || exit 7
grep -v amdgpu gpurun_out/valu_sweep4.txt | grep -v "^#" ; grep -v amdgpu gpurun_out/valu_sweep2.txt; cut -c1-80 gpurun_out/valu_mistral.txt
