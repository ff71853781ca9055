cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/int2
export SWEEP_BITS=2 SWEEP_GROUP=64
timeout -k 10 300 python -u -m pytest tests/test_model_shapes_gpu.py tests/test_gpu_parity.py tests/test_chain_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread -k "mistral or int2 or S2 or chain" > gpurun_out/int2/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/int2/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/gemv_sweep.py base > gpurun_out/int2/sweep_new.txt 2>&1 || exit $?
NAD_LIB_PATH=$PWD/neural_amd/libneural_amd_xi2old.so timeout -k 10 200 python tools/gemv_sweep.py base > gpurun_out/int2/sweep_old.txt 2>&1 || exit $?
grep -v amdgpu gpurun_out/int2/sweep_new.txt | tail -7; grep -v amdgpu gpurun_out/int2/sweep_old.txt | tail -7
timeout -k 10 200 python tools/mistral_decode.py > gpurun_out/int2/mistral_new.json 2>&1 || exit $?
NAD_LIB_PATH=$PWD/neural_amd/libneural_amd_xi2old.so timeout -k 10 200 python tools/mistral_decode.py > gpurun_out/int2/mistral_old.json 2>&1 || exit $?
tail -1 gpurun_out/int2/mistral_new.json; tail -1 gpurun_out/int2/mistral_old.json
export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_SMEM" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  for v in new old; do
    if [ $v = old ]; then export NAD_LIB_PATH=$PWD/neural_amd/libneural_amd_xi2old.so; else unset NAD_LIB_PATH; fi
    timeout -s KILL 90 rocprofv3 --pmc $set -d gpurun_out/int2/pmc_${v}_$i -o run --output-format csv -- python tools/gemv_sweep.py --shapes lm_head,o --reps 8 base > gpurun_out/int2/pmc_${v}_$i.log 2>&1 || { echo "pmc pass $v $i failed"; exit 1; }
  done
done
unset NAD_LIB_PATH
echo pmc done
