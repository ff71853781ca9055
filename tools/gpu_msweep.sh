cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm2_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "mid_m or parity" > gpurun_out/pytest_mid.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_mid.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/m_sweep.py > gpurun_out/msweep.txt 2>&1; rc=$?; cat gpurun_out/msweep.txt; exit $rc
