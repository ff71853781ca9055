mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_chain_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/chain_g4.log 2>&1; rc=$?; tail -3 gpurun_out/chain_g4.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/ab_libs.sh > gpurun_out/ab_g4.log 2>&1 || exit 4; cat gpurun_out/ab_g4.log
export TMPDIR=/tmp; T=r03d; rm -rf gpurun_out/pmc_$T; mkdir -p gpurun_out/pmc_$T
PMC_ALG_OUT=gpurun_out/pmc_$T/alg.json timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_$T/fetch -o run --output-format csv -- python tools/pmc_decode.py > gpurun_out/pmc_$T/fetch.log 2>&1 && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_$T/write -o run --output-format csv -- python tools/pmc_decode.py > gpurun_out/pmc_$T/write.log 2>&1 && python tools/pmc_traffic.py gpurun_out/pmc_$T gpurun_out/pmc_traffic_$T.json
