#!/bin/bash
# The one GPU runner (run through gpurun): tools/gpu.sh TASK [TASK ...], each GPU step under its own time limit; a step
# that faults / aborts / times out (exit >= 124) ends the call, a plain test failure (1) does not.  Outputs go to
# gpurun_out/<task>_$TAG.*.  Tasks:
#   tests      pytest -m gpu (PYTEST_K filters)              smoke    __graft_entry__.smoke()
#   bench      bench.py (STEPS, BENCH_ARGS)                  prof     rocprofv3 --kernel-trace --stats over a short bench
#   traffic    PMC FETCH_SIZE / WRITE_SIZE passes of the decode token (tools/pmc_decode.py -> tools/pmc_traffic.py)
#   sq         SQ counter passes (PMC_SETS: ';'-separated, one run each) over PMC_CMD (default: the lm_head decode GEMV sweep),
#              summarised per kernel with derived ratios (tools/pmc_derive.py)
#   trace      decode GEMV phase trace (needs neural_amd/libneural_amd_trace.so: make -C neural_amd trace)
#   ab         library A/B on the decode shapes (LIBS="old main", ROUNDS; tools/ab_libs.sh)
#   abbench    bench.py decode tok/s per library (LIBS, ROUNDS), alternating
#   abgemm     prefill GEMM TF/s per library (LIBS, ROUNDS, GEMM_ARGS), alternating
#   sweep      tools/gemv_sweep.py over the decode shapes (SWEEP_* env)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-dev}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
for task in "$@"; do
  echo "== $task ($(date +%T))"
  case $task in
    tests)
      timeout -k 10 1100 python -u -m pytest ${PYTEST_PATHS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread \
        ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
      tail -15 gpurun_out/pytest_$TAG.log; echo "pytest rc=$rc"; ok $rc || exit $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1; rc=$?
      tail -5 gpurun_out/smoke_$TAG.log; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 600 python bench.py --steps ${STEPS:-30} --warmup 5 ${BENCH_ARGS} > gpurun_out/bench_$TAG.json \
        2> gpurun_out/bench_$TAG.err; rc=$?
      cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
        python bench.py --steps 10 --warmup 2 --prefill-steps 1 --no-cpu-baseline ${BENCH_ARGS} \
        > gpurun_out/prof_bench_$TAG.json 2> gpurun_out/prof_$TAG.err; rc=$?
      echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
      find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1 | xargs cut -d, -f1-8 | head -20 ;;
    traffic)
      rm -rf gpurun_out/pmc_$TAG; mkdir -p gpurun_out/pmc_$TAG
      PMC_ALG_OUT=gpurun_out/pmc_$TAG/alg.json timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_$TAG/fetch \
        -o run --output-format csv -- python tools/pmc_decode.py > gpurun_out/pmc_$TAG/fetch.log 2>&1 || exit 124
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_$TAG/write -o run --output-format csv -- \
        python tools/pmc_decode.py > gpurun_out/pmc_$TAG/write.log 2>&1 || exit 124
      python tools/pmc_traffic.py gpurun_out/pmc_$TAG gpurun_out/pmc_traffic_$TAG.json ;;
    sq)
      d=gpurun_out/sq_$TAG; rm -rf $d; mkdir -p $d; i=0
      SETS=${PMC_SETS:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE;SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"}
      IFS=';' read -ra SETA <<< "$SETS"
      for set in "${SETA[@]}"; do
        i=$((i+1))
        timeout -s KILL 120 rocprofv3 --pmc $set -d $d/p$i -o run --output-format csv -- \
          ${PMC_CMD:-python tools/gemv_sweep.py --shapes lm_head --reps 8 base} > $d/p$i.log 2>&1 || exit 124
      done
      python tools/pmc_summarize.py $d gpurun_out/sq_$TAG.json > gpurun_out/sq_$TAG.txt
      python tools/pmc_derive.py gpurun_out/sq_$TAG.json | tee gpurun_out/sq_derived_$TAG.txt ;;
    trace)
      timeout -k 10 300 python -u tools/gemv_sweep.py --trace ${SHAPES:+--shapes $SHAPES} base 2>&1 | grep -v amdgpu.ids \
        > gpurun_out/trace_$TAG.txt || exit 124
      tail -60 gpurun_out/trace_$TAG.txt ;;
    ab)
      TAG=ab_$TAG bash tools/ab_libs.sh || exit 124 ;;
    abbench)  # decode tok/s per library (LIBS, ROUNDS), alternating: the chained token, not one shape
      f=gpurun_out/abbench_$TAG.txt; : > $f
      for r in $(seq ${ROUNDS:-3}); do for l in ${LIBS:-main}; do
        if [ "$l" = main ]; then p=neural_amd/libneural_amd.so; else p=neural_amd/libneural_amd_x$l.so; fi
        NAD_LIB_PATH=$PWD/$p timeout -k 10 300 python bench.py --steps 30 --warmup 5 --prefill-steps 1 --no-cpu-baseline \
          --no-extra --no-synthetic > gpurun_out/abbench_$l.json 2>/dev/null || exit 124
        python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d.get('decode_eager_tokens_per_s'), d['roofline']['avg_launch_us'], d.get('prefill_tflops'))" gpurun_out/abbench_$l.json $l | tee -a $f
      done; done ;;
    abgemm)  # prefill GEMM TF/s per library (LIBS, ROUNDS, GEMM_ARGS), alternating
      f=gpurun_out/abgemm_$TAG.txt; : > $f
      for r in $(seq ${ROUNDS:-2}); do for l in ${LIBS:-main}; do
        if [ "$l" = main ]; then p=neural_amd/libneural_amd.so; else p=neural_amd/libneural_amd_x$l.so; fi
        echo "#### lib $l round $r" >> $f
        NAD_LIB_PATH=$PWD/$p timeout -k 10 300 python tools/gemm_sweep.py ${GEMM_ARGS:---m 2048,4096 --act fp16 --shapes o,gate,down --kernels 7 --reps 10} 2>&1 | grep -v amdgpu.ids >> $f || exit 124
      done; done
      cat $f ;;
    sweep)
      timeout -k 10 300 python -u tools/gemv_sweep.py ${SHAPES:+--shapes $SHAPES} base 2>&1 | grep -v amdgpu.ids \
        > gpurun_out/sweep_$TAG.txt || exit 124
      cat gpurun_out/sweep_$TAG.txt ;;
    *) echo "unknown task $task"; exit 2 ;;
  esac
done
echo "== done ($(date +%T))"
