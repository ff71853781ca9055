#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprof stats.  Every GPU step has its own time limit; a step that
# faults / aborts / times out ends the session (exit codes >= 124), plain test failures (1) do not.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r01}
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
echo "== pytest -m gpu"; date
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -25 gpurun_out/pytest_gpu_$TAG.log; echo "pytest rc=$rc"; ok $rc || exit $rc
if [ "${SKIP_SMOKE:-0}" = 0 ]; then
  echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1; rc=$?
  cat gpurun_out/smoke_$TAG.log | tail -5; echo "smoke rc=$rc"; ok $rc || exit $rc
fi
echo "== bench"; date
timeout -k 10 600 python bench.py --steps ${STEPS:-30} --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err; rc=$?
cat gpurun_out/bench_$TAG.json; tail -5 gpurun_out/bench_$TAG.err; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
if [ "${SKIP_PROF:-0}" = 0 ]; then
  echo "== rocprofv3 kernel stats"; date
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --prefill-steps 1 --no-cpu-baseline > gpurun_out/prof_bench_$TAG.json 2> gpurun_out/prof_$TAG.err; rc=$?
  echo "rocprof rc=$rc"; find gpurun_out/prof_$TAG -name "*stats*" | head; [ $rc -eq 0 ] || exit $rc
fi
if [ "${SKIP_PMC:-0}" = 0 ]; then
  echo "== PMC traffic passes (FETCH_SIZE, WRITE_SIZE: one counter block per run)"; date
  export TMPDIR=/tmp
  rm -rf gpurun_out/pmc_$TAG; mkdir -p gpurun_out/pmc_$TAG
  PMC_ALG_OUT=gpurun_out/pmc_$TAG/alg.json timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_$TAG/fetch -o run --output-format csv -- python tools/pmc_decode.py > gpurun_out/pmc_$TAG/fetch.log 2>&1; rc=$?
  echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_$TAG/write -o run --output-format csv -- python tools/pmc_decode.py > gpurun_out/pmc_$TAG/write.log 2>&1; rc=$?
  echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python tools/pmc_traffic.py gpurun_out/pmc_$TAG gpurun_out/pmc_traffic_$TAG.json
fi
echo "== done"; date
