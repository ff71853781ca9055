#!/bin/bash
# Development GPU session: selected GPU tests (PYTEST_K / PYTEST_FILES), then optionally the bench.  Every GPU step has
# its own time limit; a fault / abort / timeout ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-dev}
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
echo "== pytest ${PYTEST_FILES:-tests} -m gpu ${PYTEST_K:+-k $PYTEST_K}"; date
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -q ${PYTEST_X--x} --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_$TAG.log; echo "pytest rc=$rc"; ok $rc || exit $rc
if [ "${BENCH:-0}" = 1 ]; then
  echo "== bench"; date
  timeout -k 10 600 python bench.py --steps ${STEPS:-30} --warmup 5 ${BENCH_ARGS} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err; rc=$?
  cat gpurun_out/bench_$TAG.json; tail -5 gpurun_out/bench_$TAG.err; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
echo "== done"; date
