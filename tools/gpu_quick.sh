#!/bin/bash
# Short GPU iteration: GPU parity tests (optionally filtered), then the bench without the CPU baseline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-dev}
echo "== pytest -m gpu ${PYTEST_K:+-k $PYTEST_K}"
timeout -k 10 900 python -m pytest tests -m gpu -q -x ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_$TAG.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "== bench"
timeout -k 10 600 python bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err; rc=$?
cat gpurun_out/bench_$TAG.json; tail -5 gpurun_out/bench_$TAG.err; echo "bench rc=$rc"
exit $rc
