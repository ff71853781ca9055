#!/bin/bash
# the whole GPU suite (as the driver runs it), then smoke()
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-full}
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
tail -25 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -3
