#!/bin/bash
# general (M <= 16) GEMV kernel stage count: auto (1 where a wave streams <= 2 stages) vs forced 3 (the previous kernel)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2; do
  timeout -k 10 200 python tools/msmall_probe.py 2>/dev/null || exit 4
  NAD_GEMV_NST=3 timeout -k 10 200 python tools/msmall_probe.py 2>/dev/null || exit 4
done
