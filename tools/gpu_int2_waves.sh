#!/bin/bash
# int2 g64 decode GEMV: waves per workgroup (NAD_GEMV_WAVES) and grid (NAD_GEMV_GRID) on O / gate_up (development tool)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SWEEP_BITS=2 SWEEP_GROUP=64 timeout -k 10 300 python -u tools/gemv_sweep.py --shapes o,gate_up base NAD_GEMV_WAVES=8 NAD_GEMV_WAVES=12 NAD_GEMV_GRID=128 NAD_GEMV_GRID=192 > gpurun_out/int2_waves.txt 2>&1; rc=$?
SWEEP_BITS=4 SWEEP_GROUP=128 timeout -k 10 300 python -u tools/gemv_sweep.py --shapes o base NAD_GEMV_WAVES=8 >> gpurun_out/int2_waves.txt 2>&1 || rc=$?
grep -v "^\s*$" gpurun_out/int2_waves.txt | grep -v "amdgpu.ids\|Radeon" | tail -30; exit $rc
