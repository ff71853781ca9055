#!/bin/bash
# round-4: Mistral int2 policy decode per-shape times (final build) + SQ counters of the int2 M = 1 kernel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/mistral_decode.py mistral > gpurun_out/r04m_mistral.json 2> gpurun_out/r04m_mistral.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/r04m_mistral.json')); print({k: d[k] for k in ('tokens_per_s','decode_path','launches_per_token','per_op_per_shape_us')}, d['roofline'])"
SWEEP_BITS=2 SWEEP_GROUP=64 timeout -k 10 200 python tools/gemv_sweep.py --shapes o,gate_up,qkv base > gpurun_out/r04m_int2_sweep.txt 2>&1 || exit $?
grep -v amdgpu gpurun_out/r04m_int2_sweep.txt
rm -rf gpurun_out/pmc2
SWEEP_BITS=2 SWEEP_GROUP=64 SHAPES=o timeout -k 10 400 bash tools/pmc_gemv2.sh > gpurun_out/r04m_pmc_int2.txt 2>&1; rc=$?
cat gpurun_out/r04m_pmc_int2.txt; exit $rc
