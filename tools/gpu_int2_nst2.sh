#!/bin/bash
# Mistral int2 policy decode token with the int2 ring depth forced (NAD_GEMV_NST), interleaved rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/int2_nst2.txt; : > $out
for r in 1 2; do for n in 0 3 4; do
  echo "== round $r NAD_GEMV_NST=$n" >> $out
  NAD_GEMV_NST=$n timeout -k 10 200 python -u tools/mistral_decode.py mistral 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['tokens_per_s'], d['per_op_per_shape_us'])" >> $out || exit 1
done; done
cat $out
