#!/bin/bash
# bench.py A/B over one runtime knob (development tool): ENVVAR=name, VALUES="a b", ROUNDS; alternating, one line per run
# (knob value, decode tok/s, eager tok/s, prefill TF/s) -> gpurun_out/abenv_$TAG.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; f=gpurun_out/abenv_${TAG:-dev}.txt; : > $f
for r in $(seq ${ROUNDS:-3}); do for v in ${VALUES:-0 1}; do
  env $ENVVAR=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --prefill-steps 5 --no-cpu-baseline --no-extra \
    --no-synthetic > gpurun_out/abenv_run.json 2>/dev/null || exit 124
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d.get('decode_eager_tokens_per_s'), d.get('prefill_tflops'))" gpurun_out/abenv_run.json "$ENVVAR=$v" | tee -a $f
done; done
