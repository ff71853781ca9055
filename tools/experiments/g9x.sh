#!/bin/bash
# gemm9 diagnostic builds (neural_amd/libneural_amd_g9x*.so, make g9x) against the tree's library, same box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/g9x.txt; : > $out
for v in "main:" $(ls neural_amd/libneural_amd_g9x*.so | sed 's/.*g9x\(.*\)\.so/\1/' | sed 's/^/x:/'); do
  name=${v#*:}
  if [ "$name" = "" ]; then lib=""; label=main; else lib=neural_amd/libneural_amd_g9x$name.so; label=$name; fi
  echo "== $label" >> $out
  NAD_LIB_PATH=$lib timeout -k 10 120 python -u tools/gemm_sweep.py --kernels 9 --act fp16 --shapes o,gate --m ${M:-4096} 2>&1 | grep TFLOP >> $out || exit 1
done
cat $out
