#!/bin/bash
# A/B of GEMV library builds on the decode shapes: LIBS="old new" (neural_amd/libneural_amd_x<name>.so, "main" = the
# product library), alternating ROUNDS times; gemv_sweep.py prints device time per launch (graph replay, cold weights).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/${TAG:-ab}.txt; : > $out
for r in $(seq ${ROUNDS:-2}); do
  for l in ${LIBS:-main}; do
    if [ "$l" = main ]; then p=neural_amd/libneural_amd.so; else p=neural_amd/libneural_amd_x$l.so; fi
    echo "#### lib $l round $r" >> $out
    NAD_LIB_PATH=$PWD/$p timeout -k 10 240 python -u tools/gemv_sweep.py ${SHAPES:+--shapes $SHAPES} base 2>&1 | grep -v amdgpu.ids >> $out || exit 1
  done
done
python - "$out" <<'PY'
import re, sys, collections
lib = None; shape = None; res = collections.defaultdict(list)
for line in open(sys.argv[1]):
    m = re.match(r"#### lib (\S+)", line)
    if m: lib = m.group(1); continue
    m = re.match(r"== (\S+):", line)
    if m: shape = m.group(1); continue
    m = re.match(r"\s+base\s+([\d.]+) us", line)
    if m: res[(shape, lib)].append(float(m.group(1)))
shapes = list(dict.fromkeys(s for s, _ in res)); libs = list(dict.fromkeys(l for _, l in res))
print("shape     " + "".join(f"{l:>22s}" for l in libs))
for s in shapes:
    print(f"{s:10s}" + "".join(f"{' / '.join('%.2f' % v for v in res[(s, l)]):>22s}" for l in libs))
PY
