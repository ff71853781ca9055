# gemm4 development sweep: gemm4 vs the generic kernel for the configurations gemm4 covers.
# G4CFGS: comma-separated "bits group [--asym]" entries
set -e
IFS=, read -ra CFGS <<< "${G4CFGS:-4 32,4 64 --asym,2 64,2 64 --asym,2 128}"
for cfg in "${CFGS[@]}"; do
  set -- $cfg
  timeout -k 10 150 python tools/gemm_sweep.py --m ${G4M:-2048} --act ${G4ACT:-fp16,fp32} --shapes o,gate,down \
    --kernels ${G4K:-4,0} --bits $1 --group $2 $3 --reps 10
done
