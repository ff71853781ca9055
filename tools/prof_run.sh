cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_g2 -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --prefill-steps 2 --no-cpu-baseline > gpurun_out/prof_g2_bench.json 2>/dev/null
find gpurun_out/prof_g2 -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-8 | head -20
