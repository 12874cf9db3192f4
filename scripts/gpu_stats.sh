# rocprofv3 kernel stats of a short bench run: $O/tr/run_kernel_stats.csv
set -e
O=${O:-gpurun_out/st}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --no-check ${BENCH_ARGS:-} > $O/trace.log 2>&1
