# one traced bench step: per-dispatch kernel durations (rocprofv3 --kernel-trace, csv)
set -e
mkdir -p gpurun_out/tr
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
KIND=${KIND:-text}
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tr/$KIND -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-check --no-secondary --kind $KIND > gpurun_out/tr/$KIND.log 2>&1
