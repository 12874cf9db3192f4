# Round-2 GPU session: parity tests, stress, bench, profiled bench, one-step kernel trace.
# usage: O=gpurun_out/<tag> bash scripts/gpu_r2.sh   (TESTS=0 skips pytest, TRACE=0 skips the trace)
set -e
O=${O:-gpurun_out/r2}; mkdir -p $O
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  timeout -k 10 300 python -u scripts/stress_bwt.py ${STRESS:-6} > $O/stress.log 2>&1
fi
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --profile-all --no-cpu-baseline ${BENCH_ARGS:-} > $O/bench_all.json 2> $O/bench_all.err
if [ "${TRACE:-1}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary ${BENCH_ARGS:-} > $O/trace.log 2>&1
fi
