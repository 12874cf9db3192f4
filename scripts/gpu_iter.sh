# iteration loop: gpu parity, BWT stress, a bench line, a traced step
set -e
mkdir -p gpurun_out/it
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/it/pytest.log 2>&1
timeout -k 10 200 python -u scripts/stress_bwt.py ${STRESS:-3} > gpurun_out/it/stress.log 2>&1
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > gpurun_out/it/bench.json 2> gpurun_out/it/bench.err
if [ -n "${ALT_ENV:-}" ]; then env $ALT_ENV timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > gpurun_out/it/bench_alt.json 2> gpurun_out/it/bench_alt.err; fi
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/it/tr -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-check --no-secondary > gpurun_out/it/tr.log 2>&1
