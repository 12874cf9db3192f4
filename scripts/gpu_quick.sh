# parity tests + one profiled bench (all kernel slots timed) [+ phase profile build if PHASES=1]
set -e
mkdir -p gpurun_out/q
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -m gpu -x -q > gpurun_out/q/pytest.log 2>&1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --profile-all --no-cpu-baseline > gpurun_out/q/bench_all.json 2> gpurun_out/q/bench_all.err
if [ "${PHASES:-0}" = 1 ]; then
  make -C br-archive_amd -B -j16 EXTRA=-DBRA_PHASES > gpurun_out/q/phases_build.log 2>&1
  timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-check > gpurun_out/q/phases.json 2> gpurun_out/q/phases.err
fi
if [ -n "${EXTRA_KIND:-}" ]; then
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --profile-all --no-cpu-baseline --kind $EXTRA_KIND > gpurun_out/q/bench_$EXTRA_KIND.json 2> gpurun_out/q/bench_$EXTRA_KIND.err
fi
