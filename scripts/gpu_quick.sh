# lane-exchange check, parity tests + one profiled bench (all kernel slots timed)
set -e
mkdir -p gpurun_out/q
hipcc --offload-arch=gfx950 -O3 -I br-archive_amd/csrc scripts/xlane_check.hip -o /tmp/xlane_check > gpurun_out/q/xlane.log 2>&1
timeout -k 10 60 /tmp/xlane_check >> gpurun_out/q/xlane.log 2>&1
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -m gpu -x -q > gpurun_out/q/pytest.log 2>&1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --profile-all --no-cpu-baseline > gpurun_out/q/bench_all.json 2> gpurun_out/q/bench_all.err
