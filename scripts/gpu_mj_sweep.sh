set -e
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -m gpu -x -q > gpurun_out/b6_pytest.log 2>&1
for w in 4 2 8; do
  BRA_MJ_WAVES=$w timeout -k 10 200 python bench.py --steps 3 --warmup 1 --profile-all --no-cpu-baseline > gpurun_out/b6_bench_w$w.json 2> gpurun_out/b6_bench_w$w.err
done
