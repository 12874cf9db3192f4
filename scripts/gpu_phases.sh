set -e
mkdir -p gpurun_out/ph
timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-check > gpurun_out/ph/bench.json 2> gpurun_out/ph/bench.err
