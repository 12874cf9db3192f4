set -e
mkdir -p gpurun_out/sw
for w in 2 4 8; do
  BRA_MJ_WAVES=$w timeout -k 10 200 python bench.py --steps 3 --warmup 1 --profile-all --no-cpu-baseline --no-check > gpurun_out/sw/w$w.json 2> gpurun_out/sw/w$w.err
done
