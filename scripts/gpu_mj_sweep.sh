set -e
mkdir -p gpurun_out/sw
for g in 8192:2048 1280:1280 640:640 2560:640; do
  BRA_JOBS_GRID=${g%%:*} BRA_MJOBS_GRID=${g##*:} timeout -k 10 200 python bench.py --steps 3 --warmup 1 --profile-all --no-cpu-baseline --no-check --no-secondary > gpurun_out/sw/grid_${g%%:*}_${g##*:}.json 2> gpurun_out/sw/grid.err
done
