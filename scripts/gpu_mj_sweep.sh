set -e
mkdir -p gpurun_out/sw
for g in 0 1 2 3; do
  BRA_MJ_SPLIT=$g timeout -k 10 200 python bench.py --steps 3 --warmup 1 --profile-all --no-cpu-baseline --no-check --no-secondary > gpurun_out/sw/g$g.json 2> gpurun_out/sw/g$g.err
done
