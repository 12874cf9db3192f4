# bench under several environment settings: ENVS="A=1,B=2 C=3" (space-separated sets, comma-separated vars)
set -e
O=${O:-gpurun_out/env}; mkdir -p $O
for e in $ENVS; do
  n=$(echo $e | tr ',=' '_-')
  env $(echo $e | tr ',' ' ') timeout -k 10 200 python bench.py --steps 3 --warmup 1 --profile-all --no-cpu-baseline --no-secondary ${BENCH_ARGS:-} > $O/$n.json 2> $O/$n.err
done
