# bench (kernel slot timing) under several environment settings: ENVS="A=1 B=2;C=3" (';' separates runs)
set -e
mkdir -p gpurun_out/env
i=0
IFS=';' read -ra RUNS <<< "$ENVS"
for e in "${RUNS[@]}"; do
  env $e timeout -k 10 200 python bench.py --steps 3 --warmup 1 --profile-all --no-cpu-baseline --no-secondary ${BENCH_ARGS:-} > gpurun_out/env/run$i.json 2> gpurun_out/env/run$i.err
  echo "$e" > gpurun_out/env/run$i.env
  i=$((i+1))
done
