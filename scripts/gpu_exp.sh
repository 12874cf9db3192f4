# Experiment session: parity quick check, env sweep, measurement variants (bench kernel slots).
set -e
O=gpurun_out/exp; mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -x -q > $O/pytest.log 2>&1
i=0
IFS=';' read -ra RUNS <<< "$ENVS"
for e in "${RUNS[@]}"; do
  env $e timeout -k 10 200 python bench.py --steps 3 --warmup 1 --profile-all --no-cpu-baseline --no-secondary ${BENCH_ARGS:-} > $O/env$i.json 2> $O/env$i.err
  echo "$e" > $O/env$i.env; i=$((i+1))
done
for v in ${VARIANTS:-}; do
  BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/$v/libbra_hip.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --profile-all --no-cpu-baseline --no-secondary --no-check > $O/var_$v.json 2> $O/var_$v.err
done
