# Iteration session: BWT parity tests, then bench variants (env knobs) with every slot timed.
# usage: O=gpurun_out/<tag> bash scripts/gpu_iter_r3.sh "<env1>" "<env2>" ...
set -e
O=${O:-gpurun_out/iter}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -k "not eight_shards and not round_robin" > $O/pytest.log 2>&1
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --profile-all > $O/bench_$i.json 2> $O/bench_$i.err
  echo "$e" > $O/bench_$i.env
done
echo done > $O/done
