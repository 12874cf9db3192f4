# Parity (fast part + determinism), repeat-encode stress, benches of the three workloads.
set -e
O=${O:-gpurun_out/iter5}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -k "not eight_shards" > $O/pytest.log 2>&1
timeout -k 10 300 python -u scripts/stress_repeat.py 4 > $O/stress.log 2>&1
BQ="python bench.py --no-cpu-baseline --no-secondary --profile-all"
timeout -k 10 200 $BQ --steps 5 --warmup 2 > $O/bench_prod.json 2> $O/bench_prod.err
timeout -k 10 200 $BQ --steps 3 --warmup 1 --kind random > $O/bench_random.json 2> $O/bench_random.err
timeout -k 10 200 $BQ --steps 3 --warmup 1 --kind sym16 --block-size 8388608 > $O/bench_sym16.json 2> $O/bench_sym16.err
echo done > $O/done
