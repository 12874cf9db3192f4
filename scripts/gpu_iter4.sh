# Iteration session: parity (fast part), job timing and benches of the product build and of variants.
# usage: O=gpurun_out/<tag> bash scripts/gpu_iter4.sh "<variant> ..."   (variants under build/variants)
set -e
O=${O:-gpurun_out/iter4}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -k "not eight_shards and not round_robin" > $O/pytest.log 2>&1
BQ="python bench.py --no-cpu-baseline --no-secondary --profile-all"
timeout -k 10 200 $BQ --steps 5 --warmup 2 > $O/bench_prod.json 2> $O/bench_prod.err
timeout -k 10 200 $BQ --steps 3 --warmup 1 --kind random > $O/bench_random.json 2> $O/bench_random.err
timeout -k 10 200 $BQ --steps 3 --warmup 1 --kind sym16 --block-size 8388608 > $O/bench_sym16.json 2> $O/bench_sym16.err
for v in $1; do
  BRA_HIP_LIB=br-archive_amd/build/variants/$v/libbra_hip.so timeout -k 10 200 $BQ --steps 5 --warmup 2 > $O/bench_$v.json 2> $O/bench_$v.err
done
echo done > $O/done
