# Iteration session: parity suite (fast part), job-phase timing variant, profiled benches.
set -e
O=${O:-gpurun_out/iter3}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -k "not eight_shards and not round_robin" > $O/pytest.log 2>&1
BRA_HIP_LIB=br-archive_amd/build/variants/jt/libbra_hip.so timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary --no-check > $O/bench_jt.json 2> $O/bench_jt.err
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --profile-all > $O/bench_prod.json 2> $O/bench_prod.err
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --profile-all --kind random > $O/bench_random.json 2> $O/bench_random.err
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --profile-all --kind sym16 --block-size 8388608 > $O/bench_sym16.json 2> $O/bench_sym16.err
echo done > $O/done
