#!/bin/bash
# round 4, call a: the chunk-stream tests with localisation, the stress loop; then the local-MSD
# variant (build/variants/local): full-size parity and an A/B bench line against the in-tree library
set -o pipefail
mkdir -p gpurun_out/r4a
ok() { [ $1 -le 1 ] || exit $1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_chunks.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4a/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -3 gpurun_out/r4a/pytest.log; ok $rc
timeout -k 10 400 python -u scripts/stress_chunks.py 10 > gpurun_out/r4a/stress.log 2>&1
rc=$?; echo "stress rc $rc"; cat gpurun_out/r4a/stress.log; ok $rc
timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4a/bench_base.json 2> gpurun_out/r4a/bench_base.err
rc=$?; echo "bench base rc $rc"; tail -c 600 gpurun_out/r4a/bench_base.json; ok $rc
export BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/local/libbra_hip.so
BRA_LEVEL_STATS=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary > gpurun_out/r4a/bench_local_stats.json 2> gpurun_out/r4a/level_stats_local.txt
rc=$?; echo "level stats rc $rc"; head -30 gpurun_out/r4a/level_stats_local.txt; ok $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread -k "every_block" > gpurun_out/r4a/pytest_local_full.log 2>&1
rc=$?; echo "local fullsize rc $rc"; tail -12 gpurun_out/r4a/pytest_local_full.log; ok $rc
timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4a/bench_local.json 2> gpurun_out/r4a/bench_local.err
rc=$?; echo "bench local rc $rc"; tail -c 600 gpurun_out/r4a/bench_local.json
for v in local walk1024 walk512; do
  BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/$v/libbra_hip.so timeout -k 10 120 python -u scripts/decode_bench.py --reps 5 >> gpurun_out/r4a/decode_ab.jsonl 2>> gpurun_out/r4a/decode_ab.err
  rc=$?; echo "decode $v rc $rc"; ok $rc
done
cat gpurun_out/r4a/decode_ab.jsonl
BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/nomj/libbra_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread -k "every_block" > gpurun_out/r4a/pytest_nomj_full.log 2>&1
rc=$?; echo "nomj fullsize rc $rc"; tail -12 gpurun_out/r4a/pytest_nomj_full.log; ok $rc
BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/nomj/libbra_hip.so timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4a/bench_nomj.json 2> gpurun_out/r4a/bench_nomj.err
rc=$?; echo "bench nomj rc $rc"; tail -c 600 gpurun_out/r4a/bench_nomj.json
for v in local16k nomj16k; do
  BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/$v/libbra_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k "every_block and (text_1MiB or sym16_8MiB_x32)" > gpurun_out/r4a/pytest_$v.log 2>&1
  rc=$?; echo "$v fullsize rc $rc"; tail -3 gpurun_out/r4a/pytest_$v.log; ok $rc
  BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/$v/libbra_hip.so timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > gpurun_out/r4a/bench_$v.json 2> gpurun_out/r4a/bench_$v.err
  rc=$?; echo "bench $v rc $rc"; tail -c 400 gpurun_out/r4a/bench_$v.json; ok $rc
done
