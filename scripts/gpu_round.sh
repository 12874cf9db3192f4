# One GPU session: parity tests, determinism stress, bench, rocprofv3 stats + PMC passes.
set -e
mkdir -p gpurun_out/r1
O=gpurun_out/r1
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -m gpu -x -q > $O/pytest.log 2>&1
timeout -k 10 300 python scripts/stress_bwt.py 20 > $O/stress.log 2>&1
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --profile-all --no-cpu-baseline > $O/bench_all.json 2> $O/bench_all.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-check"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- $B > $O/stats.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- $B > $O/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- $B > $O/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS -d $O/sq1 -o run --output-format csv -- $B > $O/sq1.log 2>&1
cd "$GRAFT_REPO_ROOT"
for v in ${VARIANTS:-}; do
  BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/$v/libbra_hip.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --profile-all --no-cpu-baseline --no-secondary --no-check > $O/var_$v.json 2> $O/var_$v.err
done
