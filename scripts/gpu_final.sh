# End-of-round GPU session: full -m gpu suite, stress, smoke, the bench line (N=1, CPU baseline),
# profiled bench, BASELINE suite workloads, rocprofv3 kernel stats (encode + decode) and PMC
# passes (each counter group in its own run).  usage: O=gpurun_out/<tag> bash scripts/gpu_final.sh
set -e
O=${O:-gpurun_out/final}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 python -u scripts/stress_bwt.py ${STRESS:-4} > $O/stress.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --profile-all --no-cpu-baseline > $O/bench_all.json 2> $O/bench_all.err
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --kind random > $O/suite_random_1MiB.json 2> $O/suite_random.err
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --kind sym16 --block-size 8388608 > $O/suite_sym16_8MiB.json 2> $O/suite_sym16.err
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --block-size 262144 > $O/suite_text_256KiB.json 2> $O/suite_text256.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-check --no-secondary"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr -o run --output-format csv -- $B > $O/trace.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trdec -o run --output-format csv -- python3 scripts/decode_bench.py --kind text --reps 2 > $O/trdec.log 2>&1
B1="python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-check --no-secondary"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc/fetch -o run --output-format csv -- $B1 > $O/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc/write -o run --output-format csv -- $B1 > $O/pmc_write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS -d $O/pmc/sq1 -o run --output-format csv -- $B1 > $O/pmc_sq1.log 2>&1
echo done > $O/done
