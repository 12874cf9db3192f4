#!/bin/bash
# round 4, call o: DPP-operand compare-exchange -- correctness (sort test, job re-runs, job tests,
# full-size parity) and the bench A/B against the separate-DPP-move build
set -o pipefail
O=gpurun_out/r4o; mkdir -p $O
timeout -k 10 200 python -u scripts/sortnet_stress.py 8 > $O/sortnet.json 2>&1; echo "sortnet rc $?: $(cat $O/sortnet.json)"
BRA_DIAG_DIR=$O BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/audit/libbra_hip.so timeout -k 10 200 python -u scripts/rerun_jobs.py 0 262144 1024 200 1000 > $O/rerun.log 2>&1
rc=$?; echo "audit rerun rc $rc: $(tail -1 $O/rerun.log)"; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_jobs.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc $rc: $(tail -1 $O/pytest.log)"; [ $rc -le 1 ] || exit $rc
for v in default nodpp default nodpp; do
  L=$PWD/br-archive_amd/libbra_hip.so; [ $v = default ] || L=$PWD/br-archive_amd/build/variants/$v/libbra_hip.so
  BRA_HIP_LIB=$L timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --profile-all > $O/bench_$v.json 2>> $O/bench.err
  rc=$?; echo "bench $v rc $rc"; python3 scripts/show_bench.py $O/bench_$v.json 2>/dev/null | head -12; [ $rc -eq 0 ] || exit $rc
done
