#!/bin/bash
# A/B of the in-tree library against saved variants: the whole GPU test suite on the in-tree build,
# then bench lines alternating default / variants twice.
# usage: O=gpurun_out/<tag> bash scripts/gpu_ab5.sh variant [variant ...]
set -o pipefail
O=${O:-gpurun_out/ab5}; mkdir -p $O
[ -n "$NOTEST" ] || timeout -k 10 700 python -u -m pytest tests/test_gpu_jobs.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc $rc: $(tail -1 $O/pytest.log)"; [ $rc -eq 0 ] || { tail -40 $O/pytest.log; exit $rc; }
for rep in ${REPS:-1 2}; do
  for v in default "$@"; do
    L=$PWD/br-archive_amd/libbra_hip.so; [ $v = default ] || L=$PWD/br-archive_amd/build/variants/$v/libbra_hip.so
    BRA_HIP_LIB=$L timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-check ${BENCH_ARGS---profile-all} > $O/bench_${v}_$rep.json 2>> $O/bench.err
    rc=$?; [ $rc -eq 0 ] || { echo "bench $v rc $rc"; exit $rc; }
    python3 scripts/show_bench.py $O/bench_${v}_$rep.json | python3 -c "
import sys,os; L=sys.stdin.read().splitlines(); print('$v', L[0][:60]); [print('  ', l) for l in L[1:] if any(k in l for k in (os.environ.get('SHOW','jobs,scatter').split(',')))]"
  done
done
