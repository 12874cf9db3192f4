#!/bin/bash
# A/B of the in-tree library against measurement variants built by scripts/build_variants.sh
# (br-archive_amd/build/variants/<name>/libbra_hip.so), alternating on one box: bench lines with
# every profiler slot timed, REPS rounds of default + each variant.  PARITY=1 first runs the
# full-size digest, chunk-stream and job re-run tests on the in-tree build.  A variant "env:VAR=VALUE"
# runs the in-tree library with that environment setting instead.
#   usage: O=gpurun_out/<tag> [REPS=2] [PARITY=1] [BENCH_ARGS=...] bash scripts/gpu_ab.sh variant [variant ...]
set -o pipefail
O=${O:-gpurun_out/ab}; mkdir -p $O
if [ "${PARITY:-0}" = 1 ]; then
  timeout -k 10 500 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_chunks.py tests/test_gpu_jobs.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; echo "pytest rc $rc: $(tail -1 $O/pytest.log)"; [ $rc -le 1 ] || exit $rc
fi
for rep in $(seq 1 ${REPS:-2}); do
  for v in default "$@"; do
    L=$PWD/br-archive_amd/libbra_hip.so; E=BRA_AB_NONE=1
    case $v in default) ;; env:*) E=${v#env:} ;; *) L=$PWD/br-archive_amd/build/variants/$v/libbra_hip.so ;; esac
    env $E BRA_HIP_LIB=$L timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-check --profile-all ${BENCH_ARGS:-} > $O/bench_${v}_$rep.json 2>> $O/bench.err
    rc=$?; [ $rc -eq 0 ] || { echo "bench $v rc $rc"; exit $rc; }
    python3 scripts/show_bench.py $O/bench_${v}_$rep.json | head -${SHOW_LINES:-40} | sed "s/^/[$v $rep] /"
  done
done
