#!/bin/bash
# round 4, call n: job tests, the default bench line, rocprofv3 kernel stats of the bench
set -o pipefail
O=gpurun_out/r4n; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_jobs.py -v --timeout 120 --timeout-method thread > $O/pytest_jobs.log 2>&1
rc=$?; echo "jobs rc $rc"; tail -3 $O/pytest_jobs.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc $rc"; python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline'],d.get('pipeline',{}).get('stages_ms'))"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err
echo "prof rc $?"; ls $O/prof/*/ 2>/dev/null | head
