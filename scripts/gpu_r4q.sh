#!/bin/bash
# round 4, call q: k_scan with per-segment job chains -- parity (full-size, chunks) and bench
set -o pipefail
O=gpurun_out/${TAG:-r4q}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_chunks.py tests/test_gpu_jobs.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc $rc: $(tail -1 $O/pytest.log)"; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --profile-all > $O/bench.json 2>> $O/bench.err
rc=$?; echo "bench rc $rc"; python3 scripts/show_bench.py $O/bench.json | head -12
