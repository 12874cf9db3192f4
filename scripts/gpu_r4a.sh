#!/bin/bash
# round 4, call a: the chunk-stream tests with localisation, then the stress loop
set -o pipefail
mkdir -p gpurun_out/r4a
timeout -k 10 300 python -u -m pytest tests/test_gpu_chunks.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4a/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; [ $rc -le 1 ] || exit $rc
tail -3 gpurun_out/r4a/pytest.log
timeout -k 10 400 python -u scripts/stress_chunks.py 10 > gpurun_out/r4a/stress.log 2>&1
echo "stress rc $?"
cat gpurun_out/r4a/stress.log
