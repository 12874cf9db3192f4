#!/bin/bash
# small sorts in the workgroup jobs too (wave 0 of the workgroup): W <= 2, or W <= 4 with P <= 64
set -o pipefail
O=gpurun_out/ab6j; mkdir -p $O
for v in sw2 sw4r1; do
  BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/$v/libbra_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_jobs.py -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1
  rc=$?; echo "$v pytest rc $rc: $(tail -1 $O/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
NOTEST=1 REPS="1 2" SHOW=bwt.jobs,bwt.mjobs O=$O bash scripts/gpu_ab6.sh sw2 sw4r1
