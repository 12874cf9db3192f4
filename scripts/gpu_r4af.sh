#!/bin/bash
# wave-job sorts: bitonic phases up to F then merge-path levels (F = 32 / 64 / 128; 256 = all bitonic)
set -o pipefail
O=gpurun_out/ab6f; mkdir -p $O
for v in m32 m64 m128; do
  BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/$v/libbra_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_jobs.py -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1
  rc=$?; echo "$v pytest rc $rc: $(tail -1 $O/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
NOTEST=1 REPS="1 2" SHOW=bwt.jobs O=$O bash scripts/gpu_ab6.sh m32 m64 m128
