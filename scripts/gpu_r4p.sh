#!/bin/bash
# round 4, call p: job-phase cycle breakdown (BRA_JOB_TIMING build) and MSD level counts, text 1 MiB
set -o pipefail
O=gpurun_out/r4p; mkdir -p $O
BRA_LEVEL_STATS=1 BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/jt/libbra_hip.so timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-check --no-secondary > $O/bench_jt.json 2> $O/jt.err
echo "jt rc $?"; grep -E "job timing|bwt levels|bwt finish" $O/jt.err | tail -24
