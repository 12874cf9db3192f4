#!/bin/bash
# round 4, call z: job sort-size histogram (timing build), one encode step
set -o pipefail
O=gpurun_out/r4z; mkdir -p $O
BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/jt/libbra_hip.so timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-check --no-secondary > $O/bench.json 2> $O/jt.err
rc=$?; grep "job" $O/jt.err | tail -8; exit $rc
