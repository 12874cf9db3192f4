#!/bin/bash
# round 4, call s: k_scan phase clocks (BRA_SCAN_TIMING build), text 1 MiB
set -o pipefail
O=gpurun_out/r4s; mkdir -p $O
BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/st/libbra_hip.so timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-check --no-secondary > $O/bench_st.json 2> $O/st.err
echo "st rc $?"; grep -E "scan timing" $O/st.err | tail -3
