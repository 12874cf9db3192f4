#!/bin/bash
# round 4, call u: job round 0 on carried payload digits -- audit re-runs, parity, A/B bench
set -o pipefail
O=gpurun_out/r4u; mkdir -p $O
BRA_DIAG_DIR=$O BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/audit/libbra_hip.so timeout -k 10 200 python -u scripts/rerun_jobs.py 0 262144 1024 100 1000 > $O/rerun.log 2>&1
rc=$?; echo "audit rerun rc $rc: $(tail -1 $O/rerun.log)"; grep "bwt audit" $O/rerun.log | head -5; [ $rc -le 1 ] || exit $rc
O=$O bash scripts/gpu_ab4.sh nor0
