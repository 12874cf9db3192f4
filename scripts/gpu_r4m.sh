#!/bin/bash
# round 4, call m: the scc-clobber fix -- shuffled job re-runs (audit build), the chunk-stream stress
# loop and the whole -m gpu suite on the product build
set -o pipefail
O=gpurun_out/r4m; mkdir -p $O
BRA_DIAG_DIR=$O BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/audit/libbra_hip.so timeout -k 10 200 python -u scripts/rerun_jobs.py 0 262144 1024 200 1000 > $O/rerun.log 2>&1
rc=$?; echo "audit rerun rc $rc: $(tail -1 $O/rerun.log)"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u scripts/sortnet_stress.py 8 > $O/sortnet.json 2>&1
echo "sortnet rc $?: $(cat $O/sortnet.json)"
BRA_DIAG_DIR=$O timeout -k 10 400 python -u scripts/stress_chunks.py 60 > $O/stress.log 2>&1
rc=$?; echo "stress rc $rc"; grep -v "'ok', 'sym16_256KiB_x1024': 'ok'" $O/stress.log | tail -5; [ $rc -le 1 ] || exit $rc
timeout -k 10 420 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -8
