#!/bin/bash
# RLE encode in one classification pass (decoupled look-back, variant rlelb): parity tests and the
# whole GPU suite on the variant, then A/B against the in-tree library
set -o pipefail
O=gpurun_out/ab5n; mkdir -p $O
export BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/rlelb/libbra_hip.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest_parity.log 2>&1
rc=$?; echo "parity tests rc $rc: $(tail -1 $O/pytest_parity.log)"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/pytest_parity.log | head -20; exit $rc; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "suite rc $rc: $(tail -1 $O/pytest.log)"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit $rc; }
unset BRA_HIP_LIB
NOTEST=1 REPS="1 2" SHOW=rle BENCH_ARGS="--no-secondary --profile-all" O=$O bash scripts/gpu_ab6.sh rlelb
