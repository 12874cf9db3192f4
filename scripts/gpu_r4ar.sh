#!/bin/bash
# walk grid by splitter step: decode parity tests, text and sym16 8 MiB decode
set -o pipefail
O=gpurun_out/r4ar; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "suite rc $rc: $(tail -1 $O/pytest.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/decode_bench.py --reps 5 > $O/dec_text.json && timeout -k 10 120 python -u scripts/decode_bench.py --kind sym16 --block-size 8388608 --reps 5 > $O/dec_sym16.json || exit $?
cat $O/dec_text.json $O/dec_sym16.json
