#!/bin/bash
# Huffman leaf list in closed form: tie test first, whole GPU suite, then A/B vs HEAD
set -o pipefail
O=gpurun_out/ab5m; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "huffman" -x -q --timeout 200 --timeout-method thread > $O/pytest_huf.log 2>&1
rc=$?; echo "huffman tests rc $rc: $(tail -1 $O/pytest_huf.log)"; [ $rc -eq 0 ] || { tail -30 $O/pytest_huf.log; exit $rc; }
REPS="1 2" SHOW=huf.build BENCH_ARGS="--no-secondary --profile-all" O=$O bash scripts/gpu_ab5.sh h3
