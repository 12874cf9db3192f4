#!/bin/bash
O=gpurun_out/r4ai; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log; exit $rc
