set -e
mkdir -p gpurun_out
timeout -k 10 500 python scripts/stress_bwt.py 40 > gpurun_out/stress.log 2>&1
