# Determinism + parity session (stage diagnosis on failure), then the three benches.
set -e
O=${O:-gpurun_out/det}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread -k "deterministic or duplicated" > $O/det.log 2>&1 || true
bash scripts/gpu_iter4.sh ""
