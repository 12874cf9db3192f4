# chunk-stream tests (rows f1/f2) first, then the full GPU suite
set -e
mkdir -p gpurun_out/c
timeout -k 10 300 python -m pytest tests/test_gpu_chunks.py -m gpu -x -q > gpurun_out/c/chunks.log 2>&1
timeout -k 10 500 python -m pytest tests -m gpu -x -q > gpurun_out/c/all.log 2>&1
