set -e
mkdir -p gpurun_out/dec2
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -m gpu -x -q > gpurun_out/dec2/pytest.log 2>&1
for k in text:1048576 random:1048576 sym16:8388608 tiled:65536; do
  timeout -k 10 300 python scripts/decode_bench.py --kind ${k%%:*} --block-size ${k##*:} >> gpurun_out/dec2/decode.log 2>&1
done
