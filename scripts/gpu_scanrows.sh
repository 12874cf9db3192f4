# Scan-row variants: parity of the in-tree build, then profiled benches of base / rows4 / rows16 (twice, interleaved)
set -e
O=${O:-gpurun_out/rows}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 5 --warmup 2 --profile-all --no-cpu-baseline --no-secondary > $O/base_$r.json 2> $O/base_$r.err
  for v in rows4 rows16; do
    BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/$v/libbra_hip.so timeout -k 10 200 python bench.py --steps 5 --warmup 2 --profile-all --no-cpu-baseline --no-secondary > $O/${v}_$r.json 2> $O/${v}_$r.err
  done
done
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-secondary > $O/plain.json 2> $O/plain.err
echo done > $O/done
