# Co-rank search arity variants: parity of each variant build, then profiled benches (interleaved, twice)
set -e
O=${O:-gpurun_out/ary}; mkdir -p $O
for v in ${VARIANTS}; do
  BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/$v/libbra_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1
done
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 5 --warmup 2 --profile-all --no-cpu-baseline --no-secondary > $O/base_$r.json 2> $O/base_$r.err
  for v in ${VARIANTS}; do
    BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/$v/libbra_hip.so timeout -k 10 200 python bench.py --steps 5 --warmup 2 --profile-all --no-cpu-baseline --no-secondary > $O/${v}_$r.json 2> $O/${v}_$r.err
  done
done
echo done > $O/done
