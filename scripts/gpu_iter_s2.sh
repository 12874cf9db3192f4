# parity (BWT-heavy tests) on the in-tree library, then benches of it and of measurement variants, + stream overlap
# usage: O=gpurun_out/<tag> VARIANTS="a b" bash scripts/gpu_iter_s2.sh
set -e
O=${O:-gpurun_out/it}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -k "not eight_shards and not round_robin" > $O/pytest.log 2>&1
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --profile-all --no-cpu-baseline --no-secondary > $O/base.json 2> $O/base.err
for v in $VARIANTS; do
  BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/$v/libbra_hip.so timeout -k 10 200 python bench.py --steps 5 --warmup 2 --profile-all --no-cpu-baseline --no-secondary > $O/$v.json 2> $O/$v.err
done
if [ -n "${STREAMS:-}" ]; then timeout -k 10 200 python scripts/exp_streams.py 1 2 > $O/streams.log 2>&1; fi
echo done > $O/done
