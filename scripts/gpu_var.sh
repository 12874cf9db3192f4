# bench (all kernel slots timed) with the in-tree library and each variant in $VARIANTS
set -e
O=${O:-gpurun_out/var}; mkdir -p $O
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --profile-all --no-cpu-baseline --no-secondary ${BENCH_ARGS:-} > $O/base.json 2> $O/base.err
for v in $VARIANTS; do
  BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/$v/libbra_hip.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --profile-all --no-cpu-baseline --no-secondary ${BENCH_ARGS:-} > $O/$v.json 2> $O/$v.err
done
