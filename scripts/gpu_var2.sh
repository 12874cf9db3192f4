# bench (all slots timed) with measurement variants of the library, plus the multi-context overlap experiment.
# usage: O=gpurun_out/<tag> VARIANTS="a b" bash scripts/gpu_var2.sh
set -e
O=${O:-gpurun_out/var2}; mkdir -p $O
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --profile-all --no-cpu-baseline --no-secondary > $O/base.json 2> $O/base.err
for v in $VARIANTS; do
  BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/$v/libbra_hip.so timeout -k 10 200 python bench.py --steps 5 --warmup 2 --profile-all --no-cpu-baseline --no-secondary > $O/$v.json 2> $O/$v.err
done
timeout -k 10 200 python scripts/exp_streams.py 1 2 > $O/streams.log 2>&1
echo done > $O/done
