# bench (all slots timed) of the in-tree library and measurement variants; no parity run (measurement builds only)
O=${O:-gpurun_out/var3}; mkdir -p $O
set -e
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --profile-all --no-cpu-baseline --no-secondary > $O/base.json 2> $O/base.err
for v in $VARIANTS; do
  BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/$v/libbra_hip.so timeout -k 10 200 python bench.py --steps 5 --warmup 2 --profile-all --no-cpu-baseline --no-secondary > $O/$v.json 2> $O/$v.err
done
echo done > $O/done
