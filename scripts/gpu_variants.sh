# bench (kernel slot timing) with each measurement variant of the library: VARIANTS="a b c"
set -e
mkdir -p gpurun_out/var
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --profile-all --no-cpu-baseline --no-secondary > gpurun_out/var/base.json 2> gpurun_out/var/base.err
for v in $VARIANTS; do
  BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/$v/libbra_hip.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --profile-all --no-cpu-baseline --no-secondary --no-check > gpurun_out/var/$v.json 2> gpurun_out/var/$v.err
done
