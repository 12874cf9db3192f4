# Variant comparison only: one bench per variant under build/variants (job timing to stderr for *t builds).
# usage: O=gpurun_out/<tag> bash scripts/gpu_var.sh "<variant> ..." [extra bench args]
set -e
O=${O:-gpurun_out/var}; mkdir -p $O
BQ="python bench.py --no-cpu-baseline --no-secondary --profile-all --steps 3 --warmup 1 $2"
for v in $1; do
  BRA_HIP_LIB=br-archive_amd/build/variants/$v/libbra_hip.so timeout -k 10 200 $BQ > $O/bench_$v.json 2> $O/bench_$v.err
done
echo done > $O/done
