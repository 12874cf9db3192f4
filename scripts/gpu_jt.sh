# Job-phase timing (diagnostic variant build) on the bench workload: stderr holds the phase sums.
set -e
O=${O:-gpurun_out/jt}; mkdir -p $O
for mw in 4 8; do
  BRA_MJ_WAVES=$mw BRA_HIP_LIB=br-archive_amd/build/variants/jt/libbra_hip.so timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary --no-check > $O/bench_mw$mw.json 2> $O/bench_mw$mw.err
done
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --profile-all > $O/bench_prod.json 2> $O/bench_prod.err
echo done > $O/done
