# rebuild with each EXTRA define set (space-separated, commas inside a set), then run $RUNS (gpu_dec_sweep.sh)
set -e
O0=${O:-gpurun_out/bs}; mkdir -p $O0
for x in $DEFS; do
  n=$(echo $x | tr ',=' '_-')
  make -C br-archive_amd -B -j16 EXTRA="$(echo $x | tr ',' ' ')" > $O0/build_$n.log 2>&1
  O=$O0/$n bash scripts/gpu_dec_sweep.sh
done
