# decode timing under env sets: RUNS="KIND:ENV ..." (bench with the secondary decode measurement)
set -e
O=${O:-gpurun_out/ds}; mkdir -p $O
for r in $RUNS; do
  k=${r%%:*}; e=${r#*:}; n=$(echo $r | tr ',=:' '_-_')
  bs=1048576; [ $k = sym16 ] && bs=8388608
  env $(echo $e | tr ',' ' ') timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --kind $k --block-size $bs > $O/$n.json 2> $O/$n.err
done
