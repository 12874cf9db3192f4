#!/bin/bash
# Rehearsal of the N > 1 bench path on one GPU: 2 and 4 ranks sharing the device, gloo exchange
set -o pipefail
O=gpurun_out/r4ah; mkdir -p $O
for n in 2 4; do
  timeout -k 10 400 python -u bench.py --gpus $n --backend gloo --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_g$n.json 2> $O/bench_g$n.err
  rc=$?; echo "gpus $n rc $rc"; tail -c 1200 $O/bench_g$n.json; echo; [ $rc -eq 0 ] || { tail -20 $O/bench_g$n.err; exit $rc; }
done
