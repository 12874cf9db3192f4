# BASELINE configs[0]: the reference's own CPU case (test/test.txt tiled into one 64 KiB block),
# GPU latency per block with the reference's CPU time for the same block beside it.
set -e
O=${O:-gpurun_out/cfg0}; mkdir -p $O
timeout -k 10 400 python bench.py --kind tiled --block-size 65536 --bytes-per-gpu 65536 --steps 50 --warmup 5 > $O/bench_cfg0.json 2> $O/bench_cfg0.err
echo done > $O/done
