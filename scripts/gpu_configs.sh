#!/bin/bash
# The other single-GPU workloads at HEAD (round 6 closing pass; run on the GPU box through gpurun):
# uniform random 1 MiB blocks (configs[2]), 8 MiB 16-symbol blocks (one GPU's share of configs[4]),
# .BRa 256 KiB chunks, configs[0] (one 64 KiB tiled test.txt block), 8 MiB text blocks, and the
# reference programs' wall clock on a 1 GiB file.   usage: O=gpurun_out/<tag> bash scripts/gpu_configs.sh
set -o pipefail
O=${O:-gpurun_out/cfg}; mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 400 python -u bench.py --no-cpu-baseline "$@" > $O/bench_$tag.json 2>> $O/bench.err || exit $?;
        python3 scripts/show_bench.py $O/bench_$tag.json | head -1 | sed "s/^/[$tag] /"; }
run random --kind random
run sym16_8MiB --kind sym16 --block-size 8388608
run bra_mode_256KiB --block-size 262144
run text_8MiB --block-size 8388608
timeout -k 10 300 python -u bench.py --kind tiled --block-size 65536 --bytes-per-gpu 65536 --steps 20 --warmup 3 --no-secondary > $O/bench_cfg0.json 2>> $O/bench.err || exit $?
timeout -k 10 400 python -u scripts/prog_timing.py 1024 8 /tmp/pt 128 > $O/prog.json 2> $O/prog.err || exit $?
tail -c 600 $O/prog.json
