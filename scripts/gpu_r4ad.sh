#!/bin/bash
# MSD level statistics (buckets / tiles / elements per level) of one text encode
O=gpurun_out/r4ad; mkdir -p $O
BRA_LEVEL_STATS=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-check --no-secondary > $O/bench.json 2> $O/levels.err
rc=$?; grep "bwt" $O/levels.err | tail -16; exit $rc
