#!/bin/bash
# mailbox change, default bench line (dominant + stage slots timed, no per-kernel profiling)
NOTEST=1 REPS="1 2 3" BENCH_ARGS="--no-secondary" O=gpurun_out/ab6l bash scripts/gpu_ab6.sh h2
