#!/bin/bash
# RLE write-kernel cost split (measurement builds: histogram atomics / output copy skipped)
NOTEST=1 REPS="1 2" O=gpurun_out/ab6c bash scripts/gpu_ab6.sh rnohist rnocopy
