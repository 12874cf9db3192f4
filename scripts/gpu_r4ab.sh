#!/bin/bash
NOTEST=1 REPS="1 2 3" O=gpurun_out/ab6b bash scripts/gpu_ab6.sh base s4 s32
