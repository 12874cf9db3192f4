#!/bin/bash
# presence masks through an LDS byte table (k_alpha): whole GPU suite, then A/B against HEAD
REPS="1 2" SHOW=bwt.pack O=gpurun_out/ab5g bash scripts/gpu_ab5.sh head
