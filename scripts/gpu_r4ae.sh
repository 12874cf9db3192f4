#!/bin/bash
# MSD histogram grid sweep (k_hist workgroups; default 16384)
NOTEST=1 REPS="1 2" SHOW=bwt.hist,bwt.scan,bwt.scatter O=gpurun_out/ab6e bash scripts/gpu_ab6.sh h2k h4k h8k
