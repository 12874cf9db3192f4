#!/bin/bash
# jobs mailbox posted right after the jobs (host resumes mid-step): whole GPU suite, then A/B vs HEAD
REPS="1 2" SHOW=bwt.mjobs O=gpurun_out/ab5k bash scripts/gpu_ab5.sh h2
