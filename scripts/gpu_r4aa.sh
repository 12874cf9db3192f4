#!/bin/bash
set -o pipefail
bash scripts/gpu_r4z.sh && O=gpurun_out/ab5b bash scripts/gpu_ab5.sh base
