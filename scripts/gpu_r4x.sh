#!/bin/bash
set -o pipefail
O=gpurun_out/ab5a bash scripts/gpu_ab5.sh base && VARS="default walk256 walk384 walk512 walk768" bash scripts/gpu_r4v.sh
