#!/bin/bash
set -o pipefail
bash scripts/gpu_r4w.sh && bash scripts/gpu_r4v.sh
