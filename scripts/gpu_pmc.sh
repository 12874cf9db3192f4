# PMC passes over one bench step (each pass its own rocprofv3 run; counters only with --kernel-trace-free collection)
set -e
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-check"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS -d gpurun_out/pmc/sq1 -o run --output-format csv -- $B > gpurun_out/pmc/sq1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC -d gpurun_out/pmc/sq2 -o run --output-format csv -- $B > gpurun_out/pmc/sq2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc/fetch -o run --output-format csv -- $B > gpurun_out/pmc/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc/write -o run --output-format csv -- $B > gpurun_out/pmc/write.log 2>&1
