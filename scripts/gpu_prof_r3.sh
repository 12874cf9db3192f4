# Profiling session: rocprofv3 kernel stats of the bench (text) and of a decode run, then PMC passes
# (one counter group per rocprofv3 run) for the three single-GPU BASELINE workloads.
# usage: O=gpurun_out/<tag> bash scripts/gpu_prof_r3.sh
set -e
O=${O:-gpurun_out/prof}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-check --no-secondary"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr -o run --output-format csv -- $B > $O/trace.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trdec -o run --output-format csv -- python3 scripts/decode_bench.py --kind text --reps 2 > $O/trdec.log 2>&1
for w in "text 1048576" "random 1048576" "sym16 8388608"; do
  set -- $w
  B1="python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-check --no-secondary --kind $1 --block-size $2"
  D=$O/pmc_$1_$2
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $D/fetch -o run --output-format csv -- $B1 > $D.fetch.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $D/write -o run --output-format csv -- $B1 > $D.write.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS -d $D/sq1 -o run --output-format csv -- $B1 > $D.sq1.log 2>&1
done
echo done > $O/done
