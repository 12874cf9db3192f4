#!/bin/bash
# Round-4 GPU pass: the whole -m gpu suite, smoke, the default bench line, rocprofv3 --kernel-trace
# --stats of the bench, and the PMC passes (FETCH_SIZE / WRITE_SIZE / SQ) for the three single-GPU
# BASELINE workloads.   usage: O=gpurun_out/<tag> bash scripts/gpu_final_r4.sh
set -o pipefail
O=${O:-gpurun_out/final_r4}; mkdir -p $O
step() { echo "== $1 rc $2"; [ $2 -le 1 ] || exit $2; }
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; step pytest $?
grep -E "passed|failed" $O/pytest.log | tail -1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; step smoke $?
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err; step bench $?
tail -c 400 $O/bench.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err; step prof $?
for w in "text 1048576" "random 1048576" "sym16 8388608"; do
  set -- $w
  B1="python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-check --no-secondary --kind $1 --block-size $2"
  D=$O/pmc_$1_$2
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $D/fetch -o run --output-format csv -- $B1 > $D.fetch.log 2>&1; step "pmc fetch $1" $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $D/write -o run --output-format csv -- $B1 > $D.write.log 2>&1; step "pmc write $1" $?
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS -d $D/sq1 -o run --output-format csv -- $B1 > $D.sq1.log 2>&1; step "pmc sq $1" $?
done
echo done > $O/done
