#!/bin/bash
# One GPU pass over the in-tree build (run on the GPU box through gpurun).
#   usage: O=gpurun_out/<tag> STEPS="tests smoke bench prof pmc" bash scripts/gpu_pass.sh
# Steps (any subset, in this order):
#   tests   the whole -m gpu suite                       -> $O/pytest.log
#   smoke   __graft_entry__.smoke()                       -> $O/smoke.log
#   bench   the default bench line (+ BENCH_ARGS)         -> $O/bench.json
#   prof    rocprofv3 --kernel-trace --stats of the bench -> $O/prof/run_kernel_stats.csv
#   pmc     FETCH_SIZE / WRITE_SIZE / SQ counter passes for the single-GPU BASELINE workloads
#           (PMC_WORKLOADS, default text 1 MiB, random 1 MiB, sym16 8 MiB)  -> $O/pmc_<kind>_<bs>/
# Every GPU step runs under its own timeout; the pass stops at the first step that crashes or
# times out (exit status > 1), so nothing more runs on a GPU in a bad state.
set -o pipefail
O=${O:-gpurun_out/pass}; mkdir -p $O
STEPS=${STEPS:-tests smoke bench prof}
has() { case " $STEPS " in *" $1 "*) return 0;; esac; return 1; }
step() { echo "== $1 rc $2"; [ $2 -le 1 ] || exit $2; }
if has tests; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $O/pytest.log 2>&1; step tests $?
  grep -E "passed|failed" $O/pytest.log | tail -1
fi
if has smoke; then
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; step smoke $?
fi
if has bench; then
  timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err; step bench $?
  tail -c 600 $O/bench.json
fi
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if has prof; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > $O/prof_bench.json 2> $O/prof.err; step prof $?
fi
if has pmc; then
  for w in ${PMC_WORKLOADS:-text:1048576 random:1048576 sym16:8388608}; do
    k=${w%%:*}; bs=${w#*:}
    B1="python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-check --no-secondary --kind $k --block-size $bs"
    D=$O/pmc_${k}_$bs
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $D/fetch -o run --output-format csv -- $B1 > $D.fetch.log 2>&1; step "pmc fetch $k" $?
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $D/write -o run --output-format csv -- $B1 > $D.write.log 2>&1; step "pmc write $k" $?
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS -d $D/sq1 -o run --output-format csv -- $B1 > $D.sq1.log 2>&1; step "pmc sq $k" $?
    timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $D/grbm -o run --output-format csv -- $B1 > $D.grbm.log 2>&1; step "pmc grbm $k" $?
  done
fi
echo done > $O/done
