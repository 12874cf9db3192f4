#!/bin/bash
# round 4, call w: random-gather micro-benchmark (alignment / load form), times + TCP/TA counters
set -o pipefail
O=gpurun_out/r4w; mkdir -p $O
timeout -k 10 120 python -u scripts/micro/gather.py > $O/times.jsonl 2>&1 || exit $?
cat $O/times.jsonl
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TA_TA_BUSY_sum -d $R/$O/tcp -o run --output-format csv -- python3 $R/scripts/micro/gather.py > $R/$O/tcp.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc TCC_REQ_sum TCC_HIT_sum GRBM_GUI_ACTIVE -d $R/$O/tcc -o run --output-format csv -- python3 $R/scripts/micro/gather.py > $R/$O/tcc.log 2>&1 || exit $?
echo done
