#!/bin/bash
# round 4, call t: available counters; TA / TCP / TCC busy and request counters of the bench kernels
set -o pipefail
O=gpurun_out/r4t; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 rocprofv3 --list-avail > $O/avail.txt 2>&1; echo "avail rc $?"
grep -oE "^\s*(TA|TD|TCP|TCC)_[A-Z0-9_]+" $O/avail.txt | sort -u | head -150 > $O/names.txt
B1="python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-check --no-secondary"
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum -d $O/ta -o run --output-format csv -- $B1 > $O/ta.log 2>&1; echo "ta rc $?"
timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum -d $O/tcp -o run --output-format csv -- $B1 > $O/tcp.log 2>&1; echo "tcp rc $?"
timeout -s KILL 120 rocprofv3 --pmc TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum -d $O/tcc -o run --output-format csv -- $B1 > $O/tcc.log 2>&1; echo "tcc rc $?"
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d $O/gr -o run --output-format csv -- $B1 > $O/gr.log 2>&1; echo "gr rc $?"
