set -e
O=gpurun_out/l2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum -d $O/tcc -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-check --no-secondary > $O/tcc.log 2>&1
