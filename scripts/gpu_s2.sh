# Session-2 round-3 GPU pass: full -m gpu suite, smoke, default bench, one kernel-traced text step.
# usage: O=gpurun_out/<tag> bash scripts/gpu_s2.sh
set -e
O=${O:-gpurun_out/s2}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-check --no-secondary > $O/tr.log 2>&1
echo done > $O/done
