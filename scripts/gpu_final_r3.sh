# Round-3 final GPU pass: full -m gpu suite, smoke, the default bench line, rocprofv3 --kernel-trace --stats of the bench.
# usage: O=gpurun_out/<tag> bash scripts/gpu_final_r3.sh
set -e
O=${O:-gpurun_out/final_r3}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err
echo done > $O/done
