# Round-3 GPU session: full -m gpu suite, smoke, the default bench line.
# usage: O=gpurun_out/<tag> bash scripts/gpu_r3.sh [pytest -k expression]
set -e
O=${O:-gpurun_out/r3}; mkdir -p $O
K=${1:+-k "$1"}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $K > $O/pytest.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
echo done > $O/done
