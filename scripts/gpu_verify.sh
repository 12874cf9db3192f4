# Quick tree check on the GPU box: full -m gpu suite, smoke, one default bench line.
set -e
O=${O:-gpurun_out/verify}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
echo done > $O/done
