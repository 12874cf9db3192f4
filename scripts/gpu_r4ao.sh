#!/bin/bash
# round-4 closing check of the in-tree build: whole GPU suite, smoke, default bench line
set -o pipefail
O=gpurun_out/r4ao; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "suite rc $rc: $(tail -1 $O/pytest.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?; echo "bench rc $rc"; tail -c 300 $O/bench.json; exit $rc
