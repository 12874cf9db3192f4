# GPU parity suite only (driver flags), log under $O
set -e
O=${O:-gpurun_out/t}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $O/pytest.log 2>&1
