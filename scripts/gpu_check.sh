# parity suite (test_gpu_parity) then bench of $KIND under several env sets ($ENVS, see gpu_envs2.sh)
set -e
O=${O:-gpurun_out/chk}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $O/pytest.log 2>&1
O=$O ENVS="${ENVS:-X=0}" BENCH_ARGS="${BENCH_ARGS:-}" bash scripts/gpu_envs2.sh
