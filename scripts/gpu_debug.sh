mkdir -p gpurun_out/dbg4
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "full_size_256mib and 0" > gpurun_out/dbg4/pytest.log 2>&1
echo "rc=$?"
grep -c dcheck gpurun_out/dbg4/pytest.log
grep -o "\[bra dsync\][^\[]*" gpurun_out/dbg4/pytest.log | head -3
grep -o "\[bra dcheck\][^\[]*" gpurun_out/dbg4/pytest.log | sort | uniq -c | sort -rn | head -20
