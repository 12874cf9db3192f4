# parity tests + bench for one measurement variant of the library: V=name
set -e
O=gpurun_out/vt; mkdir -p $O
export BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/$V/libbra_hip.so
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -x -q > $O/pytest_$V.log 2>&1
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --profile-all --no-cpu-baseline --no-secondary > $O/bench_$V.json 2> $O/bench_$V.err
