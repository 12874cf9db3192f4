# Scan workgroup width variants (BRA_SCAN_WAVES 1 / 2 builds) x scan grid (BRA_SCAN_GRID), profiled benches
set -e
O=${O:-gpurun_out/sw2}; mkdir -p $O
for v in sw2 sw1; do
  BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/$v/libbra_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1
done
B="python bench.py --steps 5 --warmup 2 --profile-all --no-cpu-baseline --no-secondary"
for r in 1 2; do
  timeout -k 10 200 $B > $O/base_$r.json 2> $O/base_$r.err
  BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/sw2/libbra_hip.so timeout -k 10 200 $B > $O/sw2_g4096_$r.json 2> /dev/null
  BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/sw2/libbra_hip.so BRA_SCAN_GRID=8192 timeout -k 10 200 $B > $O/sw2_g8192_$r.json 2> /dev/null
  BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/sw1/libbra_hip.so BRA_SCAN_GRID=8192 timeout -k 10 200 $B > $O/sw1_g8192_$r.json 2> /dev/null
  BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/sw1/libbra_hip.so BRA_SCAN_GRID=16384 timeout -k 10 200 $B > $O/sw1_g16384_$r.json 2> /dev/null
done
echo done > $O/done
