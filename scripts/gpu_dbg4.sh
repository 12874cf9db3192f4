# config-1 block after the determinism batch with the BWT outputs poisoned before each encode (diagnostic variant)
O=gpurun_out/dbg4; mkdir -p $O
BRA_LEVEL_STATS=1 BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/zpi/libbra_hip.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -s --timeout 150 --timeout-method thread -k "deterministic or config1" > $O/seq.log 2>&1
echo "rc=$?" > $O/rc.txt
