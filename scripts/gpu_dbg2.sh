# debug-build run of the order-dependent parity sequence (device range checks print to stdout)
O=gpurun_out/dbg2; mkdir -p $O
for i in 1 2; do
  BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/dbg/libbra_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -s --timeout 250 --timeout-method thread -k "duplicated or config1 or periodic or deterministic" > $O/run_$i.log 2>&1
  rc=$?; echo "$i rc=$rc" >> $O/rc.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
echo done > $O/done
