# A/B of library variants on the config-1 tiled block and the periodic batch (stops on anything but pass / test failure)
O=gpurun_out/dbg; mkdir -p $O
for v in hw0 hwc; do
  BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/$v/libbra_hip.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 100 --timeout-method thread -k "config1 or periodic" > $O/$v.log 2>&1
  rc=$?; echo "$v rc=$rc" >> $O/rc.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
echo done > $O/done
