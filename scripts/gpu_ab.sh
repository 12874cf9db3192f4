# A/B: the duplicated-region / periodic parity tests, 3 runs per library (main = in-tree).  Stops on anything but pass / test failure.
O=gpurun_out/ab; mkdir -p $O
for v in ${AB_VARIANTS:-main old hw0}; do
  for i in 1 2 3; do
    if [ $v = main ]; then L=$PWD/br-archive_amd/libbra_hip.so; else L=$PWD/br-archive_amd/build/variants/$v/libbra_hip.so; fi
    BRA_HIP_LIB=$L timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 100 --timeout-method thread -k "duplicated or config1 or periodic or deterministic" > $O/${v}_$i.log 2>&1
    rc=$?; echo "$v $i rc=$rc $(tail -1 $O/${v}_$i.log)" >> $O/rc.txt
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  done
done
echo done > $O/done
