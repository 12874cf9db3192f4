# level statistics of the config-1 block after the determinism batch vs alone
O=gpurun_out/dbg3; mkdir -p $O
BRA_LEVEL_STATS=1 timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -s --timeout 150 --timeout-method thread -k "deterministic or config1" > $O/seq.log 2>&1
rc=$?; echo "seq rc=$rc" >> $O/rc.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
BRA_LEVEL_STATS=1 timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -s --timeout 150 --timeout-method thread -k "config1" > $O/alone.log 2>&1
rc=$?; echo "alone rc=$rc" >> $O/rc.txt
echo done > $O/done
