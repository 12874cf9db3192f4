#!/bin/bash
# decode walk grid for 8 MiB 16-symbol blocks (splitter step 2048: 8x the TL bytes per live lane)
set -o pipefail
O=gpurun_out/r4aq; mkdir -p $O
for rep in 1 2; do
for v in default w128 w192 w256; do
  L=$PWD/br-archive_amd/libbra_hip.so; [ $v = default ] || L=$PWD/br-archive_amd/build/variants/$v/libbra_hip.so
  BRA_HIP_LIB=$L timeout -k 10 120 python -u scripts/decode_bench.py --kind sym16 --block-size 8388608 --reps 5 > $O/dec_${v}_$rep.json 2>> $O/dec.err
  rc=$?; echo "$v rc $rc $(python3 -c "import json;d=json.load(open('$O/dec_${v}_$rep.json'));print(d['decode_GBps'], d['slots_ms'].get('dec.ib_walk'), d['roundtrip'])")"; [ $rc -eq 0 ] || exit $rc
done
done
