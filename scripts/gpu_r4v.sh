#!/bin/bash
# round 4, call v: decode walk grid sweep (persistent walk workgroups = live splitters per XCD)
set -o pipefail
O=gpurun_out/r4v; mkdir -p $O
for rep in 1 2; do
for v in ${VARS:-default walk512 walk1024 walk4096}; do
  L=$PWD/br-archive_amd/libbra_hip.so; [ $v = default ] || L=$PWD/br-archive_amd/build/variants/$v/libbra_hip.so
  BRA_HIP_LIB=$L timeout -k 10 120 python -u scripts/decode_bench.py --reps 5 > $O/dec_${v}_$rep.json 2>> $O/dec.err
  rc=$?; echo "$v rc $rc $(cat $O/dec_${v}_$rep.json)"; [ $rc -eq 0 ] || exit $rc
done
done
