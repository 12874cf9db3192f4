# decode throughput with the in-tree library and each variant in $VARIANTS (kinds in $KINDS)
set -e
O=${O:-gpurun_out/decvar}; mkdir -p $O
for k in ${KINDS:-text random}; do
  timeout -k 10 200 python scripts/decode_bench.py --kind $k > $O/base_$k.json 2>&1
  for v in $VARIANTS; do
    BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/$v/libbra_hip.so timeout -k 10 200 python scripts/decode_bench.py --kind $k > $O/${v}_$k.json 2>&1
  done
done
