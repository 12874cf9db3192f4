# Repeat-encode stress (scripts/stress_repeat.py) of the in-tree library and of variants.
set -e
O=${O:-gpurun_out/sv}; mkdir -p $O
for v in $1; do
  BRA_HIP_LIB=br-archive_amd/build/variants/$v/libbra_hip.so timeout -k 10 300 python -u scripts/stress_repeat.py ${2:-6} > $O/$v.log 2>&1 || true
done
echo done > $O/done
