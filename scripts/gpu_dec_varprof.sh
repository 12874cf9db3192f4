# kernel stats (rocprofv3) of the text decode for the in-tree library and each variant in $VARIANTS
set -e
O=${O:-gpurun_out/dvp}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/base -o run --output-format csv -- python3 scripts/decode_bench.py --kind ${KIND:-text} --reps 2 > $O/base.log 2>&1
for v in $VARIANTS; do
  BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/$v/libbra_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- python3 scripts/decode_bench.py --kind ${KIND:-text} --reps 2 > $O/$v.log 2>&1
done
