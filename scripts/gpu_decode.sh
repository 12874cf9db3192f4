set -e
O=gpurun_out/dec
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for k in text:1048576 random:1048576 sym16:8388608; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${k%%:*} -o run --output-format csv -- python3 scripts/decode_bench.py --kind ${k%%:*} --block-size ${k##*:} > $O/${k%%:*}.log 2>&1
done
