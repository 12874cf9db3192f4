# decode throughput (text / random 1 MiB blocks) + rocprofv3 kernel stats of the text decode
set -e
O=${O:-gpurun_out/dec}; mkdir -p $O
for k in ${KINDS:-text random}; do
  timeout -k 10 300 python scripts/decode_bench.py --kind $k >> $O/decode.log 2>&1
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr -o run --output-format csv -- python3 scripts/decode_bench.py --kind ${PKIND:-text} --reps 2 > $O/trace.log 2>&1
