# decode throughput under several env sets ($ENVS, space-separated sets, comma-separated vars), kinds in $KINDS, block size $BS
set -e
O=${O:-gpurun_out/decenv}; mkdir -p $O
for e in $ENVS; do
  for k in ${KINDS:-text}; do
    env $(echo $e | tr ',' ' ') timeout -k 10 200 python scripts/decode_bench.py --kind $k --block-size ${BS:-1048576} >> $O/decode.log 2>&1
    echo "env $e" >> $O/decode.log
  done
done
