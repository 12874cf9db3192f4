#!/bin/bash
# Decode A/B (scripts/decode_bench.py) of the in-tree library against measurement variants
# (br-archive_amd/build/variants/<name>/libbra_hip.so), alternating on one box, then a rocprofv3
# kernel trace of the in-tree decode.
#   usage: O=gpurun_out/<tag> [REPS=2] [KINDS="text random"] bash scripts/gpu_dec_ab.sh variant [variant ...]
set -o pipefail
O=${O:-gpurun_out/dab}; mkdir -p $O
for rep in $(seq 1 ${REPS:-2}); do
  for k in ${KINDS:-text random}; do
    for v in default "$@"; do
      L=$PWD/br-archive_amd/libbra_hip.so
      [ $v = default ] || L=$PWD/br-archive_amd/build/variants/$v/libbra_hip.so
      BRA_HIP_LIB=$L timeout -k 10 200 python -u scripts/decode_bench.py $k $((1 << 20)) 5 > $O/dec_${v}_${k}_$rep.json 2>> $O/dec.err
      rc=$?; [ $rc -eq 0 ] || { echo "decode $v $k rc $rc"; exit $rc; }
      echo "[$v $k $rep] $(cat $O/dec_${v}_${k}_$rep.json)"
    done
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/decode_bench.py text $((1 << 20)) 5 > $O/prof_dec.json 2> $O/prof.err
echo "prof rc $?"
if [ "${PMC:-0}" = 1 ]; then
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT -d $O/pmc_sq -o run --output-format csv -- python3 scripts/decode_bench.py text $((1 << 20)) 1 > $O/pmc_sq.log 2>&1
  echo "pmc sq rc $?"
fi
