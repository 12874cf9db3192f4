#!/bin/bash
# round 4, call b: the intermittent chunk-stream encode mismatch with stage localisation (fixed
# prelude 2, the failing round of call a, then rotating); per-kernel profile of the local-MSD
# variant vs the default; iBWT walk grid sweep
set -o pipefail
O=gpurun_out/r4b; mkdir -p $O
ok() { [ $1 -le 1 ] || exit $1; }
timeout -k 10 300 python -u scripts/stress_chunks.py 25 2 > $O/stress_pre2.log 2>&1
rc=$?; echo "stress pre2 rc $rc"; grep -v "'ok', 'sym16_256KiB_x1024': 'ok'" $O/stress_pre2.log | tail -8; ok $rc
timeout -k 10 300 python -u scripts/stress_chunks.py 25 > $O/stress_rot.log 2>&1
rc=$?; echo "stress rot rc $rc"; grep -v "'ok', 'sym16_256KiB_x1024': 'ok'" $O/stress_rot.log | tail -8; ok $rc
timeout -k 10 120 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --profile-all > $O/bench_cur_prof.json 2> $O/bench_cur_prof.err
rc=$?; echo "bench cur rc $rc"; ok $rc
BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/local/libbra_hip.so timeout -k 10 120 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --profile-all > $O/bench_local_prof.json 2> $O/bench_local_prof.err
rc=$?; echo "bench local rc $rc"; ok $rc
for v in walk256 walk384 walk512 walk768; do
  BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/$v/libbra_hip.so timeout -k 10 120 python -u scripts/decode_bench.py --reps 5 >> $O/decode_ab.jsonl 2>> $O/decode_ab.err
  rc=$?; echo "decode $v rc $rc"; ok $rc
done
cat $O/decode_ab.jsonl
