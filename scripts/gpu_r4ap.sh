#!/bin/bash
# round-4 secondary lines: random and sym16 8 MiB bench lines, decode kernel stats
set -o pipefail
O=gpurun_out/r4ap; mkdir -p $O
timeout -k 10 300 python bench.py --kind random --no-cpu-baseline > $O/bench_random.json 2> $O/bench_random.err || exit $?
timeout -k 10 300 python bench.py --kind sym16 --block-size 8388608 --no-cpu-baseline > $O/bench_sym16_8MiB.json 2> $O/bench_sym16.err || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dprof -o run --output-format csv -- python3 scripts/decode_bench.py --reps 5 > $O/decode.json 2> $O/decode.err || exit $?
for f in $O/bench_random.json $O/bench_sym16_8MiB.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d.get('secondary',{}).get('decode_GBps'), d['reference_check'].get('digests',{}).get('bit_exact'))"; done
cat $O/decode.json
