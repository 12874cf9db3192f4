# BASELINE configs beyond the headline line (one bench.py JSON line each), 1 GPU.
set -e
O=gpurun_out/suite
mkdir -p $O
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --kind random --no-cpu-baseline > $O/random_1MiB.json 2> $O/random_1MiB.err
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --kind sym16 --block-size 8388608 --no-cpu-baseline > $O/sym16_8MiB.json 2> $O/sym16_8MiB.err
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --kind text --block-size 262144 --no-cpu-baseline > $O/text_256KiB.json 2> $O/text_256KiB.err
