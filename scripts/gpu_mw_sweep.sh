set -e
mkdir -p gpurun_out/mw
for mw in 5 6 8; do
  make -C br-archive_amd -B -j16 EXTRA=-DJOB_MIN_WAVES=$mw > gpurun_out/mw/build$mw.log 2>&1
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --profile-all --no-cpu-baseline --no-check --no-secondary > gpurun_out/mw/mw$mw.json 2> gpurun_out/mw/mw$mw.err
done
