set -e
O=gpurun_out/ph; mkdir -p $O
for k in text random sym16; do
BRA_HIP_LIB=$PWD/br-archive_amd/build/variants/phases/libbra_hip.so timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-check --no-secondary --kind $k $( [ $k = sym16 ] && echo --block-size 8388608 ) > $O/$k.json 2> $O/$k.err
done
