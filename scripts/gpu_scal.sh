set -e
O=gpurun_out/scal; mkdir -p $O
for b in 268435456 134217728 67108864; do
timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --profile-all --steps 3 --warmup 1 --bytes-per-gpu $b --no-check > $O/b_$b.json 2> $O/b_$b.err
done
echo done > $O/done
