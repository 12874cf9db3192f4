for f in gpurun_out/env/run*.json; do b=${f%.json}; echo "== $(cat $b.env)"; python scripts/show_bench.py $f | grep -E "${1:-value|jobs|scatter|hist|scan}"; done
