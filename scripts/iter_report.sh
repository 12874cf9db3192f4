tail -n 3 gpurun_out/it/pytest.log; tail -n 2 gpurun_out/it/stress.log; python scripts/show_bench.py gpurun_out/it/bench.json | head -1; python scripts/trace_steps.py gpurun_out/it/tr/run_kernel_trace.csv | head -${1:-16}
if [ -f gpurun_out/it/bench_alt.json ]; then echo ALT:; python scripts/show_bench.py gpurun_out/it/bench_alt.json | head -1; fi
