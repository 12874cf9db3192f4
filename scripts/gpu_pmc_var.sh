# one SQ instruction-count PMC pass per library variant ($VARIANTS; "base" = the in-tree library)
set -e
O=${O:-gpurun_out/pmcvar}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-check --no-secondary ${BENCH_ARGS:-}"
for v in ${VARIANTS:-base}; do
  lib=$PWD/br-archive_amd/libbra_hip.so; [ $v = base ] || lib=$PWD/br-archive_amd/build/variants/$v/libbra_hip.so
  BRA_HIP_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM -d $O/$v -o run --output-format csv -- $B > $O/$v.log 2>&1
done
