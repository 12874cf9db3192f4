#!/bin/bash
# round 4, call y: bench A/B base / rowonly / rowal, then SQ counter passes on the base library
set -o pipefail
O=gpurun_out/r4y; mkdir -p $O
for rep in 1 2; do
  for v in base rowonly rowal; do
    L=$PWD/br-archive_amd/build/variants/$v/libbra_hip.so
    BRA_HIP_LIB=$L timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-check --profile-all > $O/bench_${v}_$rep.json 2>> $O/bench.err
    rc=$?; [ $rc -eq 0 ] || { echo "bench $v rc $rc"; exit $rc; }
    python3 scripts/show_bench.py $O/bench_${v}_$rep.json | python3 -c "
import sys; L=sys.stdin.read().splitlines(); print('$v', L[0][:60]); [print('  ', l) for l in L[1:] if any(k in l for k in ('jobs','scatter'))]"
  done
done
R=$GRAFT_REPO_ROOT
export BRA_HIP_LIB=$R/br-archive_amd/build/variants/base/libbra_hip.so
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_WAIT_INST_LDS" \
           "SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_WAVES" \
           "GRBM_GUI_ACTIVE SQ_INST_LEVEL_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d $R/$O/sq$i -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-check --no-secondary > $R/$O/sq$i.log 2>&1 || { echo "pass $i rc $?"; exit 1; }
done
echo done
