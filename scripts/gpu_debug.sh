mkdir -p gpurun_out/ktdbg
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2 3 4; do
  timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/ktdbg/smoke$i -o run --output-format csv -- python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ktdbg/smoke$i.log 2>&1
  rc=$?
  echo "run $i rc=$rc dchecks=$(grep -c dcheck gpurun_out/ktdbg/smoke$i.log)"; grep -o "job mode[^\[j]*\|n_tiles[^\[]*" gpurun_out/ktdbg/smoke$i.log | sort | uniq -c | head -8; rm -f gpurun_out/ktdbg/smoke$i.log
  if [ $rc -ge 124 ]; then break; fi
done
