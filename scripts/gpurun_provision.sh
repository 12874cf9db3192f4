# Run one gpurun call, re-submitting it ONLY while the GPU pool fails to provision a box (status
# "transient" with the command never started: "run 0.0s" / "run Nones").  Any call that started
# on a box -- passed, failed or was cut off -- is final and is not re-run.
# usage: bash scripts/gpurun_provision.sh <log> <timeout_s> '<command>'
log=$1; to=$2; cmd=$3
for i in $(seq 1 12); do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $log 2>&1
  if grep -q "status=transient" $log && grep -Eq "run (0\.0s|Nones)" $log; then
    w=$(grep -oE "retry in [0-9]+s" $log | grep -oE "[0-9]+" | head -1)
    sleep $(( ${w:-60} + 30 ))
    continue
  fi
  break
done
