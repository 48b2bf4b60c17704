#!/bin/bash
# Host-side helper (never runs on the GPU box): submit one gpurun call, resubmitting it only while the pool has no
# free box (gpurun status=transient: nothing ran, nothing was charged).  Any call that reached a box - passed or
# failed - ends the loop; its output is in $OUT.
#   tools/gpu_retry.sh OUT TIMEOUT 'command' [max_tries]
OUT=$1; TO=$2; CMD=$3; N=${4:-12}
for i in $(seq "$N"); do
  timeout $((TO + 600)) /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$OUT" 2>&1
  rc=$?
  if ! grep -q "status=transient" "$OUT"; then exit $rc; fi
  sleep 180
done
exit 3
