#!/bin/bash
# Development helper (this container, not the GPU box): run one gpurun call,
# retrying ONLY while the pool has no box for it (status=transient, nothing
# ran, nothing charged) — at most 10 tries, 2 minutes apart. A call that ran
# is never repeated, whatever its result.
# usage: tools/gpu_try.sh LOGFILE TIMEOUT 'command'
log=$1; t=$2; shift 2
for i in $(seq 1 10); do
  timeout $((t + 900)) /usr/local/graft/bin/gpurun --timeout "$t" -- "$@" > "$log" 2>&1
  rc=$?
  if grep -q 'status=transient' "$log" && ! grep -q 'status=ok\|status=fail' "$log"; then
    echo "try $i: no box ($(grep -o 'retry in [0-9]*s\|no free box\|stopped responding' "$log" | head -1)); waiting" >&2
    sleep 120
    continue
  fi
  exit $rc
done
exit 3
