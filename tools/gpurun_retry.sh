#!/bin/bash
# Re-submit a gpurun call only when the infrastructure reports a transient failure (nothing ran,
# nothing charged). Any real result (pass, fail, crash, timeout) is returned as is.
# usage: tools/gpurun_retry.sh <timeout> '<command>'  (log: /tmp/gpurun_last.log)
T=$1; shift
for i in 1 2 3 4 5; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > /tmp/gpurun_last.log 2>&1
  rc=$?
  if grep -q "status=transient" /tmp/gpurun_last.log || [ $rc -eq 3 ]; then
    echo "transient (attempt $i), retrying" >&2; sleep 30; continue
  fi
  tail -6 /tmp/gpurun_last.log; exit $rc
done
tail -6 /tmp/gpurun_last.log; exit 3
