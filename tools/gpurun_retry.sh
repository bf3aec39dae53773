#!/bin/bash
# Re-submit a gpurun call only when the infrastructure reports a transient failure (nothing ran,
# nothing charged), waiting as long as gpurun's back-off asks. Any real result (pass, fail, crash,
# timeout) is returned as is.
# usage: tools/gpurun_retry.sh <timeout> '<command>'  (log: ${GPURUN_LOG:-/tmp/gpurun_last.log})
T=$1; shift
LOG=${GPURUN_LOG:-/tmp/gpurun_last.log}
for i in $(seq 1 ${GPURUN_TRIES:-12}); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient" "$LOG" || [ $rc -eq 3 ]; then
    w=$(grep -o 'retry in [0-9]*s' "$LOG" | grep -o '[0-9]*' | tail -1)
    w=${w:-45}
    echo "transient (attempt $i), retrying in $((w + 10))s" >&2; sleep $((w + 10)); continue
  fi
  tail -6 "$LOG"; exit $rc
done
tail -6 "$LOG"; exit 3
