#!/bin/bash
# Run a command on the GPU box via gpurun; retry only when the infrastructure
# (not our command) failed: box not prepared / no slot (status transient, rc 3).
# Honours gpurun's "retry in Ns" back-off hint.
# Usage: tools/gpu.sh TIMEOUT 'command'
T=$1; shift
for attempt in $(seq 1 ${GPU_ATTEMPTS:-8}); do
  rm -f gpurun_out/.last_call.json
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > /tmp/gpurun_last.out 2>&1
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json'))['status'])" 2>/dev/null)
  if [ "$st" = "transient" ] || [ $rc -eq 3 ] || grep -q "backing off" /tmp/gpurun_last.out; then
    wait_s=$(grep -o "retry in [0-9]*s" /tmp/gpurun_last.out | grep -o "[0-9]*" | tail -1)
    wait_s=$(( ${wait_s:-30} + 10 ))
    echo "[gpu.sh] transient infrastructure failure (attempt $attempt), retrying in ${wait_s}s"
    sleep "$wait_s"; continue
  fi
  tail -3 /tmp/gpurun_last.out
  exit $rc
done
echo "[gpu.sh] giving up after repeated transient failures"; exit 3
