#!/bin/bash
# Run one command on the GPU box via gpurun.  Re-requests the box ONLY when gpurun reports
# status=transient (the box failed before the command started: nothing ran, nothing charged);
# a command that ran — whatever its exit code — is never re-run.
# usage: tools/gpu.sh <timeout-seconds> '<command>'
T=$1; shift
for attempt in 1 2 3 4; do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1)
  rc=$?
  if echo "$out" | grep -q "status=transient"; then
    echo "[gpu.sh] box not ready (attempt $attempt), waiting" >&2
    sleep 75
    continue
  fi
  echo "$out"
  exit $rc
done
echo "$out"
exit 3
