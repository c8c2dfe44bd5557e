#!/bin/bash
# Run one gpurun call, waiting for a free GPU slot: retried ONLY while gpurun reports that no slot / box is
# free (nothing ran, nothing charged); any other outcome -- success or a failure of the command -- ends it.
# usage: bash tools/gpurun_wait.sh TIMEOUT 'command'
T=$1; shift
for i in $(seq 1 20); do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1)
  rc=$?
  echo "$out" | tail -25
  if echo "$out" | grep -q "slot(s) on this pod are busy\|no box\|status=transient\|backing off"; then
    sleep 90
    continue
  fi
  exit $rc
done
exit 3
