#!/bin/bash
# Runs a command on the GPU box via gpurun; retries infrastructure-transient
# failures (box lost before the command ran) a few times.  Usage:
#   tools/gpu.sh TIMEOUT 'command'
t=$1; shift
for i in 1 2 3 4 5; do
  out=$(/usr/local/graft/bin/gpurun --timeout "$t" -- "$@" 2>&1); rc=$?
  if echo "$out" | grep -q "status=transient\|no box\|slot free"; then
    echo "[gpu.sh] transient (attempt $i), retrying" >&2; sleep 30; continue
  fi
  echo "$out" | tail -25
  exit $rc
done
echo "$out" | tail -5
exit 3
