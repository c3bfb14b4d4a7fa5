#!/bin/bash
# retry a gpurun call while the pool reports a transient (no box / box lost while being prepared)
# usage: tools/gpu/retry.sh TIMEOUT SCRIPT [tries]
t=$1; script=$2; tries=${3:-8}
for i in $(seq 1 $tries); do
  out=$(timeout $((t + 900)) /usr/local/graft/bin/gpurun --timeout $t -- bash $script 2>&1)
  echo "$out" | grep -v "every call sends the whole tree" | tail -60
  echo "$out" | grep -q "status=transient" || exit 0
  sleep 75
done
