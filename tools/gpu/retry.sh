#!/bin/bash
# retry a gpurun call while the pool reports a transient (no box / box lost while being prepared),
# sleeping as long as gpurun's back-off asks.  usage: tools/gpu/retry.sh TIMEOUT SCRIPT [tries]
t=$1; script=$2; tries=${3:-12}
for i in $(seq 1 $tries); do
  out=$(timeout $((t + 900)) /usr/local/graft/bin/gpurun --timeout $t -- bash $script 2>&1)
  echo "$out" | grep -v "every call sends the whole tree" | tail -60
  echo "$out" | grep -q "status=transient" || exit 0
  w=$(echo "$out" | grep -o "retry in [0-9]*s" | grep -o "[0-9]*" | tail -1)
  sleep $(( ${w:-90} + 5 ))
done
exit 3
