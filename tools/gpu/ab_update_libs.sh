#!/bin/bash
# GameMLP update timing (tools/bench_update.py, fused path, graphed) of several library builds,
# alternating in fresh processes on one box: bash tools/gpu/ab_update_libs.sh <rounds> <lib.so>... ("cur" =
# the working build)
cd "${GRAFT_REPO_ROOT:-.}"
R=$1; shift
for r in $(seq $R); do
  for lib in "$@"; do
    if [ "$lib" = cur ]; then unset G2048_LIB; else export G2048_LIB=$lib; fi
    out=$(timeout -k 10 200 python3 tools/bench_update.py --which fused --samples 2097152 --iters 5 2>&1 | grep '^fused ')
    rc=$?; [ $rc -eq 0 ] || { echo "$lib rc=$rc"; exit 1; }
    echo "$lib $out"
  done
done
