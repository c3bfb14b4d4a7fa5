#!/bin/bash
# Rollout-leg timing (tools/time_env_rollout.py) of several library builds, alternating in fresh
# processes on one box: bash tools/gpu/ab_rollout_libs.sh <rounds> <lib.so>... ("cur" = the working build)
cd "${GRAFT_REPO_ROOT:-.}"
R=$1; shift
for r in $(seq $R); do
  for lib in "$@"; do
    if [ "$lib" = cur ]; then unset G2048_LIB; else export G2048_LIB=$lib; fi
    echo "== $lib"
    timeout -k 10 200 python3 tools/time_env_rollout.py 100 1024 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
