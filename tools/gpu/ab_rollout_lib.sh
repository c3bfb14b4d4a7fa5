#!/bin/bash
# A/B of the rollout leg (tools/time_env_rollout.py) between the working build ("B") and
# 2048-ppo_amd/g2048/_ab/libg2048_a.so ("A"), alternating in fresh processes.
cd "${GRAFT_REPO_ROOT:-.}"
R=${1:-3}
for r in $(seq $R); do
  for v in A B; do
    if [ $v = A ]; then export G2048_LIB=2048-ppo_amd/g2048/_ab/libg2048_a.so; else unset G2048_LIB; fi
    echo "== $v"
    timeout -k 10 200 python3 tools/time_env_rollout.py 100 1024 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
