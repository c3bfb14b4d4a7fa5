#!/bin/bash
# A/B of the GameURM projection-kernel calls (tools/time_urm_train_linear.py) between the working
# build ("B") and 2048-ppo_amd/g2048/_ab/libg2048_a.so ("A"), alternating in fresh processes.
cd "${GRAFT_REPO_ROOT:-.}"
R=${1:-2}
for r in $(seq $R); do
  for v in A B; do
    if [ $v = A ]; then export G2048_LIB=2048-ppo_amd/g2048/_ab/libg2048_a.so; else unset G2048_LIB; fi
    echo "== $v"
    timeout -k 10 200 python3 tools/time_urm_train_linear.py 65536 || exit 1
  done
done
