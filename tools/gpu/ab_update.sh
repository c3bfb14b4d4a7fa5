#!/bin/bash
# A/B of the GameMLP update (tools/bench_update.py, fused path, graphed) between the working build
# (2048-ppo_amd/g2048/libg2048.so, "B") and another build ("A": 2048-ppo_amd/g2048/_ab/libg2048_a.so),
# alternating A B A B ... in fresh processes on one box.  Usage: bash tools/gpu/ab_update.sh <rounds> [samples]
cd "${GRAFT_REPO_ROOT:-.}"
R=${1:-3}; S=${2:-2097152}
for r in $(seq $R); do
  for v in A B; do
    if [ $v = A ]; then export G2048_LIB=2048-ppo_amd/g2048/_ab/libg2048_a.so; else unset G2048_LIB; fi
    out=$(timeout -k 10 200 python3 tools/bench_update.py --which fused --samples $S --iters 5 2>&1 | grep '^fused ')
    rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; exit 1; }
    echo "$v $out"
  done
done
