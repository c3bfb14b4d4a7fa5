#!/bin/bash
# A/B of the fused Muon/AdamW step (tools/time_muon.py, h 196, 13 parts) between the working build
# ("B") and 2048-ppo_amd/g2048/_ab/libg2048_a.so ("A"), alternating in fresh processes.
cd "${GRAFT_REPO_ROOT:-.}"
R=${1:-3}
for r in $(seq $R); do
  for v in A B; do
    lib=-; [ $v = A ] && lib=2048-ppo_amd/g2048/_ab/libg2048_a.so
    echo "== $v"; timeout -k 10 120 python3 tools/time_muon.py $lib 196 quick 2>&1 | grep -v amdgpu.ids | head -4 || exit 1
  done
done
