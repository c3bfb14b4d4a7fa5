#!/bin/bash
# round 4 (e): Muon momentum race fix (multi-CU parts write their momentum rows after every part has
# read them), keep-bit test fix; timings with the keep bits.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04e; mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
T="python -u -m pytest -m gpu -q --timeout 240 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_ppo_fused.py -k "muon or keep_bits" > $O/tests.log 2>&1
rc=$?; echo "muon/keep tests rc=$rc"; tail -2 $O/tests.log; grep -E "^FAILED|^ERROR" $O/tests.log | head; fatal $rc tests
timeout -k 10 300 $T tests/test_gpu_dist.py > $O/dist.log 2>&1
rc=$?; echo "dist rc=$rc"; tail -2 $O/dist.log; fatal $rc dist
for v in r03 cur; do
  lib=tools/alt/libg2048_$v.so; [ $v = cur ] && lib=2048-ppo_amd/g2048/libg2048.so
  echo "== $v" >> $O/time.log
  timeout -k 10 120 env G2048_LIB=$lib python -u tools/time_fused.py 65536 >> $O/time.log 2>&1
  rc=$?; fatal $rc "time $v"
done
grep -v amdgpu.ids $O/time.log
for parts in 8 12; do
  echo "== parts $parts" >> $O/time_muon.log
  G2048_MUON_PARTS=$parts timeout -k 10 120 python -u tools/time_muon.py - 196 >> $O/time_muon.log 2>&1
  rc=$?; fatal $rc "muon $parts"
done
grep -v "amdgpu.ids\|Warning\|detach\|checksum" $O/time_muon.log
