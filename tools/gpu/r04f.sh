#!/bin/bash
# round 4 (f): Muon normalisation by reciprocal + fma correction, pipelined exchange copy
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04f; mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
T="python -u -m pytest -m gpu -q --timeout 240 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_ppo_fused.py -k "muon" > $O/tests.log 2>&1
rc=$?; echo "muon tests rc=$rc"; tail -2 $O/tests.log; grep -E "^FAILED|^ERROR" $O/tests.log | head; fatal $rc tests
for parts in 8 12; do
  echo "== parts $parts" >> $O/time_muon.log
  G2048_MUON_PARTS=$parts timeout -k 10 120 python -u tools/time_muon.py - 196 >> $O/time_muon.log 2>&1
  rc=$?; fatal $rc "muon $parts"
done
grep -v "amdgpu.ids\|Warning\|detach\|checksum" $O/time_muon.log
for parts in 8 12; do
  echo "== trace parts $parts" >> $O/trace_muon.log
  timeout -k 10 120 python -u tools/trace_muon.py tools/alt/libg2048_mtrace.so $parts >> $O/trace_muon.log 2>&1
  rc=$?; fatal $rc "trace $parts"
done
grep -v "amdgpu.ids" $O/trace_muon.log | head -12
