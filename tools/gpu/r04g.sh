#!/bin/bash
# round 4 (g): one-launch weight gradients (mlp_wgrad.hip), Muon XCD placement + 13 parts +
# unrolled normalisation; fused tests, timings, Muon phase clocks.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04g; mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
T="python -u -m pytest -m gpu -q --timeout 240 --timeout-method thread"
timeout -k 10 200 $T tests/test_gpu_ppo_fused.py -k "mlp_wgrad or one_launch or muon" > $O/tests_new.log 2>&1
rc=$?; echo "new tests rc=$rc"; tail -2 $O/tests_new.log; grep -E "^FAILED|^ERROR" $O/tests_new.log | head; fatal $rc tests_new
timeout -k 10 400 $T tests/test_gpu_ppo_fused.py tests/test_gpu_train.py tests/test_gpu_dist.py tests/test_gpu_rccl.py > $O/tests.log 2>&1
rc=$?; echo "fused/train/dist tests rc=$rc"; tail -2 $O/tests.log; grep -E "^FAILED|^ERROR" $O/tests.log | head; fatal $rc tests
timeout -k 10 120 python -u tools/time_fused.py 65536 > $O/time.log 2>&1
rc=$?; fatal $rc time; grep -v amdgpu.ids $O/time.log
for parts in 8 12 13; do
  echo "== parts $parts" >> $O/time_muon.log
  G2048_MUON_PARTS=$parts timeout -k 10 120 python -u tools/time_muon.py - 196 >> $O/time_muon.log 2>&1
  rc=$?; fatal $rc "muon $parts"
done
grep -v "amdgpu.ids\|Warning\|detach\|checksum" $O/time_muon.log
timeout -k 10 120 python -u tools/trace_muon.py tools/alt/libg2048_mtrace.so 13 > $O/trace_muon.log 2>&1
rc=$?; fatal $rc trace; grep -v "amdgpu.ids" $O/trace_muon.log | head -8
