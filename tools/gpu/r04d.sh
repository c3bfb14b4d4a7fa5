#!/bin/bash
# round 4 (d): the restored one-wave-per-SIMD backward with stored keep bits, the Muon counter reset
# (no memset node); the 2-rank test (one-CU Muon as the bisection when it fails); A/B timings; Muon
# phase clocks; the train-loop bench.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04d; mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
T="python -u -m pytest -m gpu -q --timeout 240 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_ppo_fused.py tests/test_gpu_train.py tests/test_gpu_rccl.py > $O/tests.log 2>&1
rc=$?; echo "fused/train/rccl tests rc=$rc"; tail -2 $O/tests.log; grep -E "^FAILED|^ERROR" $O/tests.log | head; fatal $rc tests
timeout -k 10 300 $T tests/test_gpu_dist.py > $O/dist.log 2>&1
rc=$?; echo "dist rc=$rc"; tail -2 $O/dist.log; grep -E "^E .*AssertionError|^E .*\(" $O/dist.log | head -5; fatal $rc dist
if [ $rc -ne 0 ]; then
  G2048_MUON_ONE_CU=1 timeout -k 10 300 $T tests/test_gpu_dist.py > $O/dist_onecu.log 2>&1
  rc=$?; echo "dist one-CU rc=$rc"; tail -2 $O/dist_onecu.log; fatal $rc dist1
fi
for v in r03 cur; do
  lib=tools/alt/libg2048_$v.so; [ $v = cur ] && lib=2048-ppo_amd/g2048/libg2048.so
  echo "== $v" >> $O/time.log
  timeout -k 10 120 env G2048_LIB=$lib python -u tools/time_fused.py 65536 >> $O/time.log 2>&1
  rc=$?; fatal $rc "time $v"
done
grep -v amdgpu.ids $O/time.log
for parts in 1 8 12; do
  echo "== parts $parts" >> $O/time_muon.log
  G2048_MUON_PARTS=$parts timeout -k 10 120 python -u tools/time_muon.py - 196 >> $O/time_muon.log 2>&1
  rc=$?; fatal $rc "muon $parts"
done
grep -v "amdgpu.ids\|Warning\|detach\|checksum" $O/time_muon.log
for parts in 1 8 12; do
  echo "== trace parts $parts" >> $O/trace_muon.log
  timeout -k 10 120 python -u tools/trace_muon.py tools/alt/libg2048_mtrace.so $parts >> $O/trace_muon.log 2>&1
  rc=$?; fatal $rc "trace $parts"
done
grep -v "amdgpu.ids" $O/trace_muon.log | head -60
timeout -k 10 300 python3 bench.py --cpu-seconds 0 --urm-steps 0 --single-steps 0 --sweep '' > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; fatal $rc bench
python3 -c "
import json
for l in open('$O/bench.log'):
    if l.startswith('{'):
        d=json.loads(l); tl=d.get('train_loop',{}); print('value',d['value'],'train_loop',tl.get('value'),tl.get('ms_per_iter'))
"
