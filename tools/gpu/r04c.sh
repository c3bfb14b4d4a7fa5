#!/bin/bash
# round 4 (c): the whole -m gpu suite on the committed kernels, A/B timings of the fused passes
# (round-3 build vs this tree vs variants), the Muon step in a hipGraph by CU count, the default bench
# and a kernel trace of it.  A crash / abort / time limit ends the script.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04c; mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 540 python -u -m pytest -m gpu -q --timeout 240 --timeout-method thread tests > $O/tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $O/tests.log; grep -E "^FAILED|^ERROR" $O/tests.log | head -20; fatal $rc tests
for v in r03 cur unrolled w4 fp8bp4; do
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
timeout -k 10 330 python3 bench.py > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3000 $O/bench.log; fatal $rc bench
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --urm-steps 0 --single-steps 0 --sweep '' > $O/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; fatal $rc trace
head -25 $O/trace/run_kernel_stats.csv
