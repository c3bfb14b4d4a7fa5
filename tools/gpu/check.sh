#!/bin/bash
# GPU box recipes behind the committed profiles (one gpurun call each; every GPU step has its own
# time limit, the chain stops at the first failure or fault):
#   TAG=r04x bash tools/gpu/check.sh env    env parity tests, the env bench line, trace + FETCH /
#                                           WRITE / SQ passes of the rollout leg (-> pmc_env_rollout.json)
#   TAG=r04x bash tools/gpu/check.sh fused  GameMLP update: fused tests, train-loop trace, SQ passes of
#                                           tools/time_fused.py
#   TAG=r04x bash tools/gpu/check.sh urm    GameURM: tests, bench leg, kernel trace, torch-op census,
#                                           SQ passes of the one-launch forward
#   TAG=r04x bash tools/gpu/check.sh full   every GPU test, smoke, the default bench line
#   TAG=r06a bash tools/gpu/check.sh dist   stale-memory detector of the update, the 2-rank and RCCL tests
#   TAG=r06b bash tools/gpu/check.sh urmhbm the GameURM update's HBM bytes (-> urm_update_hbm.json)
#   TAG=r05a bash tools/gpu/check.sh muon   Muon: its tests, the MUON_TRACE build (make trace) at 13 and 8
#                                           parts (phase clocks + bound checks), HIP-event timing
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${TAG:-check}
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
run_tests() {  # run_tests <log> <timeout> <pytest args...>
  local log=$1 lim=$2; shift 2
  timeout -k 10 $lim python -u -m pytest -m gpu -q --timeout 240 --timeout-method thread "$@" > $log 2>&1
  local rc=$?; echo "tests rc=$rc"; tail -2 $log; grep -E "^FAILED|^ERROR" $log | head -20; fatal $rc tests
  [ $rc -eq 0 ] || exit 1
}
case "$1" in
env)
  run_tests $O/tests.log 300 tests/test_gpu_env.py tests/test_gpu_train.py
  timeout -k 10 300 python3 bench.py --cpu-seconds 0 --urm-steps 0 --train-iters 0 --single-steps 0 --sweep '' > $O/bench_env.log 2>&1
  rc=$?; echo "bench rc=$rc"; fatal $rc bench
  TAG=$TAG ARGS="--steps 20 --warmup 3 --cpu-seconds 0 --train-iters 0 --urm-steps 0 --single-steps 0 --sweep=" \
    PMC_ARGS="--steps 4 --warmup 1 --cpu-seconds 0 --single-steps 0 --train-iters 0 --urm-steps 0 --sweep=" \
    bash tools/profile.sh > $O/prof.log 2>&1
  rc=$?; echo "prof rc=$rc"; tail -6 $O/prof.log; fatal $rc prof
  # the PMC passes ran bench.py at its default --chunk (1024 steps per launch since round 6)
  PMC_CHUNK=1024 python3 tools/summarize_profile.py gpurun_out/prof_$TAG $O/summary > /dev/null 2>&1
  python3 -c "import json; d=json.load(open('$O/summary/pmc_env_rollout.json')); print({k: d[k] for k in ('valu_per_wave_step', 'lds_per_wave_step', 'hbm_bytes_per_env_step')})"
  ;;
fused)
  run_tests $O/tests.log 400 tests/test_gpu_ppo_fused.py
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --urm-steps 0 --single-steps 0 --sweep '' > $O/trace.log 2>&1
  rc=$?; echo "trace rc=$rc"; fatal $rc trace
  TAG=${TAG}_fused bash tools/pmc_kernel.sh python3 tools/time_fused.py 65536 > $O/pmc.log 2>&1
  echo "pmc rc=$?"; python3 tools/pmc_table.py gpurun_out/pmck_${TAG}_fused mlp_ 2>&1 | head -60
  ;;
urm)
  run_tests $O/tests.log 400 tests/test_gpu_urm.py
  timeout -k 10 300 python3 bench.py --cpu-seconds 0 --train-iters 0 --urm-steps 16 --urm-iters 3 --single-steps 0 --sweep '' > $O/bench_urm.log 2>&1
  rc=$?; echo "bench rc=$rc"; fatal $rc bench
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/urm -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --train-iters 0 --urm-steps 16 --urm-iters 1 --single-steps 0 --sweep '' > $O/urm_trace.log 2>&1
  rc=$?; echo "urm trace rc=$rc"; fatal $rc urm
  timeout -k 10 400 python3 tools/prof_urm_ops.py 65536 16 > $O/prof_ops.log 2>&1
  echo "census rc=$?"
  TAG=${TAG}_urmfwd bash tools/pmc_kernel.sh python3 tools/time_urm.py 65536 64 3 > $O/pmc.log 2>&1
  echo "pmc rc=$?"; python3 tools/pmc_table.py gpurun_out/pmck_${TAG}_urmfwd urm_forward 2>&1 | head -30
  ;;
muon)
  make -C 2048-ppo_amd/csrc trace > $O/make_trace.log 2>&1 || { echo "make trace failed"; tail -5 $O/make_trace.log; exit 1; }
  run_tests $O/tests.log 300 tests/test_gpu_ppo_fused.py -k "muon or Muon"
  for p in 13 8; do
    timeout -k 10 120 python3 tools/trace_muon.py tools/alt/libg2048_mtrace.so $p > $O/trace_muon_$p.log 2>&1
    rc=$?; echo "trace parts=$p rc=$rc"; grep -c MUON_CHECK $O/trace_muon_$p.log; tail -3 $O/trace_muon_$p.log; fatal $rc trace
    [ $rc -eq 0 ] || exit 1
  done
  timeout -k 10 120 python3 tools/time_muon.py > $O/time_muon.log 2>&1
  echo "time rc=$?"; head -6 $O/time_muon.log
  ;;
dist)
  run_tests $O/stale.log 400 tests/test_gpu_stale_reads.py
  run_tests $O/dist.log 400 tests/test_gpu_dist.py tests/test_gpu_rccl.py
  ;;
urmhbm)
  # the GameURM update's FETCH / WRITE bytes between tools/urm_update_pmc.py's markers
  P=gpurun_out/purmhbm_$TAG; mkdir -p $P
  for c in FETCH_SIZE WRITE_SIZE; do
    n=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
    timeout -s KILL 300 rocprofv3 --pmc $c -T --output-format csv -d $P/$n -o run -- python3 tools/urm_update_pmc.py > $P/$n.log 2>&1
    rc=$?; echo "$c rc=$rc"; tail -1 $P/$n.log; fatal $rc $c; [ $rc -eq 0 ] || exit 1
  done
  python3 tools/urm_update_hbm.py $P $O/urm_update_hbm.json
  ;;
full)
  run_tests $O/tests.log 700 tests
  timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; fatal $rc smoke
  timeout -k 10 600 python3 bench.py > $O/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; fatal $rc bench
  ;;
*) echo "usage: TAG=... bash tools/gpu/check.sh env|fused|urm|full"; exit 2 ;;
esac
