#!/bin/bash
# round 4 (l): env_rollout_kernel with packed statistics, table maxima and pre-spawn kLine12 reads:
# env parity tests, the env bench line, trace + FETCH/WRITE/SQ passes of the rollout leg
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04l; mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread tests/test_gpu_env.py tests/test_gpu_train.py > $O/tests.log 2>&1
rc=$?; echo "env tests rc=$rc"; tail -2 $O/tests.log; grep -E "^FAILED|^ERROR" $O/tests.log | head -20; fatal $rc tests
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python3 bench.py --cpu-seconds 0 --urm-steps 0 --train-iters 0 --single-steps 0 --sweep '' > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; fatal $rc bench
grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value',d['value'],'ms',d['ms_per_step'],'avg_launch_us',d['roofline']['avg_launch_us'])"
TAG=r04l ARGS="--steps 20 --warmup 3 --cpu-seconds 0 --train-iters 0 --urm-steps 0 --single-steps 0 --sweep=" PMC_ARGS="--steps 4 --warmup 1 --cpu-seconds 0 --single-steps 0 --train-iters 0 --urm-steps 0 --sweep=" bash tools/profile.sh > $O/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; cat $O/prof.log | tail -8
python3 tools/summarize_profile.py gpurun_out/prof_r04l gpurun_out/r04l/summary > /dev/null 2>&1
python3 -c "
import json; d=json.load(open('gpurun_out/r04l/summary/pmc_env_rollout.json')); print({k:d[k] for k in ('valu_per_wave_step','lds_per_wave_step','salu_per_wave_step','lds_conflict_per_lds_inst','hbm_bytes_per_env_step')})"
