#!/bin/bash
# round 4 (q): o_proj / down_proj fused with the residual RMSNorm in URM training (LinResRMSFn);
# torch-op census of one URM iteration; URM tests, bench leg, trace
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04q; mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest -m gpu -q --timeout 200 --timeout-method thread tests/test_gpu_urm.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; grep -E "^FAILED|^ERROR" $O/tests.log | head -20; fatal $rc tests
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python3 bench.py --cpu-seconds 0 --train-iters 0 --urm-steps 16 --urm-iters 3 --single-steps 0 --sweep '' > $O/bench_urm.log 2>&1
rc=$?; echo "bench rc=$rc"; fatal $rc bench
grep '^{' $O/bench_urm.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); u=d['urm']; print('urm fwd ms', u['forward_ms'], 'train ms/iter', u['train_iter']['ms_per_iter'], u['train_iter']['phase_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/urm -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --train-iters 0 --urm-steps 16 --urm-iters 1 --single-steps 0 --sweep '' > $O/urm_trace.log 2>&1
rc=$?; echo "urm trace rc=$rc"; fatal $rc urm
head -14 $O/urm/run_kernel_stats.csv
timeout -k 10 400 python3 tools/prof_urm_ops.py 65536 16 > $O/prof_ops.log 2>&1
echo "census rc=$?"; head -75 $O/prof_ops.log
