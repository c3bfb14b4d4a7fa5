#!/bin/bash
# round 4 (k): KL pass with the statistics folded in, device row offset + multi-step graphs;
# tests, bench, training-loop trace, GameURM training trace, SQ counters of the fused kernels
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04k; mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 540 python -u -m pytest -m gpu -q --timeout 240 --timeout-method thread tests > $O/tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 $O/tests.log; grep -E "^FAILED|^ERROR" $O/tests.log | head -20; fatal $rc tests
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python3 bench.py --cpu-seconds 0 --urm-steps 0 --single-steps 0 --sweep '' > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; fatal $rc bench
python3 -c "
import json
for l in open('$O/bench.log'):
    if l.startswith('{'):
        d=json.loads(l); tl=d.get('train_loop',{}); print('value',d['value'],'train_loop',tl.get('value'),tl.get('ms_per_iter'))
"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --urm-steps 0 --single-steps 0 --sweep '' > $O/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; fatal $rc trace
head -12 $O/trace/run_kernel_stats.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/urm -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --train-iters 0 --urm-steps 16 --urm-iters 1 --single-steps 0 --sweep '' > $O/urm.log 2>&1
rc=$?; echo "urm trace rc=$rc"; fatal $rc urm
head -16 $O/urm/run_kernel_stats.csv
TAG=r04k_fused bash tools/pmc_kernel.sh python3 tools/time_fused.py 65536 > $O/pmc.log 2>&1
echo "pmc rc=$?"; python3 tools/pmc_table.py gpurun_out/pmck_r04k_fused mlp_ 2>&1 | head -60
