#!/bin/bash
# round 4 (j): env record pointers per lane, column sums that price the gradient norm; tests, bench,
# training-loop kernel trace
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04j; mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 540 python -u -m pytest -m gpu -q --timeout 240 --timeout-method thread tests > $O/tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 $O/tests.log; grep -E "^FAILED|^ERROR" $O/tests.log | head -20; fatal $rc tests
timeout -k 10 300 python3 bench.py --cpu-seconds 0 --urm-steps 0 --single-steps 0 --sweep '' > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; fatal $rc bench
python3 -c "
import json
for l in open('$O/bench.log'):
    if l.startswith('{'):
        d=json.loads(l); tl=d.get('train_loop',{}); print('value',d['value'],'env_us',d['roofline'].get('avg_launch_us'),'train_loop',tl.get('value'),tl.get('ms_per_iter'))
"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --urm-steps 0 --single-steps 0 --sweep '' > $O/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; fatal $rc trace
head -16 $O/trace/run_kernel_stats.csv
