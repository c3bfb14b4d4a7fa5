#!/bin/bash
# round 4 (i): the whole -m gpu suite, the default bench, a kernel trace of the training loop
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04i; mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 540 python -u -m pytest -m gpu -q --timeout 240 --timeout-method thread tests > $O/tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 $O/tests.log; grep -E "^FAILED|^ERROR" $O/tests.log | head -20; fatal $rc tests
timeout -k 10 360 python3 bench.py > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; fatal $rc bench
python3 -c "
import json
for l in open('$O/bench.log'):
    if l.startswith('{'):
        d=json.loads(l); tl=d.get('train_loop',{}); print('value',d['value'],'train_loop',tl.get('value'),tl.get('ms_per_iter'),tl.get('phase_ms'))
"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --urm-steps 0 --single-steps 0 --sweep '' > $O/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; fatal $rc trace
head -22 $O/trace/run_kernel_stats.csv
