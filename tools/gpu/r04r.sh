#!/bin/bash
# round 4 (r): checkpoint -- full GPU test suite, default bench line, smoke
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04r; mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 700 python -u -m pytest -m gpu -q --timeout 240 --timeout-method thread tests > $O/tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 $O/tests.log; grep -E "^FAILED|^ERROR" $O/tests.log | head -20; fatal $rc tests
[ $rc -ne 0 ] && exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log; fatal $rc smoke
timeout -k 10 600 python3 bench.py > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; fatal $rc bench
grep '^{' $O/bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); tl=d.get('train_loop',{}); u=d.get('urm',{})
print('value',d['value'],'frac',d['roofline']['frac'],'avg_us',d['roofline']['avg_launch_us'])
print('train_loop',tl.get('value'),tl.get('ms_per_iter'))
print('urm fwd',u.get('forward_ms'),'train',u.get('train_iter',{}).get('ms_per_iter'))
print('cpu',d.get('cpu_baseline',{}).get('value'))"
