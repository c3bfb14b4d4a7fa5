#!/bin/bash
# round 4 (m): hardware bf16 rounding in the URM kernels; env kernel spawn row/column re-read;
# URM + env parity tests, URM forward variants (no-SLP, NB=1, stage-once timing probe), URM bench leg
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04m; mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest -m gpu -q --timeout 200 --timeout-method thread tests/test_gpu_env.py tests/test_gpu_urm.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; grep -E "^FAILED|^ERROR" $O/tests.log | head -20; fatal $rc tests
[ $rc -ne 0 ] && exit 1
for v in "" tools/alt/libg2048_urm_noslp.so tools/alt/libg2048_urm_nb1.so tools/alt/libg2048_urm_once.so; do
  echo "== ${v:-in-tree}"
  G2048_LIB=$v timeout -k 10 120 python3 tools/time_urm.py 65536 64 10 2>&1 | tail -1; fatal $? time_urm
done
timeout -k 10 300 python3 bench.py --cpu-seconds 0 --train-iters 0 --urm-steps 16 --urm-iters 3 --single-steps 0 --sweep '' > $O/bench_urm.log 2>&1
rc=$?; echo "bench rc=$rc"; fatal $rc bench
grep '^{' $O/bench_urm.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); u=d['urm']; print('urm fwd ms', u['forward_ms'], 'train ms/iter', u['train_iter']['ms_per_iter'], u['train_iter']['phase_ms']); print('env value', d['value'])"
