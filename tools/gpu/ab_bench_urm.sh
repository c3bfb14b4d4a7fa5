#!/bin/bash
# A/B of bench.py's GameURM leg between the working build and another library (swapped in place of
# 2048-ppo_amd/g2048/libg2048.so on the box's scratch copy, restored after each run):
#   bash tools/gpu/ab_bench_urm.sh <rounds> <lib.so>
cd "${GRAFT_REPO_ROOT:-.}"
R=$1; ALT=$2; LIB=2048-ppo_amd/g2048/libg2048.so
cp $LIB /tmp/libg2048_cur.so
for r in $(seq $R); do
  for v in cur alt; do
    if [ $v = alt ]; then cp $ALT $LIB; else cp /tmp/libg2048_cur.so $LIB; fi
    timeout -k 10 300 python3 bench.py --cpu-seconds 0 --train-iters 0 --urm-steps 16 --urm-iters 3 --single-steps 0 --sweep '' --steps 2 --warmup 1 > /tmp/b.log 2>&1
    rc=$?; cp /tmp/libg2048_cur.so $LIB; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -5 /tmp/b.log; exit 1; }
    python3 -c "
import json
for l in open('/tmp/b.log'):
    if l.startswith('{'):
        u=json.loads(l)['urm']; t=u['train_iter']; print('$v', round(u['forward_ms'],4), round(t['ms_per_iter'],2), t['phase_ms'])"
  done
done
