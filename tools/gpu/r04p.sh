#!/bin/bash
# round 4 (p): torch-op census of one GameURM training iteration (eager)
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04p; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 tools/prof_urm_ops.py 65536 16 > $O/prof_ops.log 2>&1
echo "rc=$?"; head -80 $O/prof_ops.log
