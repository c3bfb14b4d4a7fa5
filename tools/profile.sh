#!/bin/bash
# rocprofv3 passes for the bench command (GPU box): kernel trace + stats, then one PMC pass per
# TCC counter (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950).  No sys/hip tracing with PMC.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${TAG:-r01}
ARGS=${ARGS:---steps 20 --warmup 3 --cpu-seconds 0}
PMC_ARGS=${PMC_ARGS:---steps 5 --warmup 1 --cpu-seconds 0 --single-steps 64}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
find $OUT/trace -name "*kernel_trace.csv" -size +20M -delete  # keep gpurun_out under its copy-back cap
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $OUT/fetch -o run -- python3 bench.py $PMC_ARGS > $OUT/fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $OUT/write -o run -- python3 bench.py $PMC_ARGS > $OUT/write.log 2>&1
rc=$?; echo "write rc=$rc"; exit $rc
