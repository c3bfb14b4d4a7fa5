set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/ptrain_r03f; mkdir -p $OUT
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 --single-steps 0 --train-iters 3 --train-warmup 1 --urm-steps 0 --sweep= > $OUT/bench.log 2>&1
echo "bench rc=$?"; tail -c 1200 $OUT/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 --single-steps 0 --train-iters 2 --train-warmup 1 --urm-steps 0 --sweep= > $OUT/trace.log 2>&1
echo "trace rc=$?"
find $OUT/trace -name "*kernel_trace.csv" -size +20M -delete
