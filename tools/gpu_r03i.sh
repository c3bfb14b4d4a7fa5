set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ppo_fused.py -q -x --timeout 240 --timeout-method thread -k "wgrad_pair or backward or same_update" > gpurun_out/gpu_pair_r03i.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_pair_r03i.log; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/ptrain_r03i; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 --single-steps 0 --train-iters 2 --train-warmup 1 --urm-steps 0 --sweep= > $OUT/trace.log 2>&1
echo "trace rc=$?"
find $OUT/trace -name "*kernel_trace.csv" -size +20M -delete
grep -o '"train_loop": {"value": [0-9.e+]*, "unit": "env-steps/s", "ms_per_iter": [0-9.]*' $OUT/trace.log
