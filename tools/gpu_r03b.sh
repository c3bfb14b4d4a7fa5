set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ppo_fused.py -q -x --timeout 240 --timeout-method thread > gpurun_out/gpu_fused_r03b.log 2>&1
rc=$?; echo "pytest-fused rc=$rc"; tail -30 gpurun_out/gpu_fused_r03b.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/gpu_all_r03b.log 2>&1
rc=$?; echo "pytest-all rc=$rc"; tail -15 gpurun_out/gpu_all_r03b.log; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/ptrain_r03b; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 --single-steps 0 --train-iters 2 --train-warmup 1 --urm-steps 0 --sweep= > $OUT/trace.log 2>&1
echo "trace rc=$?"; tail -c 1500 $OUT/trace.log
