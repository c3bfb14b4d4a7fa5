# env_rollout_kernel with the kLine12 table: env GPU tests, default bench line, kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_env.py tests/test_gpu_policy_rollout.py -q -x --timeout 240 --timeout-method thread > gpurun_out/gpu_env_r03m.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_env_r03m.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --cpu-seconds 0 --train-iters 0 --urm-steps 0 > gpurun_out/bench_env_r03m.log 2>&1
rc=$?; tail -c 700 gpurun_out/bench_env_r03m.log; echo; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/penv_r03m; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 20 --warmup 2 --cpu-seconds 0 --single-steps 0 --train-iters 0 --urm-steps 0 --sweep= > $OUT/trace.log 2>&1
echo "trace rc=$?"
grep env_rollout $OUT/trace/run_kernel_stats.csv
