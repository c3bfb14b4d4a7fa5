# URM golden at the default config on the GPU; env-only kernel trace of the headline (roofline check)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r03q
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_urm.py tests/test_gpu_ppo_fused.py -k "golden" -v -s --timeout 240 --timeout-method thread > gpurun_out/r03q/gpu_urm_golden.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|passed|failed|restatement" gpurun_out/r03q/gpu_urm_golden.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/r03q/trace -o run -- python3 bench.py --cpu-seconds 0 --train-iters 0 --urm-steps 0 --single-steps 0 --sweep= > gpurun_out/r03q/trace.log 2>&1
echo "trace rc=$?"
find gpurun_out/r03q/trace -name "*kernel_trace.csv" -size +20M -delete
grep env_rollout gpurun_out/r03q/trace/run_kernel_stats.csv
