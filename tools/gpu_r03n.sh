# URM: no-grad gate_up on the inference epilogue, 16-byte stores in the training epilogue
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_urm.py tests/test_gpu_ppo_fused.py -k "urm or muon" -q -x --timeout 240 --timeout-method thread > gpurun_out/gpu_urm_r03n.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_urm_r03n.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/time_urm_train.py 0.1 > gpurun_out/time_urm_r03n.log 2>&1; head -3 gpurun_out/time_urm_r03n.log
timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 --single-steps 0 --train-iters 0 --urm-steps 16 --sweep= > gpurun_out/urm_bench_r03n.log 2>&1
rc=$?; grep -o '"train_iter": {"value": [^,]*, "unit": "env-steps/s", "ms_per_iter": [0-9.]*' gpurun_out/urm_bench_r03n.log; exit $rc
