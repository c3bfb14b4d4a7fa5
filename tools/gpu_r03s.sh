# GameURM loop-start add + bf16 copy fused (AddCastFn): URM tests, fwd+bwd timing, URM bench leg
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r03s
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_urm.py -q -x --timeout 240 --timeout-method thread > gpurun_out/r03s/gpu_urm.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r03s/gpu_urm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/time_urm_train.py 0.1 > gpurun_out/r03s/time_urm.log 2>&1; head -3 gpurun_out/r03s/time_urm.log
timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 --single-steps 0 --train-iters 0 --urm-steps 16 --sweep= > gpurun_out/r03s/urm_bench.log 2>&1
rc=$?; grep -o '"train_iter": {"value": [^,]*, "unit": "env-steps/s", "ms_per_iter": [0-9.]*' gpurun_out/r03s/urm_bench.log; exit $rc
