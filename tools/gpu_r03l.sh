# captured GameURM update: URM GPU tests, then the URM bench leg untraced
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_urm.py -q -x --timeout 240 --timeout-method thread > gpurun_out/gpu_urm_r03l.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_urm_r03l.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 --single-steps 0 --train-iters 0 --urm-steps 16 --sweep= > gpurun_out/urm_bench_r03l.log 2>&1
rc=$?; grep -o '"train_iter": {[^}]*' gpurun_out/urm_bench_r03l.log; exit $rc
