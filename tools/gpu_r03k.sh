# URM training GEMMs on g2048_urm_linear: URM GPU tests, fwd+bwd timing, URM-leg kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_urm.py -q -x --timeout 240 --timeout-method thread > gpurun_out/gpu_urm_r03k.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_urm_r03k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/time_urm_train.py 0.1 > gpurun_out/time_urm_r03k.log 2>&1
rc=$?; echo "time rc=$rc"; cat gpurun_out/time_urm_r03k.log; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/purm_r03k; mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 --single-steps 0 --train-iters 0 --urm-steps 16 --sweep= > $OUT/trace.log 2>&1
echo "trace rc=$?"
find $OUT/trace -name "*kernel_trace.csv" -size +20M -delete
grep -o '"train_iter": {"value": [0-9.e+]*, "unit": "env-steps/s", "ms_per_iter": [0-9.]*' $OUT/trace.log
