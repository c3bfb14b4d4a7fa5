# round 4: fused train / KL passes at 2 waves per SIMD -- parity tests + kernel timings
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04a
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ppo_fused.py -m gpu -x -v --timeout 200 --timeout-method thread -k "fused_train_pass or fused_kl_pass or fused_backward or graphed_update or split_graph or same_update" > gpurun_out/r04a/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r04a/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/time_fused.py > gpurun_out/r04a/time_fused.log 2>&1
rc=$?; echo "time rc=$rc"; cat gpurun_out/r04a/time_fused.log; exit $rc
