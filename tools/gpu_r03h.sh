set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ppo_fused.py -q -x --timeout 240 --timeout-method thread -k "backward or same_update" > gpurun_out/gpu_back_r03h.log 2>&1
rc=$?; echo "pytest-back rc=$rc"; tail -3 gpurun_out/gpu_back_r03h.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/time_back.py
