set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo_fused.py -q -x --timeout 240 --timeout-method thread -k "backward or same_update" > gpurun_out/gpu_back_r03e.log 2>&1
rc=$?; echo "pytest-back rc=$rc"; tail -30 gpurun_out/gpu_back_r03e.log; exit $rc
