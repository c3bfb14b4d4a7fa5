set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -k "dist or config5 or fallbacks or urm_trainer_steps or wgrad or readme" > gpurun_out/gpu_new_r03a.log 2>&1
rc=$?; echo "pytest-new rc=$rc"; tail -25 gpurun_out/gpu_new_r03a.log; [ $rc -eq 0 ] || exit $rc
TAG=r03a bash tools/pmc_train.sh
