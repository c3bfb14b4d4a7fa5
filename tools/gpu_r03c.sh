set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ppo_fused.py tests/test_gpu_train.py tests/test_gpu_urm.py -q -x --timeout 240 --timeout-method thread -k "muon or optim" > gpurun_out/gpu_muon_r03c.log 2>&1
rc=$?; echo "pytest-muon rc=$rc"; tail -20 gpurun_out/gpu_muon_r03c.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/time_muon.py - 196 && G2048_MUON_GENERIC=1 timeout -k 10 120 python tools/time_muon.py - 196
