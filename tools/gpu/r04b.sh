# round 4: A/B timings of the fused passes (round-3 build vs this tree) over minibatch sizes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04b
export TMPDIR=/tmp
timeout -k 10 120 env G2048_LIB=tools/alt/libg2048_r03.so python -u tools/time_fused.py 512,4096,16384,65536,262144 > gpurun_out/r04b/time_r03.log 2>&1
rc=$?; cat gpurun_out/r04b/time_r03.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/time_fused.py 512,4096,16384,65536,262144 > gpurun_out/r04b/time_new.log 2>&1
rc=$?; cat gpurun_out/r04b/time_new.log; exit $rc
